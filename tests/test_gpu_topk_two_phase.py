"""The bound-first top-K scan (topk.hip topk_impl: 2048-row blocks in a fixed permuted order, cut
into geometric ranges, each range scanned against the k-th score of the exact list of all earlier
ranges, then selected) used for many queries over large shards (Q > 64, N >= 2^20; the C4 shape).
Reference: src/trainer.py:204-212 (np.dot + argpartition), app/recommendation_service.py:71-72
(IndexFlatIP.search); order contract (-score, index), SURVEY A.8.

On dyadic-grid data every score is exact, so the two-phase result must equal the oracle bit for bit,
ties included, and equal the single-pass list scan (RS_TOPK_LIST_SCAN). A query whose candidates
overflow their slots (mass ties at the bound) must fall back to the list scan and still be exact."""
import numpy as np
import pytest

from conftest import oracle, pkg

pytestmark = pytest.mark.gpu

N_TP = (1 << 20) + 4099      # just past the two-phase minimum, not a multiple of any tile


def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _run(F, q, it, k, prec, two_phase=True):
    S, I = F.topk_ip(q, it, k, precision=prec, list_scan=not two_phase)
    return S.cpu().numpy().astype(np.float64), I.cpu().numpy()


@pytest.fixture(scope="module")
def dyadic(cuda):
    rng = np.random.default_rng(31)
    D = 128
    q = rng.integers(-16, 17, (96, D)).astype(np.float32) / 16.0
    it = rng.integers(-16, 17, (N_TP, D)).astype(np.float32) / 16.0
    # ties across range boundaries: copies of good rows in the first range and in later ones
    for j in range(0, 96, 5):
        it[[7 + j, N_TP // 2 + j, N_TP - 1 - j]] = q[j]
    sc, idx = oracle().topk_ip_chunked(q, it, 100, 4)
    return dict(q=_t(q, cuda), it=_t(it, cuda), sc=sc, idx=idx)


@pytest.mark.parametrize("prec", [6, 9, 0])
@pytest.mark.parametrize("two_phase", [True, False])
def test_two_phase_dyadic_bitexact(dyadic, prec, two_phase):
    F = pkg("functional")
    S, I = _run(F, dyadic["q"], dyadic["it"], 100, prec, two_phase)
    assert np.array_equal(I, dyadic["idx"])
    assert np.array_equal(S, dyadic["sc"])


def test_two_phase_equals_list_scan_gaussian(cuda):
    """Non-dyadic data: both paths score every (query, item) with the same split MFMA sums, so
    the lists are bitwise equal (not only equal up to rounding)."""
    F = pkg("functional")
    rng = np.random.default_rng(5)
    q = _t(rng.standard_normal((300, 128)).astype(np.float32), cuda)
    it = _t(rng.standard_normal((N_TP, 128)).astype(np.float32), cuda)
    for k in (1, 37, 128):
        S2, I2 = _run(F, q, it, k, 6)
        S1, I1 = _run(F, q, it, k, 6, two_phase=False)
        assert np.array_equal(I2, I1), k
        assert np.array_equal(S2, S1), k


def test_two_phase_overflow_falls_back(cuda):
    """Every item scores the same (zero rows): every item reaches every bound, the candidate slots
    overflow, and the call reruns as the list scan: indices 0..k-1 by the index order."""
    F = pkg("functional")
    q = _t(np.ones((80, 128), np.float32), cuda)
    it = _t(np.zeros((N_TP, 128), np.float32), cuda)
    S, I = _run(F, q, it, 50, 6)
    assert (S == 0).all()
    assert (I == np.arange(50)[None, :]).all()


def test_two_phase_adversarial_order(cuda):
    """Items sorted by ascending score for every query (in table order the early rows hold the
    worst items; the permuted block order samples the whole table in every range): exact, and
    bitwise the list scan's lists."""
    F = pkg("functional")
    rng = np.random.default_rng(11)
    D = 128
    lv = np.sort(rng.integers(0, 1024, N_TP)).astype(np.float32)
    it = np.zeros((N_TP, D), np.float32)
    it[:, 0] = lv / 64.0
    it[:, 1:] = rng.integers(-1, 2, (N_TP, D - 1)).astype(np.float32) / 64.0
    q = np.zeros((72, D), np.float32)
    q[:, 0] = 1.0
    q[:, 1:] = rng.integers(-2, 3, (72, D - 1)).astype(np.float32) / 64.0
    sc, idx = oracle().topk_ip_chunked(q, it, 64, 6)
    S, I = _run(F, _t(q, cuda), _t(it, cuda), 64, 6)
    assert np.array_equal(I, idx)
    assert np.array_equal(S, sc)
    S1, I1 = _run(F, _t(q, cuda), _t(it, cuda), 64, 6, two_phase=False)
    assert np.array_equal(I1, I) and np.array_equal(S1, S)


def test_two_phase_norm_ordered_table(cuda):
    """Row norms rising down the table by powers of two (dyadic, so scores stay exact), the order
    that made every contiguous range beat its bound: exact against the oracle, bitwise the list
    scan, over a row count that is no multiple of the 2048-row block (a partial last block)."""
    F = pkg("functional")
    rng = np.random.default_rng(12)
    D, N = 128, N_TP
    it = rng.integers(-8, 9, (N, D)).astype(np.float32) / 16.0
    it *= (2.0 ** np.floor(np.arange(N) * 6 / N)).astype(np.float32)[:, None]
    q = rng.integers(-8, 9, (100, D)).astype(np.float32) / 16.0
    sc, idx = oracle().topk_ip_chunked(q, it, 100, 4)
    S, I = _run(F, _t(q, cuda), _t(it, cuda), 100, 6)
    assert np.array_equal(I, idx)
    assert np.array_equal(S, sc)
    S1, I1 = _run(F, _t(q, cuda), _t(it, cuda), 100, 6, two_phase=False)
    assert np.array_equal(I1, I) and np.array_equal(S1, S)
