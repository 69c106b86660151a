"""The data-parallel step's sparse work without sorts (round 6): the local deduplication over the
step's id plan (rs_sparse_dedupe_planned_f32) against the sorting deduplication, and the stable order
of the exchanged (rank-ordered, per-rank unique ascending) ids by binary-search merge
(rs_merge_runs_order_i64) against numpy's stable argsort, with the update that takes it bitwise equal
to the update that sorts (MirroredStrategy's rule, src/trainer.py:45-48,148,163)."""
import numpy as np
import pytest

from conftest import pkg

pytestmark = pytest.mark.gpu


def _zipf(rng, n, vocab, a=1.05):
    r = rng.zipf(a, size=n * 2)
    r = r[r <= vocab][:n]
    while r.size < n:
        e = rng.zipf(a, size=n)
        r = np.concatenate([r, e[e <= vocab]])[:n]
    return ((r.astype(np.int64) * (2654435761 % vocab or 1)) % vocab) + 1


@pytest.mark.parametrize("B,urows,crows,D", [(7, 10, 12, 128), (5000, 300, 70000, 64), (65536, 10_000_001, 1_000_001, 128)])
def test_planned_dedupe_bitwise_equal_to_sorting_dedupe(cuda, B, urows, crows, D):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(B + D)
    uid = _zipf(rng, B, urows - 1)
    iid = _zipf(rng, B, crows - 1)
    if B > 4:
        uid[0], uid[3], iid[1] = -5, urows, crows + 2          # out-of-range ids: dropped
    tu, ti = (torch.from_numpy(x).to(cuda) for x in (uid, iid))
    plan = F.inbatch_unique_ids_pair(tu, ti, urows, crows, order=True, dids=True)
    for side, ids, rows in ((0, tu, urows), (1, ti, crows)):
        g = torch.randn((B, D), device=cuda)
        a = F.sparse_dedupe(ids, g, rows)
        pl = plan[side]
        b = F.sparse_dedupe(ids, g, rows, plan=(pl[5], pl[7], pl[6], pl[3][0:1]))
        torch.cuda.synchronize()
        n = int(a[2])
        assert n == int(b[2]), side
        want = np.unique(ids.cpu().numpy()[(ids.cpu().numpy() >= 0) & (ids.cpu().numpy() < rows)])
        assert n == want.size, side
        assert int(pl[4][4 + side]) == n, side        # the plan's early count = the dedupe's (info[4 + side])
        assert np.array_equal(a[0][:n].cpu().numpy(), want), side
        assert torch.equal(a[0][:n], b[0][:n]), side
        assert torch.equal(a[1][:n], b[1][:n]), side
        assert torch.equal(a[3], b[3]), side


@pytest.mark.parametrize("ranks,B,rows", [(1, 3000, 500), (2, 20000, 100_000), (8, 65536, 10_000_001)])
def test_merge_runs_order_is_the_stable_sort_and_update_bitwise(cuda, ranks, B, rows):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(ranks * 7 + B)
    runs = [np.unique(_zipf(rng, B, rows - 1)) for _ in range(ranks)]
    ids = np.concatenate(runs)
    offs = np.concatenate([[0], np.cumsum([r.size for r in runs])])
    tids = torch.from_numpy(ids).to(cuda)
    order = F.merge_runs_order(tids, offs.tolist())
    torch.cuda.synchronize()
    assert np.array_equal(order.cpu().numpy(), np.argsort(ids, kind="stable"))
    # the exchanged update: merge order vs the update's own sort, bitwise (two tables of one width)
    n = ids.size
    g = [torch.randn((n, 128), device=cuda) * 1e-2, torch.randn((n, 128), device=cuda) * 1e-2]
    ssq = [(x.double() ** 2).sum().float().reshape(()) for x in g]
    out = []
    for ordered in (False, True):
        tabs = [torch.randn((rows, 128), device=cuda, generator=torch.Generator(cuda).manual_seed(3)) for _ in range(2)]
        accs = [torch.full_like(t, 0.1) for t in tabs]
        it = torch.zeros((), dtype=torch.int64, device=cuda)
        F.sparse_adagrad_multi(tabs, accs, [tids, tids], g, it, 0.05, 0.96, 1000, 1.0, 1e-7, sumsq=ssq,
                               increment=True, orders=[order, order] if ordered else None)
        torch.cuda.synchronize()
        out.append((tabs, accs))
    for j in range(2):
        assert torch.equal(out[0][0][j], out[1][0][j]), j
        assert torch.equal(out[0][1][j], out[1][1][j]), j
