"""Config-5 extension parity (DCN-v2 matrix cross stack, multi-feature assembly, the ranker
model): HIP vs the oracle's restatement (no reference model exists for it: SURVEY §0 item 4)."""
import numpy as np
import pytest

from conftest import assert_close, oracle, pkg

pytestmark = pytest.mark.gpu


def _t(x, dev, dtype=None):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    elif t.dtype == torch.float64:
        t = t.float()
    return t.to(dev)


def _n(t):
    return t.detach().double().cpu().numpy()


@pytest.mark.parametrize("prec", [0, 6, 9])
@pytest.mark.parametrize("B,d,L", [(257, 64, 3), (100, 132, 1), (64, 3344, 2), (5, 16, 0)])
def test_cross_matrix_fwd_bwd(cuda, B, d, L, prec):
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(B + d + L)
    x0 = (rng.standard_normal((B, d)) * 0.5).astype(np.float32).astype(np.float64)
    W = (rng.standard_normal((L, d, d)) / np.sqrt(d)).astype(np.float32).astype(np.float64)
    b = (rng.standard_normal((L, d)) * 0.1).astype(np.float32).astype(np.float64)
    g = rng.standard_normal((B, d)).astype(np.float32).astype(np.float64)
    extra = rng.standard_normal((B, d)).astype(np.float32).astype(np.float64)
    xL, xs = O.cross_matrix_forward(x0, W, b)
    gx0, gW, gb = O.cross_matrix_backward(x0, xs, W, b, g)
    tx0, tW, tb = _t(x0, cuda), _t(W.reshape(max(L, 0), d, d), cuda), _t(b, cuda)
    XS, US = F.dcn_cross_mat_fwd(tx0, tW, tb, precision=prec)
    if L > 0:
        assert_close(_n(XS[L - 1]), xL, 1e-4, "x_L")
    GX0, GW, GB = F.dcn_cross_mat_bwd(tx0, XS, US, tW, _t(g, cuda), _t(extra, cuda), precision=prec)
    assert_close(_n(GX0), gx0 + extra, 1e-4, "g_x0", floor=0.0)
    if L > 0:
        assert_close(_n(GW), gW, 1e-4, "g_W", floor=0.0)
        assert_close(_n(GB), gb, 1e-4, "g_b", floor=0.0)


def test_multi_embedding_gather_bitexact(cuda):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(0)
    Fn, E, nd, B = 5, 32, 13, 300
    tables = [rng.standard_normal((50 + 10 * f, E)).astype(np.float32) for f in range(Fn)]
    ids = np.stack([rng.integers(0, 50 + 10 * f, B) for f in range(Fn)]).astype(np.int64)
    ids[2, 7] = 10 ** 6                                      # out of range -> zeros + counted
    dense = rng.standard_normal((B, nd)).astype(np.float32)
    ld = 176                                                 # 5*32 + 13 = 173 -> padded
    tt = [_t(t, cuda) for t in tables]
    ptrs = torch.tensor([t.data_ptr() for t in tt], dtype=torch.int64, device=cuda)
    nrows = torch.tensor([t.shape[0] for t in tables], dtype=torch.int64, device=cuda)
    bad = torch.zeros((1,), dtype=torch.int32, device=cuda)
    x0 = F.multi_embedding_gather(ptrs, nrows, E, _t(ids, cuda), _t(dense, cuda), ld, bad).cpu().numpy()
    ref = np.zeros((B, ld), np.float32)
    for f in range(Fn):
        ok = ids[f] < tables[f].shape[0]
        ref[ok, f * E:(f + 1) * E] = tables[f][ids[f][ok]]
    ref[:, Fn * E:Fn * E + nd] = dense
    assert np.array_equal(x0, ref)
    assert int(bad.item()) == 1


def test_sparse_adagrad_strided_rows_equal_contiguous(cuda):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(1)
    V, D, n = 40, 32, 500
    G = rng.standard_normal((n, 3 * D)).astype(np.float32)
    ids = rng.integers(0, V, n).astype(np.int64)
    outs = []
    for strided in (False, True):
        T = _t(np.ones((V, D), np.float32), cuda)
        A = torch.full((V, D), 0.1, device=cuda)
        it = torch.zeros((), dtype=torch.int64, device=cuda)
        g = _t(G, cuda)[:, D:2 * D]
        F.sparse_adagrad(T, A, _t(ids, cuda), g if strided else g.contiguous(), it, 0.1)
        outs.append(T.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])


def test_dcn2_ranker_loss_and_grads(cuda):
    import torch
    models = pkg("models")
    O = oracle()
    vocab = [40, 25, 60]
    E, nd, B, L = 32, 5, 200, 2
    deep = [64, 32]
    m = models.DCNv2Ranker(vocab, embedding_dim=E, num_dense=nd, cross_layers=L, deep_layers=deep, device=cuda)
    d = m.d
    assert d == 112 and m.d_raw == 101
    rng = np.random.default_rng(3)
    # non-zero padding weights must stay inert: perturb them
    with torch.no_grad():
        m.cross_W[:, m.d_raw:, :] = 0.3
        m.cross_b[:, m.d_raw:] = 0.2
    P = {k: v.detach().double().cpu().numpy() for k, v in m.state_dict().items()}
    ids = np.stack([rng.integers(0, v + 1, B) for v in vocab]).astype(np.int64)
    dense = rng.standard_normal((B, nd)).astype(np.float32)
    y = (rng.random(B) < 0.3).astype(np.float32)
    loss = m.compute_loss(_t(ids, cuda), _t(dense, cuda), _t(y, cuda))
    loss.backward()
    ref = O.dcn2_ranker_loss_and_grads(P, len(vocab), E, d, deep, ids, dense.astype(np.float64), y.astype(np.float64))
    assert abs(float(loss) - ref["loss"]) <= 1e-4
    named = dict(m.named_parameters())
    for k, g in ref["grads"].items():
        if isinstance(g, tuple):
            f = int(k.split(".")[1])
            gi, gr = m.tables[f].sink.gathered()
            assert np.array_equal(gi.cpu().numpy(), g[0])
            assert_close(_n(gr), g[1], 1e-4, k, floor=0.0)
        else:
            assert_close(_n(named[k].grad).reshape(g.shape), g, 1e-4, k, floor=0.0)
    # padded rows/cols of W receive no gradient
    gW = named["cross_W"].grad
    assert float(gW[:, m.d_raw:, :].abs().max()) == 0.0 and float(gW[:, :, m.d_raw:].abs().max()) == 0.0


@pytest.mark.parametrize("B", [1000, 257])
def test_dcn2_trunk_node_matches_two_nodes(cuda, B, monkeypatch):
    """The DCN-v2 trunk as one node (cross stack + deep tower on the plane-pair GEMM, the tower's
    dL/dx0 folded into the cross backward) against the two-node form (DCNCrossMatFn +
    MLPFn on the split-at-staging GEMM): same products, other fp32 association — loss and every
    gradient within 1e-5 of the largest entry."""
    import torch
    models = pkg("models")
    vocab = [300, 70, 1000, 45, 12]
    rng = np.random.default_rng(B)
    ids = np.stack([rng.integers(0, v + 1, B) for v in vocab]).astype(np.int64)
    dense = rng.standard_normal((B, 13)).astype(np.float32)
    y = (rng.random(B) < 0.3).astype(np.float32)
    res = []
    for trunk in (False, True):
        monkeypatch.setattr(models, "DCN2_TRUNK", trunk)
        m = models.DCNv2Ranker(vocab, embedding_dim=64, num_dense=13, cross_layers=3, deep_layers=[256, 128, 64],
                               device=cuda, precision=6, seed=5)
        loss = m.compute_loss(_t(ids, cuda), _t(dense, cuda), _t(y, cuda))
        loss.backward()
        torch.cuda.synchronize()
        grads = {k: _n(p.grad) for k, p in m.named_parameters() if p.grad is not None}
        grads.update({f"table{f}": _n(t.sink.gathered()[1]) for f, t in enumerate(m.tables)})
        res.append((float(loss), grads))
    assert abs(res[0][0] - res[1][0]) <= 1e-6 * max(1.0, abs(res[0][0]))
    assert res[0][1].keys() == res[1][1].keys()
    for k in res[0][1]:
        a, b = res[0][1][k], res[1][1][k]
        assert np.abs(a - b).max() <= 1e-5 * max(np.abs(a).max(), 1e-30), k


@pytest.mark.parametrize("graphed", [False, True])
def test_multi_table_sparse_update_bitwise_equal(cuda, graphed, monkeypatch):
    """From SPARSE_MULTI_MIN_TABLES tables on, the sparse Adagrad updates of all tables run as one
    launch sequence (rs_sparse_adagrad_multi_f32, optim.Adagrad.step): bitwise the same training as
    one update per table, eager and under hipGraph replay. Each table is looked up twice per step,
    so every sink holds two slices (fresh torch.cat results)."""
    import torch
    models, optim, graphs = pkg("models"), pkg("optim"), pkg("graphs")
    vocab = [30, 45, 20, 60, 25]
    B = 256

    def make_batch(seed):
        rng = np.random.default_rng(seed)
        ids = np.stack([rng.integers(0, v + 1, B) for v in vocab]).astype(np.int64)
        dense = rng.standard_normal((B, 7)).astype(np.float32)
        y = (rng.random(B) < 0.4).astype(np.float32)
        return ({"user_id": _t(ids, cuda), "dense": _t(dense, cuda)}, {"y": _t(y, cuda)})

    finals = []
    for min_tables in (10 ** 9, 2):
        monkeypatch.setattr(optim, "SPARSE_MULTI_MIN_TABLES", min_tables)
        m = models.DCNv2Ranker(vocab, embedding_dim=32, num_dense=7, cross_layers=2, deep_layers=[64, 32],
                               device=cuda, precision=6, seed=3)
        opt = optim.Adagrad(m.dense_parameters(), m.embedding_modules(), 0.05, clipnorm=1.0)

        def step(batch):
            opt.zero_grad()
            ids, dense, y = batch[0]["user_id"], batch[0]["dense"], batch[1]["y"]
            loss = m.compute_loss(ids, dense, y) + m.compute_loss(ids.flip(1), dense, y)
            loss.backward()
            opt.step()
            return loss.detach()

        runner = graphs.GraphedTrainStep(step, make_batch(0)) if graphed else step
        losses = [float(runner(make_batch(i))) for i in range(4)]
        torch.cuda.synchronize()
        assert all(len(t.sink.slices) == 2 for t in m.tables) or graphed
        finals.append(({k: v.clone() for k, v in m.state_dict().items()}, losses))
    assert finals[0][1] == finals[1][1]
    for k in finals[0][0]:
        assert torch.equal(finals[0][0][k], finals[1][0][k]), k


@pytest.mark.parametrize("prec", [6])
@pytest.mark.parametrize("B,d,L", [(257, 64, 3), (100, 132, 1), (600, 3344, 2), (5, 16, 1), (1030, 520, 4),
                                   (5120, 3344, 1),   # 280 tiles: the last partial round split over K
                                   (4096, 3344, 4)])
def test_cross_matrix_planes_path(cuda, B, d, L, prec):
    """The plane-image path (xgemm images, two cross products per 16x16x32 MFMA) of the DCN-v2
    stack against the float64 oracle at the fp32 bar, and against the split-at-staging path of the
    same precision (same products, other order of the fp32 additions: a few ulps)."""
    import torch
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(B * 3 + d + L)
    x0 = (rng.standard_normal((B, d)) * 0.5).astype(np.float32)
    W = (rng.standard_normal((L, d, d)) / np.sqrt(d)).astype(np.float32)
    b = (rng.standard_normal((L, d)) * 0.1).astype(np.float32)
    g = rng.standard_normal((B, d)).astype(np.float32)
    extra = rng.standard_normal((B, d)).astype(np.float32)
    tx0, tW, tb, tg, te = (_t(v, cuda) for v in (x0, W, b, g, extra))
    XS, US = F.dcn_cross_mat_fwd(tx0, tW, tb, precision=prec)
    XSp, USp, ximg = F.dcn_cross_mat_fwd_planes(tx0, tW, tb, precision=prec)
    GX0, GW, GB = F.dcn_cross_mat_bwd(tx0, XS, US, tW, tg, te, precision=prec)
    GX0p, GWp, GBp = F.dcn_cross_mat_bwd_planes(tx0, XSp, USp, tW, ximg, tg, te, precision=prec)
    torch.cuda.synchronize()
    for a, b_, name in ((XS, XSp, "xs"), (US, USp, "us"), (GX0, GX0p, "g_x0"), (GW, GWp, "g_W"), (GB, GBp, "g_b")):
        scale = max(float(a.abs().max()), 1e-30)
        assert float((a - b_).abs().max()) <= 1e-5 * scale, name
    x64 = x0.astype(np.float64)
    xL, xs = O.cross_matrix_forward(x64, W.astype(np.float64), b.astype(np.float64))
    gx0, gW, gb = O.cross_matrix_backward(x64, xs, W.astype(np.float64), b.astype(np.float64), g.astype(np.float64))
    assert_close(_n(XSp[L - 1]), xL, 1e-4, "x_L")
    assert_close(_n(GX0p), gx0 + extra, 1e-4, "g_x0", floor=0.0)
    assert_close(_n(GWp), gW, 1e-4, "g_W", floor=0.0)
    assert_close(_n(GBp), gb, 1e-4, "g_b", floor=0.0)
