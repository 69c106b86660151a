"""Per-kernel parity: HIP (via the C-ABI) vs the CPU oracle, on seeded inputs.

Bars (north_star): integer/index work bit-exact; fp32 logits/losses within 1e-4 (scaled as in
conftest.assert_close); top-K indices bit-exact after the (-score, index) order on dyadic-grid
data where every fp32 dot product is exact.
"""
import numpy as np
import pytest

from conftest import assert_close, oracle, pkg, score_tiles, stack_gates

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
    return t.detach().double().cpu().numpy() if t.dtype.is_floating_point else t.detach().cpu().numpy()


# ---------------------------------------------------------------------------------------------
# a2: embedding gather (bit-exact)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("V,D,n", [(1, 4, 1), (100, 32, 257), (5000, 128, 4099), (777, 64, 0), (3000, 64, 70001),
                                   (20000, 128, 300007), (50, 36, 999)])
def test_gather_bitexact(cuda, V, D, n):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(V + D + n)
    T = rng.standard_normal((V, D)).astype(np.float32)
    ids = rng.integers(0, V, size=n).astype(np.int64)
    out = F.embedding_gather(_t(T, cuda), _t(ids, cuda))
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), T[ids])


@pytest.mark.parametrize("D", [4, 32, 128])
def test_gather_bad_ids_zero_rows_and_count(cuda, D):
    import torch
    F = pkg("functional")
    T = np.arange(10 * D, dtype=np.float32).reshape(10, D)
    ids = np.array([0, -1, 9, 10, 3] * 20, dtype=np.int64)
    bad = torch.zeros((1,), dtype=torch.int32, device=cuda)
    out = F.embedding_gather(_t(T, cuda), _t(ids, cuda), bad).cpu().numpy()
    assert int(bad.item()) == 40
    good = np.isin(np.arange(100) % 5, [0, 2, 4])
    assert np.array_equal(out[good], T[ids[good]])
    assert not out[~good].any()


@pytest.mark.parametrize("D,sizes", [(128, [(10_000, 65536), (3000, 65536)]), (32, [(100, 1), (5000, 0), (70, 4099)]),
                                     (64, [(7, 300007)]), (36, [(50, 999), (60, 17)]),
                                     (128, [(40 + j, 100 * j + 1) for j in range(8)])])
def test_gather_tables_bitexact(cuda, D, sizes):
    """The one-launch lookup of several tables (the user + item Embeddings of a step) is the
    per-table row copy, bit for bit, including empty id lists and the fallback widths."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(D + len(sizes))
    Ts = [rng.standard_normal((V, D)).astype(np.float32) for V, _ in sizes]
    ids = [rng.integers(0, V, size=n).astype(np.int64) for V, n in sizes]
    outs = F.embedding_gather_tables([_t(T, cuda) for T in Ts], [_t(i, cuda) for i in ids])
    torch.cuda.synchronize()
    for o, T, i in zip(outs, Ts, ids):
        assert o.shape == (len(i), D)
        assert np.array_equal(o.cpu().numpy(), T[i])


# ---------------------------------------------------------------------------------------------
# a3/a8: GEMM
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(1, 4, 4), (130, 64, 128), (257, 256, 64), (64, 32, 36), (1000, 128, 256)])
def test_gemm_layouts(cuda, ta, tb, M, N, K):
    F = pkg("functional")
    N_ = pkg("_native")
    valid = (not ta or M % 4 == 0) and (tb or N % 4 == 0) and (K % 4 == 0 or (ta and not tb))
    if not valid:  # the C-ABI rejects layouts its float4 staging cannot move
        with pytest.raises(N_.NativeError):
            F.gemm(_t(np.zeros((K, M) if ta else (M, K), np.float32), cuda),
                   _t(np.zeros((N, K) if tb else (K, N), np.float32), cuda), trans_a=bool(ta), trans_b=bool(tb))
        return
    rng = np.random.default_rng(M * 7 + N * 3 + K + ta * 2 + tb)
    A = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
    Bm = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
    ref = (A.T if ta else A).astype(np.float64) @ (Bm.T if tb else Bm).astype(np.float64)
    out = F.gemm(_t(A, cuda), _t(Bm, cuda), trans_a=bool(ta), trans_b=bool(tb))
    assert_close(_n(out), ref, 1e-5, f"gemm ta={ta} tb={tb}", floor=0.0)


@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(4, 4, 4), (130, 64, 128), (257, 256, 64), (64, 32, 36), (1000, 128, 256),
                                   (300, 200, 1000)])
def test_gemm_split_precision(cuda, prec, ta, tb, M, N, K):
    """Split-operand GEMM (exact bf16 splits on the bf16 MFMA): within the f32 GEMM's error budget
    of the float64 product, every layout and ragged edge."""
    F = pkg("functional")
    valid = (not ta or M % 4 == 0) and (tb or N % 4 == 0) and (K % 4 == 0 or (ta and not tb))
    if not valid:
        return
    rng = np.random.default_rng(M * 5 + N * 3 + K + ta * 2 + tb + prec)
    A = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
    Bm = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
    ref = (A.T if ta else A).astype(np.float64) @ (Bm.T if tb else Bm).astype(np.float64)
    tA, tB = _t(A, cuda), _t(Bm, cuda)
    out = _n(F.gemm(tA, tB, trans_a=bool(ta), trans_b=bool(tb), precision=prec))
    out32 = _n(F.gemm(tA, tB, trans_a=bool(ta), trans_b=bool(tb), precision=0))
    assert_close(out, ref, 1e-5, f"gemm x{prec} ta={ta} tb={tb}", floor=0.0)
    e_split, e_f32 = np.abs(out - ref).max(), np.abs(out32 - ref).max()
    assert e_split <= 4.0 * e_f32 + 1e-6, (e_split, e_f32)


@pytest.mark.parametrize("prec", [6, 9])
def test_gemm_split_precision_exact_on_dyadic_and_epilogues(cuda, prec):
    """On dyadic operands every product and sum is exact: the split GEMM equals the f32 GEMM bit
    for bit, through the bias / ReLU / mask / beta epilogue and the split-K path."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(prec)
    M, N, K = 300, 128, 96
    A = rng.integers(-8, 9, (M, K)) / 8.0
    W = rng.integers(-8, 9, (K, N)) / 16.0
    b = rng.integers(-8, 9, N) / 4.0
    mask = rng.standard_normal((M, N))
    C0 = rng.integers(-8, 9, (M, N)) / 2.0
    tA, tW, tb, tm = _t(A, cuda), _t(W, cuda), _t(b, cuda), _t(mask, cuda)
    outs = []
    for pr in (0, prec):
        Ct = _t(C0, cuda)
        F.gemm(tA, tW, bias=tb, relu=True, mask=tm, out=Ct, beta=0.5, precision=pr)
        outs.append(Ct)
    assert torch.equal(outs[0], outs[1])
    X = _t(rng.integers(-8, 9, (2048, 64)) / 8.0, cuda)
    G = _t(rng.integers(-8, 9, (2048, 96)) / 8.0, cuda)
    s0 = F.gemm_splitk(X, G, trans_a=True, precision=0)
    s1 = F.gemm_splitk(X, G, trans_a=True, precision=prec)
    assert torch.equal(s0, s1)


def test_gemm_epilogue(cuda):
    F = pkg("functional")
    rng = np.random.default_rng(5)
    M, N, K = 300, 128, 96
    A = rng.standard_normal((M, K)).astype(np.float32)
    W = rng.standard_normal((K, N)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    mask = rng.standard_normal((M, N)).astype(np.float32)
    C0 = rng.standard_normal((M, N)).astype(np.float32)
    z = A.astype(np.float64) @ W + b
    out = F.gemm(_t(A, cuda), _t(W, cuda), bias=_t(b, cuda), relu=True)
    assert_close(_n(out), np.maximum(z, 0), 1e-5, "bias+relu", floor=0.0)
    Ct = _t(C0, cuda)
    F.gemm(_t(A, cuda), _t(W, cuda), bias=_t(b, cuda), mask=_t(mask, cuda), out=Ct, beta=0.5)
    assert_close(_n(Ct), z * (mask > 0) + 0.5 * C0, 1e-5, "mask+beta", floor=0.0)


@pytest.mark.parametrize("M,N,K", [(128, 256, 4096), (64, 128, 1000), (256, 64, 33), (4, 4, 0), (4, 12, 2000),
                                   (3344, 260, 512)])
def test_gemm_splitk_weight_grad(cuda, M, N, K):
    """Split-K with an addend (float4 slab reduction; lda / ldb are multiples of 4 by contract);
    the 3344-row output (>= 256 tiles) takes at least 2 K slices on 128 x 256 tiles."""
    F = pkg("functional")
    rng = np.random.default_rng(M + N + K)
    X = rng.standard_normal((K, M)).astype(np.float32)
    G = rng.standard_normal((K, N)).astype(np.float32)
    W = rng.standard_normal((M, N)).astype(np.float32)
    out = F.gemm_splitk(_t(X, cuda), _t(G, cuda), trans_a=True, addend=_t(W, cuda), addend_scale=2e-4)
    ref = X.T.astype(np.float64) @ G + 2e-4 * W
    assert_close(_n(out), ref, 1e-5, "splitk", floor=1.0)


@pytest.mark.parametrize("M,N", [(1000, 96), (1, 8), (17, 3), (4096, 256), (65536, 64), (300, 3344), (999, 260)])
def test_relu_bwd_colsum(cuda, M, N):
    """ReLU-backward mask (bitwise) and ordered column sums; N % 4 == 0 takes the float4 pass."""
    F = pkg("functional")
    rng = np.random.default_rng(11 + M + N)
    dy = rng.standard_normal((M, N)).astype(np.float32)
    y = rng.standard_normal((M, N)).astype(np.float32)
    g, cs = F.relu_bwd_colsum(_t(dy, cuda), _t(y, cuda))
    assert np.array_equal(g.cpu().numpy(), dy * (y > 0))
    assert_close(_n(cs), (dy * (y > 0)).astype(np.float64).sum(0), 1e-5, "colsum", floor=1.0)
    _, cs2 = F.relu_bwd_colsum(_t(dy, cuda))             # colsum only (bias grad of a linear layer)
    assert_close(_n(cs2), dy.astype(np.float64).sum(0), 1e-5, "colsum-only", floor=1.0)
    g2, cs3 = F.relu_bwd_colsum(_t(dy, cuda), _t(y, cuda))
    assert np.array_equal(_n(cs3), _n(cs)) and np.array_equal(_n(g2), _n(g))   # deterministic


# ---------------------------------------------------------------------------------------------
# a5/a7: DCN vector cross
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("B,D,L", [(1, 16, 1), (257, 64, 3), (1000, 128, 3), (65, 32, 5)])
def test_dcn_cross_fwd_bwd(cuda, B, D, L):
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(B + D + L)
    u = rng.standard_normal((B, D)) * 0.3
    v = rng.standard_normal((B, D)) * 0.3
    w = rng.uniform(-0.15, 0.15, (L, 2 * D))
    b = rng.standard_normal((L, 2 * D)) * 0.1
    gxl = rng.standard_normal((B, 2 * D))
    gx0e = rng.standard_normal((B, 2 * D))
    x0 = np.concatenate([u, v], 1)
    xL, xs, s = O.cross_forward(x0, w, b)
    gx0, gw, gb = O.cross_backward(x0, xs, s, w, gxl)
    tw, tb = _t(w, cuda), _t(b, cuda)
    X0, XL, S = F.dcn_cross_fwd(_t(u, cuda), _t(v, cuda), tw, tb)
    assert np.array_equal(_n(X0), x0.astype(np.float32).astype(np.float64))
    assert_close(_n(XL), xL, 1e-5, "xL")
    assert_close(_n(S)[:, :L], s, 1e-5, "s")
    gu, gv, GW, GB = F.dcn_cross_bwd(X0, S, tw, tb, _t(gxl, cuda), _t(gx0e, cuda))
    assert_close(np.concatenate([_n(gu), _n(gv)], 1), gx0 + gx0e, 1e-5, "g_x0")
    assert_close(_n(GW), gw, 1e-5, "g_w", floor=0.0)
    assert_close(_n(GB), gb, 1e-5, "g_b", floor=0.0)


# ---------------------------------------------------------------------------------------------
# a9/a11: heads + ranking losses
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("B", [1, 300, 4096])
def test_heads_and_ranking_losses(cuda, B, mode):
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(B + mode)
    dx, dh = 256, 128
    xl = rng.standard_normal((B, dx)) * 0.2
    h = np.abs(rng.standard_normal((B, dh))) * 0.2
    wr, wc = rng.standard_normal((dx + dh, 1)) * 0.05, rng.standard_normal((dx + dh, 1)) * 0.05
    br, bc = np.array([0.3]), np.array([-0.1])
    y = rng.integers(1, 6, B).astype(np.float64)
    yi = (y >= 4).astype(np.float64)
    cw = {0: 0.8, 1: 1.3}
    z = np.concatenate([xl, h], 1)
    r = z @ wr + br
    p = O.sigmoid(z @ wc + bc)
    lr_, lc_, dr, dp = O.ranking_losses(r, p, y, yi, cw, mode)
    R, Pp = F.heads_fwd(_t(xl, cuda), _t(h, cuda), _t(wr, cuda), _t(br, cuda), _t(wc, cuda), _t(bc, cuda))
    assert_close(_n(R), r, 1e-5, "rating")
    assert_close(_n(Pp), p, 1e-5, "ctr")
    loss, ur, uc = F.ranking_losses(R, Pp, _t(y, cuda), _t(yi, cuda), cw, mode)
    assert_close(_n(loss)[0], lr_, 1e-4, "mse")
    assert_close(_n(loss)[1], lc_, 1e-4, "bce")
    # backward with upstream weights 0.2 / 2.0 on the two losses
    import torch
    gsr = torch.tensor(0.2, device=cuda)
    gsc = torch.tensor(2.0, device=cuda)
    gxl, gh, gwr, gbr, gwc, gbc = F.heads_bwd(_t(xl, cuda), _t(h, cuda), _t(wr, cuda), _t(wc, cuda), Pp,
                                              unit_r=ur, unit_c=uc, gs_rat=gsr, gs_ctr=gsc)
    grat = 0.2 * dr
    gt = 2.0 * dp * p[:, 0] * (1 - p[:, 0])
    gz = grat[:, None] * wr[:, 0] + gt[:, None] * wc[:, 0]
    assert_close(np.concatenate([_n(gxl), _n(gh)], 1), gz, 1e-4, "g_z", floor=0.0)
    assert_close(_n(gwr)[:, 0], z.T @ grat, 1e-4, "g_wr", floor=0.0)
    assert_close(_n(gwc)[:, 0], z.T @ gt, 1e-4, "g_wc", floor=0.0)
    assert_close(_n(gbr), [grat.sum()], 1e-4, "g_br")
    assert_close(_n(gbc), [gt.sum()], 1e-4, "g_bc")


# ---------------------------------------------------------------------------------------------
# a10: in-batch softmax (retrieval) fwd + bwd
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("B,D", [(1, 32), (7, 64), (33, 128), (100, 32), (1000, 128), (4096, 64), (4100, 128)])
def test_inbatch_softmax(cuda, B, D):
    import torch
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(B * 3 + D)
    U = rng.standard_normal((B, D)) * 0.4
    C = rng.standard_normal((B, D)) * 0.4
    U32, C32 = U.astype(np.float32).astype(np.float64), C.astype(np.float32).astype(np.float64)
    row, tot, lse = O.retrieval_loss(U32, C32)
    dU, dC = O.retrieval_grads(U32, C32, lse)
    T, ROW, LSE, DU, T64 = F.inbatch_softmax_fwd(_t(U, cuda), _t(C, cuda))
    assert_close(_n(ROW), row, 1e-4, "row loss")
    assert_close(_n(LSE), lse, 1e-4, "lse")
    assert abs(float(T64.item()) - tot) <= 1e-4 * max(1.0, abs(tot)), (float(T64.item()), tot)
    assert abs(float(T.item()) - tot) <= 1e-4 * max(1.0, abs(tot))
    assert_close(_n(DU), dU, 1e-4, "dU (unit)")
    g = torch.tensor(0.75, device=cuda)
    DUs, DC = F.inbatch_softmax_bwd(_t(U, cuda), _t(C, cuda), LSE, gscale=g, dU_unit=DU)
    assert_close(_n(DUs), 0.75 * dU, 1e-4, "dU")
    assert_close(_n(DC), 0.75 * dC, 1e-4, "dC")


@pytest.mark.parametrize("B,D", [(1, 32), (33, 128), (100, 64), (1000, 128), (4100, 128), (8191, 32)])
def test_inbatch_stored_scores_bitwise_equal_to_recompute(cuda, B, D):
    """The score-storing pair (forward keeps U C^T, backward reads it) gives bit-identical
    outputs to the recomputing pair, and both match the oracle."""
    import torch
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(B + 7 * D)
    U = rng.standard_normal((B, D)) * 0.4
    C = rng.standard_normal((B, D)) * 0.4
    tU, tC = _t(U, cuda), _t(C, cuda)
    S = F.inbatch_scores_buffer(B, cuda)
    a = F.inbatch_softmax_fwd(tU, tC)
    b = F.inbatch_softmax_fwd(tU, tC, scores=S)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    g = torch.tensor(1.25, device=cuda)
    da = F.inbatch_softmax_bwd(tU, tC, a[2], gscale=g, dU_unit=a[3])
    db = F.inbatch_softmax_bwd(tU, tC, b[2], gscale=g, dU_unit=b[3], scores=S)
    assert torch.equal(da[0], db[0]) and torch.equal(da[1], db[1])
    U32, C32 = U.astype(np.float32).astype(np.float64), C.astype(np.float32).astype(np.float64)
    _, _, lse = O.retrieval_loss(U32, C32)
    _, dC = O.retrieval_grads(U32, C32, lse)
    assert_close(_n(db[1]), 1.25 * dC, 1e-4, "dC (stored)")


@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("B", [1, 33, 1000, 4100, 8191])
def test_inbatch_split_precision_matches_oracle_at_fp32_level(cuda, B, prec):
    """Split-operand kernels (fp32 operands as exact three-term bf16 splits on the bf16 MFMA):
    within the north-star tolerance of the oracle, and no further from the float64 truth than
    the f32-MFMA kernels are (the error budget of an fp32 GEMM)."""
    import torch
    F = pkg("functional")
    O = oracle()
    D = 128
    rng = np.random.default_rng(B + 11 * prec)
    U = rng.standard_normal((B, D)) * 0.4
    C = rng.standard_normal((B, D)) * 0.4
    tU, tC = _t(U, cuda), _t(C, cuda)
    U32, C32 = U.astype(np.float32).astype(np.float64), C.astype(np.float32).astype(np.float64)
    row, tot, lse = O.retrieval_loss(U32, C32)
    dU, dC = O.retrieval_grads(U32, C32, lse)
    g = torch.tensor(1.25, device=cuda)
    res = {}
    for pr in (0, prec):
        S = F.inbatch_scores_buffer(B, cuda)
        T, ROW, LSE, DU, T64 = F.inbatch_softmax_fwd(tU, tC, scores=S, precision=pr)
        DUs, DC = F.inbatch_softmax_bwd(tU, tC, LSE, gscale=g, dU_unit=DU, scores=S, precision=pr)
        res[pr] = (_n(ROW), _n(LSE), _n(DU), _n(DC), float(T64.item()))
    ROW, LSE, DU, DC, T64 = res[prec]
    assert_close(ROW, row, 1e-4, "row loss")
    assert_close(LSE, lse, 1e-4, "lse")
    assert_close(DU, dU, 1e-4, "dU (unit)")
    assert_close(DC, 1.25 * dC, 1e-4, "dC")
    assert abs(T64 - tot) <= 1e-4 * max(1.0, abs(tot))
    for j, ref in enumerate((row, lse, dU, 1.25 * dC)):
        e_split = np.abs(res[prec][j] - ref).max()
        e_f32 = np.abs(res[0][j] - ref).max()
        assert e_split <= 4.0 * e_f32 + 1e-6, (j, e_split, e_f32)


def _scores_matrix(S, B):
    """The B x B scores from the stored-score buffer (32 x 32 tiles (item tile, user tile),
    conftest.score_tiles); padding rows and columns dropped."""
    NT = (B + 31) // 32
    T = score_tiles(_n(S)[:NT * NT * 1024].reshape(NT, NT, 1024))          # [it, ut, user, item]
    M = T.transpose(1, 2, 0, 3).reshape(NT * 32, NT * 32)                   # [user, item]
    return M[:B, :B]


@pytest.mark.parametrize("prec", [6, 9])
def test_inbatch_split_scores_exact_on_dyadic_inputs(cuda, prec):
    """Operand maps: on dyadic inputs every product and partial sum is exact, so the stored
    scores of the split kernels equal the f32-MFMA kernels' bit for bit; lse and row losses
    agree to fp32 rounding (the 16x16x32 row pass sums the exponentials in another order)."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(prec)
    B, D = 300, 128
    U = rng.integers(-8, 9, (B, D)) / 16.0
    C = rng.integers(-8, 9, (B, D)) / 16.0
    tU, tC = _t(U, cuda), _t(C, cuda)
    outs = {}
    for pr in (0, prec):
        S = F.inbatch_scores_buffer(B, cuda)
        outs[pr] = (F.inbatch_softmax_fwd(tU, tC, scores=S, precision=pr), S)
    assert np.array_equal(_scores_matrix(outs[0][1], B), _scores_matrix(outs[prec][1], B))
    for j in (1, 2):   # row loss, lse
        a, b = _n(outs[0][0][j]), _n(outs[prec][0][j])
        assert np.abs(a - b).max() <= 4e-7 * np.abs(a).max(), (j, np.abs(a - b).max())
    assert np.abs(_n(outs[0][0][3]) - _n(outs[prec][0][3])).max() < 1e-5


def test_inbatch_softmax_large_logits_stable(cuda):
    """Online max: logits ~ +-60 would overflow a naive exp."""
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(3)
    B, D = 513, 32
    U = rng.standard_normal((B, D)) * 2.0
    C = rng.standard_normal((B, D)) * 2.0
    U32, C32 = U.astype(np.float32).astype(np.float64), C.astype(np.float32).astype(np.float64)
    row, tot, lse = O.retrieval_loss(U32, C32)
    _, ROW, LSE, _, _ = F.inbatch_softmax_fwd(_t(U, cuda), _t(C, cuda))
    assert np.isfinite(_n(ROW)).all()
    assert_close(_n(LSE), lse, 1e-4, "lse", floor=1.0)


# ---------------------------------------------------------------------------------------------
# a13: optimizers
# ---------------------------------------------------------------------------------------------
def test_sparse_adagrad_padded_ids_equal_unpadded(cuda):
    """The sync-free data-parallel exchange hands the update padded slices (id -1, zero rows)
    between ranks' real rows: bitwise the same update as the exact concatenation."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(4)
    V, D = 50, 32
    parts = [(rng.integers(0, V, n), rng.standard_normal((n, D)).astype(np.float32)) for n in (40, 25)]
    ids_u = np.concatenate([p[0] for p in parts]).astype(np.int64)
    rows_u = np.concatenate([p[1] for p in parts])
    pad = 48
    ids_p = np.full(2 * pad, -1, np.int64)
    rows_p = np.zeros((2 * pad, D), np.float32)
    for r, (i, x) in enumerate(parts):
        ids_p[r * pad: r * pad + len(i)] = i
        rows_p[r * pad: r * pad + len(i)] = x
    outs = []
    for ids, rows in ((ids_u, rows_u), (ids_p, rows_p)):
        T = _t(np.ones((V, D), np.float32), cuda)
        A = torch.full((V, D), 0.1, device=cuda)
        it = torch.zeros((), dtype=torch.int64, device=cuda)
        F.sparse_adagrad(T, A, _t(ids, cuda), _t(rows, cuda), it, 0.1, clipnorm=1.0)
        outs.append((T.cpu().numpy(), A.cpu().numpy()))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


def test_sparse_adagrad_dedupe_clip(cuda):
    import torch
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(17)
    V, D, n = 50, 32, 300
    T = rng.standard_normal((V, D)).astype(np.float32)
    A = np.full((V, D), 0.1, np.float32)
    ids = rng.integers(0, V, n).astype(np.int64)
    ids[:40] = 7                       # a hot id
    rows = rng.standard_normal((n, D)).astype(np.float32) * 0.05
    Pt, At = T.astype(np.float64), A.astype(np.float64)
    P = {"e": Pt.copy()}
    Aa = {"e": At.copy()}
    O.adagrad_apply(P, Aa, {"e": (ids, rows.astype(np.float64))}, 2500, 0.01, clipnorm=1.0)
    tt, ta = _t(T, cuda), _t(A, cuda)
    it = torch.tensor(2500, dtype=torch.int64, device=cuda)
    F.sparse_adagrad(tt, ta, _t(ids, cuda), _t(rows, cuda), it, 0.01, clipnorm=1.0)
    assert_close(_n(tt), P["e"], 1e-5, "table")
    assert_close(_n(ta), Aa["e"], 1e-5, "accum")
    # untouched rows are bit-identical
    untouched = np.setdiff1d(np.arange(V), ids)
    assert np.array_equal(tt.cpu().numpy()[untouched], T[untouched])


def test_sparse_adagrad_deterministic(cuda):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(2)
    V, D, n = 1000, 128, 20000
    T = rng.standard_normal((V, D)).astype(np.float32)
    ids = (rng.zipf(1.2, n) % V).astype(np.int64)
    rows = rng.standard_normal((n, D)).astype(np.float32)
    outs = []
    for _ in range(2):
        tt, ta = _t(T, cuda), torch.full((V, D), 0.1, device=cuda)
        it = torch.zeros((), dtype=torch.int64, device=cuda)
        F.sparse_adagrad(tt, ta, _t(ids, cuda), _t(rows, cuda), it, 0.05)
        outs.append(tt.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("D", [32, 128, 200])
@pytest.mark.parametrize("equal_n", [True, False])
@pytest.mark.parametrize("ext_sumsq", [False, True])
def test_sparse_adagrad_multi_matches_single(cuda, D, equal_n, ext_sumsq):
    """rs_sparse_adagrad_multi_f32 against one rs_sparse_adagrad_*_f32 per table: bitwise when
    every table has the same entry count (same windows, same ordered sums), within fp32 rounding
    of the association otherwise; invalid ids (-1, num_rows), a hot id, an empty table, strided
    gradient rows and caller-supplied clip norms^2 included."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(D + 7 * equal_n + 3 * ext_sumsq)
    V = [50, 300, 7, 1000, 64]
    ns = [700] * 5 if equal_n else [700, 0, 37, 2000, 129]
    tabs, ids, rows, ssq = [], [], [], []
    for v, n in zip(V, ns):
        tabs.append(rng.standard_normal((v, D)).astype(np.float32))
        i = (rng.zipf(1.3, n) % (v + 2) - 1).astype(np.int64)  # -1 .. v: invalid ids at both ends
        ids.append(i)
        g = rng.standard_normal((n, D + 8)).astype(np.float32) * 0.05  # rows of stride D + 8
        rows.append(g)
        ssq.append(np.float32((g[:, :D].astype(np.float64) ** 2).sum() * 0.5))
    it = torch.tensor(1234, dtype=torch.int64, device=cuda)
    single, multi = [], []
    for k in range(5):
        tt, ta = _t(tabs[k], cuda), torch.full((V[k], D), 0.1, device=cuda)
        g = _t(rows[k], cuda)[:, :D]
        F.sparse_adagrad(tt, ta, _t(ids[k], cuda), g, it, 0.05, clipnorm=1.0,
                         sumsq=_t(np.array(ssq[k]), cuda) if ext_sumsq else None)
        single.append((tt.cpu().numpy(), ta.cpu().numpy()))
    tts = [_t(t, cuda) for t in tabs]
    tas = [torch.full((v, D), 0.1, device=cuda) for v in V]
    F.sparse_adagrad_multi(tts, tas, [_t(i, cuda) for i in ids], [_t(r, cuda)[:, :D] for r in rows], it, 0.05,
                           clipnorm=1.0, sumsq=[_t(np.array(s), cuda) for s in ssq] if ext_sumsq else None)
    torch.cuda.synchronize()
    for k in range(5):
        t_m, a_m = tts[k].cpu().numpy(), tas[k].cpu().numpy()
        if equal_n:
            assert np.array_equal(t_m, single[k][0]) and np.array_equal(a_m, single[k][1]), k
        else:
            assert np.allclose(t_m, single[k][0], rtol=1e-6, atol=1e-6), k
            assert np.allclose(a_m, single[k][1], rtol=1e-5, atol=1e-7), k
        untouched = np.setdiff1d(np.arange(V[k]), ids[k])
        assert np.array_equal(t_m[untouched], tabs[k][untouched]), k


@pytest.mark.parametrize("D,ns", [(64, [700, 0, 37, 2000, 129]), (128, [65536, 65536]), (32, [4096, 4096])])
def test_sparse_adagrad_ordered_equals_sorted(cuda, D, ns):
    """rs_sparse_adagrad_multi_step_ordered_f32 (each table's stable ascending-id order supplied, as
    the in-batch id plan's order entry; the update's own sort skipped) against the sorting entry:
    tables, accumulators and the step counter bitwise equal; invalid ids at both ends, a hot id,
    an empty table."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(D + len(ns))
    V = [50, 300, 7, 1000, 64][: len(ns)] if len(ns) == 5 else [1000000, 100000]
    res = []
    for ordered in (False, True):
        r2 = np.random.default_rng(5)
        tts, tas, ids, rows, orders = [], [], [], [], []
        for v, n in zip(V, ns):
            tts.append(_t(r2.standard_normal((v, D)).astype(np.float32), cuda))
            tas.append(torch.full((v, D), 0.1, device=cuda))
            i = (r2.zipf(1.3, n) % (v + 2) - 1).astype(np.int64)
            ids.append(_t(i, cuda))
            rows.append(_t(r2.standard_normal((n, D)).astype(np.float32) * 0.05, cuda))
            key = np.where((i < 0) | (i >= v), v, i)
            orders.append(_t(np.argsort(key, kind="stable").astype(np.int32), cuda, torch.int32))
        it = torch.tensor(1234, dtype=torch.int64, device=cuda)
        F.sparse_adagrad_multi(tts, tas, ids, rows, it, 0.05, clipnorm=1.0, increment=True,
                               orders=orders if ordered else None)
        torch.cuda.synchronize()
        res.append([t.cpu() for t in tts] + [a.cpu() for a in tas] + [it.cpu()])
    assert int(res[1][-1]) == 1235
    for k, (a, b) in enumerate(zip(*res)):
        assert torch.equal(a, b), k


def test_dense_adagrad_multi_tensor(cuda):
    import torch
    optim = pkg("optim")
    O = oracle()
    rng = np.random.default_rng(4)
    shapes = [(128, 256), (256,), (3, 256), (1,), (384, 1)]
    params = [torch.nn.Parameter(_t(rng.standard_normal(s).astype(np.float32), cuda)) for s in shapes]
    grads = [rng.standard_normal(s).astype(np.float32) * (0.01 if i % 2 else 3.0) for i, s in enumerate(shapes)]
    P = {str(i): params[i].detach().cpu().double().numpy().copy() for i in range(len(shapes))}
    A = {k: np.full_like(v, 0.1) for k, v in P.items()}
    G = {str(i): grads[i].astype(np.float64) for i in range(len(shapes))}

    class _E:  # no embeddings
        pass

    opt = optim.Adagrad(params, [], learning_rate=optim.ExponentialDecay(0.02, 1000, 0.96, True), clipnorm=1.0)
    for step in range(3):
        for p, g in zip(params, grads):
            p.grad = _t(g, cuda)
        opt.step()
        O.adagrad_apply(P, A, G, step, 0.02, clipnorm=1.0)
    assert int(opt.iterations.item()) == 3
    for i in range(len(shapes)):
        assert_close(_n(params[i]), P[str(i)], 1e-5, f"param {i}")
        assert_close(_n(opt.accum[i]), A[str(i)], 1e-5, f"accum {i}")


# ---------------------------------------------------------------------------------------------
# a16: top-K (bit-exact on dyadic grid)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("Q,N,D,k,lvl", [
    (1, 5000, 128, 100, 8), (37, 3000, 64, 10, 8), (64, 10000, 128, 50, 8), (5, 100, 32, 100, 8),
    (16, 20000, 128, 128, 8), (17, 20000, 128, 1, 8), (5, 5, 32, 5, 8), (3, 31, 64, 7, 8),
    # heavy ties: few distinct values -> order decided by the index
    (9, 40000, 32, 100, 1), (33, 7000, 128, 64, 1),
    # multi-slice, XCD-aware mapping (slice count a multiple of 8)
    (1, 100000, 128, 10, 8), (40, 300000, 128, 100, 8), (300, 50000, 64, 20, 8)])
def test_topk_dyadic_bitexact(cuda, Q, N, D, k, lvl):
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(Q + N + D + k)
    q = rng.integers(-lvl, lvl + 1, (Q, D)).astype(np.float32) / 16.0
    it = rng.integers(-lvl, lvl + 1, (N, D)).astype(np.float32) / 16.0
    sc, idx = O.topk_ip(q, it, k)
    S, I = F.topk_ip(_t(q, cuda), _t(it, cuda), k)
    assert np.array_equal(I.cpu().numpy(), idx)
    assert np.array_equal(S.cpu().numpy().astype(np.float64), sc)


@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("Q,N,k,lvl", [(65, 3000, 10, 8), (100, 50000, 100, 8), (300, 20000, 50, 2),
                                       (1024, 40000, 100, 16)])
def test_topk_split_precision_dyadic_bitexact(cuda, Q, N, k, lvl, prec):
    """Split-operand scan (Q > 64, D = 128): on dyadic data every product and partial sum is
    exact, so scores and indices equal the oracle's bit for bit (ties included)."""
    F = pkg("functional")
    O = oracle()
    D = 128
    rng = np.random.default_rng(Q + N + k + prec)
    q = rng.integers(-lvl, lvl + 1, (Q, D)).astype(np.float32) / 16.0
    it = rng.integers(-lvl, lvl + 1, (N, D)).astype(np.float32) / 16.0
    sc, idx = O.topk_ip(q, it, k)
    S, I = F.topk_ip(_t(q, cuda), _t(it, cuda), k, precision=prec)
    assert np.array_equal(I.cpu().numpy(), idx)
    assert np.array_equal(S.cpu().numpy().astype(np.float64), sc)


@pytest.mark.parametrize("prec", [6, 9])
def test_topk_split_precision_gaussian(cuda, prec):
    """Gaussian data: the split scan's scores are within fp32 rounding of the float64 truth and
    its lists are the true top-k except where two scores are within that rounding."""
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(prec)
    Q, N, D, k = 200, 30000, 128, 50
    q = rng.standard_normal((Q, D)).astype(np.float32)
    it = rng.standard_normal((N, D)).astype(np.float32)
    sc, idx = O.topk_ip(q.astype(np.float64), it.astype(np.float64), k)
    S, I = F.topk_ip(_t(q, cuda), _t(it, cuda), k, precision=prec)
    S, I = S.cpu().numpy().astype(np.float64), I.cpu().numpy()
    assert np.abs(S - sc).max() < 1e-4
    exact = (q.astype(np.float64) @ it.astype(np.float64).T)
    got_true = np.take_along_axis(exact, I, 1)
    # every returned item's true score is within 1e-4 of the true k-th best score or better
    assert (got_true >= sc[:, -1:] - 1e-4).all()


def test_topk_shard_merge(cuda):
    import torch
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(9)
    Q, N, D, k, shards = 8, 4000, 64, 20, 4
    q = rng.integers(-8, 9, (Q, D)).astype(np.float32) / 16.0
    it = rng.integers(-8, 9, (N, D)).astype(np.float32) / 16.0
    sc, idx = O.topk_ip(q, it, k)
    per = N // shards
    parts_s, parts_i = [], []
    for s in range(shards):
        S, I = F.topk_ip(_t(q, cuda), _t(it[s * per:(s + 1) * per], cuda), k, index_base=s * per)
        parts_s.append(S)
        parts_i.append(I)
    S, I = F.topk_merge(torch.stack(parts_s, 1).contiguous(), torch.stack(parts_i, 1).contiguous(), k)
    assert np.array_equal(I.cpu().numpy(), idx)


# ---------------------------------------------------------------------------------------------
# plane-image GEMM (pre-split operands, LDS-DMA ring): bitwise the split GEMM's sums
# ---------------------------------------------------------------------------------------------
# the row GEMM's layout rule: M % 4 == 0, and N % 4 == 0 unless B is transposed (only valid
# cases are generated, so a skip in this test is a real skip)
_PLANE_CASES = [(ta, tb, M, N, K) for ta, tb in [(0, 0), (0, 1), (1, 0), (1, 1)]
                for M, N, K in [(300, 200, 100), (256, 256, 16), (517, 1030, 333), (64, 3344, 3344), (33, 7, 5),
                                (36, 7, 5)]
                if M % 4 == 0 and (tb or N % 4 == 0)]


@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("ta,tb,M,N,K", _PLANE_CASES)
def test_gemm_planes_bitwise_equal_to_split_gemm(cuda, prec, ta, tb, M, N, K):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(M + N + K + 10 * ta + 20 * tb)
    Ka = K if K % 4 == 0 or (ta and not tb) else K + (4 - K % 4)   # the row GEMM's K % 4 rule
    a = rng.standard_normal((Ka, M) if ta else (M, Ka)).astype(np.float32)
    b = rng.standard_normal((N, Ka) if tb else (Ka, N)).astype(np.float32)
    ta_, tb_ = _t(a, cuda), _t(b, cuda)
    bias = _t(rng.standard_normal(N).astype(np.float32), cuda)
    ref = F.gemm(ta_, tb_, trans_a=bool(ta), trans_b=bool(tb), bias=bias, relu=True, precision=prec)
    a_img = F.plane_image(ta_, F.PLANE_KM if ta else F.PLANE_KC)
    b_img = F.plane_image(tb_, F.PLANE_KC if tb else F.PLANE_KM)
    out = F.gemm_planes(a_img, b_img, M, N, Ka, bool(ta), bool(tb), bias=bias, relu=True, precision=prec)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    a64 = a.astype(np.float64).T if ta else a.astype(np.float64)
    b64 = b.astype(np.float64).T if tb else b.astype(np.float64)
    assert_close(_n(out), np.maximum(a64 @ b64 + _n(bias), 0.0), 1e-5, "planes vs fp64")


@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("M,N,K", [(3344, 3344, 4096), (128, 256, 65536), (200, 300, 1000)])
def test_gemm_planes_splitk_weight_grad(cuda, prec, M, N, K):
    F = pkg("functional")
    rng = np.random.default_rng(M * N + K)
    x = rng.standard_normal((K, M)).astype(np.float32)
    g = rng.standard_normal((K, N)).astype(np.float32)
    add = rng.standard_normal((M, N)).astype(np.float32)
    tx, tg = _t(x, cuda), _t(g, cuda)
    dW = F.gemm_planes_splitk(F.plane_image(tx, F.PLANE_KM), F.plane_image(tg, F.PLANE_KM), M, N, K, True, False,
                              addend=_t(add, cuda), addend_scale=0.5, precision=prec)
    ref = x.astype(np.float64).T @ g.astype(np.float64) + 0.5 * add
    assert_close(_n(dW), ref, 1e-5, "dW", floor=0.0)


# ---------------------------------------------------------------------------------------------
# data-parallel exchange kernels: local deduplication, update with the exchanged norm
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n,V,D", [(1, 5, 32), (1000, 50, 128), (70000, 3000, 64), (65536, 10_000_000, 128)])
def test_sparse_dedupe(cuda, n, V, D):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(n + V)
    ids = rng.integers(-2, V + 2, n).astype(np.int64) if V < 100 else rng.zipf(1.1, n).astype(np.int64) % (V + 3) - 1
    G = (rng.integers(-64, 65, (n, 2 * D)) / 64.0).astype(np.float32)     # dyadic: exact sums
    rows = _t(G, cuda)[:, D // 2: D // 2 + D]                                # row-strided view
    uid, urows, count, ss = F.sparse_dedupe(_t(ids, cuda), rows, V)
    torch.cuda.synchronize()
    ok = (ids >= 0) & (ids < V)
    u, inv = np.unique(ids[ok], return_inverse=True)
    ref = np.zeros((len(u), D))
    np.add.at(ref, inv, G[ok][:, D // 2: D // 2 + D].astype(np.float64))
    c = int(count.item())
    assert c == len(u)
    assert np.array_equal(uid.cpu().numpy()[:c], u)
    assert np.array_equal(urows.cpu().numpy()[:c].astype(np.float64), ref)
    raw = G[:, D // 2: D // 2 + D].astype(np.float64)
    assert abs(float(ss) - np.sum(raw ** 2)) <= 1e-6 * np.sum(raw ** 2)


def test_sparse_update_on_deduplicated_rows_with_external_norm(cuda):
    """What every replica applies after the deduplicated exchange (two replicas' unique rows in
    rank order + the all-reduced raw norm) equals the update on the raw concatenation."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(7)
    V, D, n = 500, 128, 6000
    ids = [rng.zipf(1.2, n).astype(np.int64) % V for _ in range(2)]
    rows = [rng.standard_normal((n, D)).astype(np.float32) * 0.01 for _ in range(2)]
    T0 = rng.standard_normal((V, D)).astype(np.float32)
    outs = []
    for mode in ("raw", "dedupe"):
        T = _t(T0, cuda)
        A = torch.full((V, D), 0.1, device=cuda)
        it = torch.zeros((), dtype=torch.int64, device=cuda)
        if mode == "raw":
            F.sparse_adagrad(T, A, _t(np.concatenate(ids), cuda), _t(np.concatenate(rows), cuda), it, 0.05)
        else:
            parts = [F.sparse_dedupe(_t(i, cuda), _t(r, cuda), V) for i, r in zip(ids, rows)]
            gi = torch.cat([p[0][:int(p[2])] for p in parts])
            gr = torch.cat([p[1][:int(p[2])] for p in parts])
            ss = parts[0][3] + parts[1][3]
            F.sparse_adagrad(T, A, gi, gr, it, 0.05, sumsq=ss)
        torch.cuda.synchronize()
        outs.append((T.cpu().numpy(), A.cpu().numpy()))
    assert np.abs(outs[0][0] - outs[1][0]).max() <= 1e-6
    assert np.abs(outs[0][1] - outs[1][1]).max() <= 1e-6


@pytest.mark.parametrize("M,N,K,trans_a,trans_b", [(300, 200, 100, 0, 1), (5, 8, 4, 0, 0), (600, 3344, 3344, 0, 1),
                                                   (1032, 516, 76, 1, 0), (257, 1024, 3344, 0, 1)])
def test_xgemm_matches_fp64(cuda, M, N, K, trans_a, trans_b):
    """Plane-pair GEMM (rs_xgemm_*: images built from either orientation, two cross products per
    16x16x32 MFMA) with bias + ReLU against float64 at the fp32 bar, and equal to the split-at-
    staging GEMM of the same precision within a few ulps."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(M + N + K)
    a = rng.standard_normal((K, M) if trans_a else (M, K)).astype(np.float32)
    b = rng.standard_normal((N, K) if trans_b else (K, N)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    ta, tb, tbias = _t(a, cuda), _t(b, cuda), _t(bias, cuda)
    a_img = F.xgemm_image(ta, trans=bool(trans_a))          # A viewed as [M][K]
    b_img = F.xgemm_image(tb, trans=not trans_b)            # B viewed as [N][K]
    out = F.xgemm(a_img, b_img, M, N, K, bias=tbias, relu=True)
    ref = F.gemm(ta, tb, trans_a=bool(trans_a), trans_b=bool(trans_b), bias=tbias, relu=True, precision=6)
    torch.cuda.synchronize()
    a64 = (a.T if trans_a else a).astype(np.float64)
    b64 = (b.T if trans_b else b).astype(np.float64)
    assert_close(_n(out), np.maximum(a64 @ b64 + bias, 0.0), 1e-5, "xgemm vs fp64")
    assert float((out - ref).abs().max()) <= 4e-6 * max(float(ref.abs().max()), 1.0)


@pytest.mark.parametrize("M,N,K", [(3344, 3344, 16384), (128, 256, 65536), (64, 48, 1000)])
def test_xgemm_splitk_weight_grad(cuda, M, N, K):
    """dW = X^T G on the plane-pair kernel with the contraction split over workgroups (ordered
    slabs), including the K = 65536 contraction of the c3 tower dW, against float64."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(M * 7 + N + K)
    x = (rng.standard_normal((K, M)) * 0.5).astype(np.float32)
    g = rng.standard_normal((K, N)).astype(np.float32)
    tx, tg = _t(x, cuda), _t(g, cuda)
    dW = F.xgemm_splitk(F.xgemm_image(tx, trans=True), F.xgemm_image(tg, trans=True), M, N, K)
    torch.cuda.synchronize()
    ref = x.astype(np.float64).T @ g.astype(np.float64)
    assert_close(_n(dW), ref, 1e-5, "xgemm splitk vs fp64")


@pytest.mark.parametrize("prec", [0, 6])
@pytest.mark.parametrize("M,N,K", [(128, 256, 4096), (256, 128, 65536), (4, 4, 5), (3344, 1024, 300)])
def test_gemm_wgrad_bias(cuda, prec, M, N, K):
    """dW = X^T G and db = colsum(G) from one split-K GEMM (the all-ones row of X^T), against
    float64."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(M + 3 * N + K)
    x = rng.standard_normal((K, M)).astype(np.float32)
    g = rng.standard_normal((K, N)).astype(np.float32)
    dW, db = F.gemm_wgrad_bias(_t(x, cuda), _t(g, cuda), prec)
    W = rng.standard_normal((M, N)).astype(np.float32)
    sc = _t(np.array(0.5, dtype=np.float32), cuda)
    dW2, db2 = F.gemm_wgrad_bias(_t(x, cuda), _t(g, cuda), prec, W=_t(W, cuda), w_scale=2e-3, w_dscale=sc)
    torch.cuda.synchronize()
    assert_close(_n(dW), x.astype(np.float64).T @ g.astype(np.float64), 1e-5, "dW")
    assert_close(_n(db), g.astype(np.float64).sum(0), 1e-5, "db")
    # the l2 regularizer gradient folded into the reduction with a device-side scale
    assert_close(_n(dW2), x.astype(np.float64).T @ g.astype(np.float64) + 1e-3 * W, 1e-5, "dW + 2 l2 g W")
    assert torch.equal(db, db2)


@pytest.mark.parametrize("prec", [0, 6])
@pytest.mark.parametrize("G,M,K,N", [(2, 4096, 128, 256), (2, 300, 64, 48), (3, 1000, 256, 128), (2, 65536, 64, 128),
                                     (4, 17, 12, 8)])
def test_gemm_group_matches_single(cuda, prec, G, M, K, N):
    """Grouped launches (one grid for G problems of one shape: the two towers' Dense layers) give
    each problem bitwise the result of its own launch: forward with bias + ReLU, dX with the ReLU
    mask epilogue, and dW + db from the split-K weight-gradient GEMM."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(G * M + K + N + prec)
    xs = [_t(rng.standard_normal((M, K)).astype(np.float32), cuda) for _ in range(G)]
    Ws = [_t((rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32), cuda) for _ in range(G)]
    bs = [_t(rng.standard_normal(N).astype(np.float32), cuda) for _ in range(G)]
    gy = [_t(rng.standard_normal((M, N)).astype(np.float32), cuda) for _ in range(G)]
    ys = F.gemm_group(xs, Ws, bias=bs, relu=True, precision=prec)
    dxs = F.gemm_group(gy, Ws, trans_b=True, mask=xs, precision=prec)
    wg = F.gemm_wgrad_bias_group(xs, gy, prec)
    for g in range(G):
        y1 = F.gemm(xs[g], Ws[g], bias=bs[g], relu=True, precision=prec)
        dx1 = F.gemm(gy[g], Ws[g], trans_b=True, mask=xs[g], precision=prec)
        dW1, db1 = F.gemm_wgrad_bias(xs[g], gy[g], prec)
        assert torch.equal(ys[g], y1), g
        assert torch.equal(dxs[g], dx1), g
        assert torch.equal(wg[g][0], dW1) and torch.equal(wg[g][1], db1), g
    ref = np.maximum(_n(xs[0]).astype(np.float64) @ _n(Ws[0]) + _n(bs[0]), 0)
    assert_close(_n(ys[0]), ref, 1e-5, "y")


@pytest.mark.parametrize("prec", [0, 6])
def test_tower_group_node_matches_separate(cuda, prec):
    """The user and item towers as one MLPGroupFn node (models.dense_stack_group) against one
    MLPFn per tower: outputs, input gradients and every parameter gradient bitwise equal."""
    import torch
    models = pkg("models")
    outs = []
    for grouped in (False, True):
        towers = [models.Tower(128, [256, 128, 64], 128, seed=s, device=cuda) for s in (10, 30)]
        for t in towers:
            for layer in t.layers:
                layer.precision = prec
        g = torch.Generator(device="cpu").manual_seed(1)
        xs = [torch.randn(4096, 128, generator=g).to(cuda).requires_grad_(True) for _ in range(2)]
        gys = [torch.randn(4096, 128, generator=g).to(cuda) for _ in range(2)]
        if grouped:
            ys = models.dense_stack_group([t.layers for t in towers], xs)
        else:
            ys = [models.dense_stack(t.layers, x) for t, x in zip(towers, xs)]
        torch.autograd.backward(ys, gys)
        torch.cuda.synchronize()
        outs.append([y.detach().clone() for y in ys] + [x.grad.clone() for x in xs]
                    + [p.grad.clone() for t in towers for p in t.parameters()])
    assert len(outs[0]) == len(outs[1])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("M,dims,relus", [(4096, (128, 256, 128, 64, 128), (1, 1, 1, 0)),   # a Tower
                                          (300, (256, 256, 128, 64), (1, 1, 1)),            # the deep net
                                          (1, (96, 64), (0,)), (33, (32, 128, 256), (1, 0))])
def test_mlp_forward_one_launch(cuda, prec, M, dims, relus):
    """rs_mlp_fwd_prec_f32 (a whole Dense stack in one launch, 32 rows per workgroup carried
    through every layer in LDS): every layer's output against float64 at the split precision's
    bar and against the per-layer GEMMs at that precision (same products, other k-sum order:
    fp32 rounding apart), ragged row counts; two stacks in one grid give each stack bitwise its
    own one-stack launch."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(M + sum(dims) + prec)
    L = len(relus)
    xs = [_t(rng.standard_normal((M, dims[0])).astype(np.float32), cuda) for _ in range(2)]
    Ws = [[_t((rng.standard_normal((dims[l], dims[l + 1])) / np.sqrt(dims[l])).astype(np.float32), cuda)
           for l in range(L)] for _ in range(2)]
    bs = [[_t(rng.standard_normal(dims[l + 1]).astype(np.float32), cuda) for l in range(L)] for _ in range(2)]
    ys2 = F.mlp_forward(xs, Ws, bs, relus, prec)
    ys1 = F.mlp_forward(xs[:1], Ws[:1], bs[:1], relus, prec)
    torch.cuda.synchronize()
    for g in range(2):
        ref = _n(xs[g]).astype(np.float64)
        y = xs[g]
        for l in range(L):
            ref = ref @ _n(Ws[g][l]).astype(np.float64) + _n(bs[g][l])
            if relus[l]:
                ref = np.maximum(ref, 0)
            assert ys2[l][g].shape == (M, dims[l + 1])
            assert_close(_n(ys2[l][g]), ref, 1e-5, f"stack {g} layer {l}")
            # the per-layer GEMM on the fused kernel's own input of this layer
            y1 = F.gemm(y, Ws[g][l], bias=bs[g][l], relu=bool(relus[l]), precision=prec)
            torch.cuda.synchronize()
            assert_close(_n(ys2[l][g]), _n(y1).astype(np.float64), 1e-5, f"vs gemm {g} {l}")
            y = ys2[l][g]
    for l in range(L):
        assert torch.equal(ys2[l][0], ys1[l][0]), l


@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("M,dims,relus,want_dx", [(4096, (128, 256, 128, 64, 128), (1, 1, 1, 0), True),
                                                  (300, (256, 256, 128, 64), (1, 1, 1), True),
                                                  (77, (96, 64, 128), (1, 1), False), (1, (64, 64), (0,), True)])
def test_mlp_backward_chain_one_launch(cuda, prec, M, dims, relus, want_dx):
    """rs_mlp_bwd_chain_prec_f32 (the input-gradient chain of a Dense stack in one launch): every
    layer's input gradient, masked by the previous layer's ReLU (y > 0), against float64 and
    against the per-layer dX GEMM with the mask epilogue; dL/dx skipped when not wanted; two stacks
    in one grid bitwise their one-stack launches."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(M + sum(dims) + prec + 1)
    L = len(relus)
    Ws = [[_t((rng.standard_normal((dims[l], dims[l + 1])) / np.sqrt(dims[l])).astype(np.float32), cuda)
           for l in range(L)] for _ in range(2)]
    # forward outputs with ReLU zeros where the layer has one
    ys = [[_t(np.maximum(rng.standard_normal((M, dims[l + 1])), 0 if relus[l] else -9).astype(np.float32), cuda)
           for l in range(L)] for _ in range(2)]
    gt = [_t(rng.standard_normal((M, dims[L])).astype(np.float32), cuda) for _ in range(2)]
    gin2 = F.mlp_backward_chain(gt, Ws, ys, relus, prec, want_dx)
    gin1 = F.mlp_backward_chain(gt[:1], Ws[:1], ys[:1], relus, prec, want_dx)
    torch.cuda.synchronize()
    for s in range(2):
        ref = _n(gt[s]).astype(np.float64)
        g = gt[s]
        for l in range(L - 1, -1, -1):
            ref = ref @ _n(Ws[s][l]).astype(np.float64).T
            m = ys[s][l - 1] if l > 0 and relus[l - 1] else None
            if m is not None:
                ref = ref * (_n(m) > 0)
            if l == 0 and not want_dx:
                assert gin2[0][s] is None
                break
            assert gin2[l][s].shape == (M, dims[l])
            assert_close(_n(gin2[l][s]), ref, 1e-5, f"stack {s} layer {l}")
            g1 = F.gemm(g, Ws[s][l], trans_b=True, mask=m, precision=prec)
            torch.cuda.synchronize()
            assert_close(_n(gin2[l][s]), _n(g1), 1e-5, f"vs gemm {s} {l}")
            if m is not None:
                assert bool(((gin2[l][s] != 0) <= (m > 0)).all())
            g = gin2[l][s]
    for l in range(L):
        if gin1[l][0] is not None:
            assert torch.equal(gin2[l][0], gin1[l][0]), l


@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("M,dims", [(4096, (128, 256, 128, 64, 128)), (300, (256, 256, 128, 64)), (100, (64, 64)),
                                    (16384, (128, 64))])
def test_mlp_wgrad_one_launch(cuda, prec, M, dims):
    """rs_mlp_wgrad_prec_f32 (every layer's dW = x^T g and db = colsum g of a stack in one launch,
    M split into slices summed in order by each tile's last workgroup): against float64 at the
    split precision's bar and gemm_wgrad_bias, with and without the folded l2 term; a second launch
    bitwise the first (the tickets reset themselves); two stacks bitwise their one-stack launches."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(M + sum(dims) + prec + 2)
    L = len(dims) - 1
    xs = [[_t(rng.standard_normal((M, dims[l])).astype(np.float32), cuda) for l in range(L)] for _ in range(2)]
    gs = [[_t(rng.standard_normal((M, dims[l + 1])).astype(np.float32), cuda) for l in range(L)] for _ in range(2)]
    Ws = [[_t(rng.standard_normal((dims[l], dims[l + 1])).astype(np.float32), cuda) for l in range(L)]
          for _ in range(2)]
    sc = torch.tensor(0.25, device=cuda)
    w2 = F.mlp_wgrad(xs, gs, prec)
    w2b = F.mlp_wgrad(xs, gs, prec)
    w1 = F.mlp_wgrad(xs[:1], gs[:1], prec)
    wr = F.mlp_wgrad(xs, gs, prec, W_lists=Ws, w_scale=2e-3, w_dscale=sc)
    torch.cuda.synchronize()
    for s in range(2):
        for l in range(L):
            x, g = _n(xs[s][l]), _n(gs[s][l])
            ref_w, ref_b = x.T @ g, g.sum(0)
            dW, db = w2[s][l]
            assert dW.shape == (dims[l], dims[l + 1]) and db.shape == (dims[l + 1],)
            assert_close(_n(dW), ref_w, 1e-5, f"dW {s} {l}")
            assert_close(_n(db), ref_b, 1e-5, f"db {s} {l}")
            dW1, db1 = F.gemm_wgrad_bias(xs[s][l], gs[s][l], prec)
            torch.cuda.synchronize()
            assert_close(_n(dW), _n(dW1), 1e-5, f"vs gemm_wgrad_bias {s} {l}")
            assert torch.equal(dW, w2b[s][l][0]) and torch.equal(db, w2b[s][l][1])
            if s == 0:
                assert torch.equal(dW, w1[0][l][0]) and torch.equal(db, w1[0][l][1])
            assert_close(_n(wr[s][l][0]), ref_w + 5e-4 * _n(Ws[s][l]), 1e-5, f"dW + l2 {s} {l}")
            assert torch.equal(wr[s][l][1], db)


def test_mlp_wgrad_empty_batch(cuda):
    """rs_mlp_wgrad_prec_f32 with M = 0 writes dW = 0 and db = 0, or the folded
    l2 term w_scale * w_dscale * W, into outputs the caller allocated uninitialised."""
    import torch
    F = pkg("functional")
    dims = (128, 256, 64)
    xs = [[torch.empty((0, dims[l]), device=cuda) for l in range(2)]]
    gs = [[torch.empty((0, dims[l + 1]), device=cuda) for l in range(2)]]
    Ws = [[torch.randn((dims[l], dims[l + 1]), device=cuda) for l in range(2)]]
    sc = torch.tensor(0.5, device=cuda)
    for W_lists in (None, Ws):
        out = F.mlp_wgrad(xs, gs, 6, W_lists=W_lists, w_scale=0.25 if W_lists else 0.0,
                          w_dscale=sc if W_lists else None)
        torch.cuda.synchronize()
        for l in range(2):
            dW, db = out[0][l]
            want = 0.125 * Ws[0][l] if W_lists else torch.zeros_like(Ws[0][l])
            assert torch.equal(dW, want) and torch.equal(db, torch.zeros_like(db)), l


@pytest.mark.parametrize("act", ["linear", "relu"])
@pytest.mark.parametrize("mode", ["per_layer", "wgrad_only", "fused"])
def test_tower_stack_paths_agree(cuda, monkeypatch, mode, act):
    """The tower group node on each of its three forms (per-layer GEMMs; per-layer forward / dX with
    the one-launch weight gradients, the large-batch form; the one-launch forward, chain and weight
    gradients): outputs, dL/dx and every parameter gradient against float64 under the ReLU gates
    that form's own forward produced (functional.record_relu_gates, checked against its backward),
    at the north-star 1e-4. (The one-launch forward sums k in another order than the per-layer
    GEMMs, so a pre-activation within rounding of zero can take the other side of its gate: each
    form is held to the oracle under its own gates, never to another GPU form.)"""
    import torch
    F = pkg("functional")
    models = pkg("models")
    O = oracle()
    limits = {"per_layer": (0, 0), "wgrad_only": (0, 1 << 30), "fused": (1 << 30, 1 << 30)}[mode]
    monkeypatch.setattr(F, "MLP_FUSED_MAX_M", limits[0])
    monkeypatch.setattr(F, "MLP_WGRAD_MAX_M", limits[1])
    towers = [models.Tower(128, [256, 128, 64], 128, seed=s, device=cuda) for s in (10, 30)]
    for t in towers:
        for layer in t.layers:
            layer.precision = 6
            layer.bias.data.uniform_(-0.05, 0.05)
            if act == "linear":
                layer.activation = "linear"
    g = torch.Generator(device="cpu").manual_seed(2)
    xs = [torch.randn(3000, 128, generator=g).to(cuda).requires_grad_(True) for _ in range(2)]
    gys = [torch.randn(3000, 128, generator=g).to(cuda) for _ in range(2)]
    with F.record_relu_gates() as rec:
        ys = models.dense_stack_group([t.layers for t in towers], xs)
        torch.autograd.backward(ys, gys)
    torch.cuda.synchronize()
    for t, x, gy, y in zip(towers, xs, gys, ys):
        layers = [(_n(layer.kernel), _n(layer.bias)) for layer in t.layers]
        if act == "relu":
            gates = stack_gates(t.layers, rec)
            masks = gates + [None]
        else:    # linear hidden layers: the oracle's gates all open
            assert rec["fwd"][t.layers[0].kernel.data_ptr()] == []
            masks = [np.ones((x.shape[0], layer.kernel.shape[1]), bool) for layer in t.layers[:-1]] + [None]
        # (oracle.mlp_forward with relu_last=False gates the hidden layers only)
        ref_y, acts = O.mlp_forward(_n(x), layers, relu_last=False, masks=masks)
        ref_gx, ref_g = O.mlp_backward(acts, layers, _n(gy), relu_last=False, masks=masks)
        assert_close(_n(y), ref_y, 1e-4, "y", floor=0.0)
        assert_close(_n(x.grad), ref_gx, 1e-4, "dL/dx", floor=0.0)
        for k, layer in enumerate(t.layers):
            assert_close(_n(layer.kernel.grad), ref_g[k][0], 1e-4, f"dW {k}", floor=0.0)
            assert_close(_n(layer.bias.grad), ref_g[k][1], 1e-4, f"db {k}", floor=0.0)


def test_tower_skinny_weight_images_bitwise(cuda, monkeypatch):
    """The large-batch tower GEMMs with their weights from fragment images (the skinny kernel stages
    pre-split fragments, rs_gemm_group_img_prec_f32) against the same GEMMs splitting the weights
    themselves: outputs, input gradients and every parameter gradient bitwise equal."""
    import torch
    F = pkg("functional")
    models = pkg("models")
    monkeypatch.setattr(F, "MLP_FUSED_MAX_M", 0)
    monkeypatch.setattr(F, "MLP_WGRAD_MAX_M", 0)
    outs = []
    for img in (False, True):
        monkeypatch.setattr(F, "SKINNY_IMG", img)
        towers = [models.Tower(128, [256, 128, 64], 128, seed=s, device=cuda) for s in (10, 30)]
        for t in towers:
            for layer in t.layers:
                layer.precision = 6
        g = torch.Generator(device="cpu").manual_seed(3)
        xs = [torch.randn(20000, 128, generator=g).to(cuda).requires_grad_(True) for _ in range(2)]
        gys = [torch.randn(20000, 128, generator=g).to(cuda) for _ in range(2)]
        ys = models.dense_stack_group([t.layers for t in towers], xs)
        torch.autograd.backward(ys, gys)
        torch.cuda.synchronize()
        outs.append([y.detach().clone() for y in ys] + [x.grad.clone() for x in xs]
                    + [p.grad.clone() for t in towers for p in t.parameters()])
    for i, (a, b) in enumerate(zip(*outs)):
        assert torch.equal(a, b), i


def test_mlp_forward_rejects_unsupported_widths(cuda):
    """Widths outside the one-launch kernel's set are refused with an error, not computed."""
    F = pkg("functional")
    import torch
    x = torch.zeros((64, 128), device=cuda)
    W = torch.zeros((128, 48), device=cuda)
    assert not F.mlp_fused_ok(64, 128, [W], 6)
    with pytest.raises(Exception, match="width"):
        F.mlp_forward([x], [[W]], [[None]], (1,), 6)


def test_sum_squares_multi(cuda):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(5)
    xs = [rng.standard_normal(n).astype(np.float32) for n in (256 * 256, 256 * 128, 7, 1)]
    out = F.sum_squares_multi([_t(x, cuda) for x in xs], 1e-4)
    torch.cuda.synchronize()
    ref = 1e-4 * sum(float((x.astype(np.float64) ** 2).sum()) for x in xs)
    assert abs(float(out) - ref) <= 1e-6 * abs(ref)


# ---------------------------------------------------------------------------------------------
# skinny split GEMM (the Dense layers' forward / dX when the batch gives >= 256 workgroups of 128
# rows x all N, weights staged once per 32-k chunk): against float64 at the split precision's bar
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("M,K,N", [(65536, 128, 256), (65536, 256, 128), (32768, 64, 128), (40007, 128, 64),
                                   (33001, 32, 192), (32800, 256, 32)])
def test_skinny_gemm_forward_and_dx(cuda, prec, M, K, N):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(M + 7 * K + N + prec)
    x = rng.standard_normal((M, K)).astype(np.float32)
    W = (rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    gy = rng.standard_normal((M, N)).astype(np.float32)
    mask = np.where(rng.random((M, K)) < 0.4, 0.0, rng.random((M, K)) + 0.1).astype(np.float32)
    c0 = rng.standard_normal((M, K)).astype(np.float32)
    xt, Wt = _t(x, cuda), _t(W, cuda)
    y = F.gemm(xt, Wt, bias=_t(b, cuda), relu=True, precision=prec)
    out = _t(c0, cuda)
    dx = F.gemm(_t(gy, cuda), Wt, trans_b=True, mask=_t(mask, cuda), out=out, beta=0.5, precision=prec)
    torch.cuda.synchronize()
    x64, W64 = x.astype(np.float64), W.astype(np.float64)
    ref_y = np.maximum(x64 @ W64 + b, 0.0)
    ref_dx = np.where(mask > 0, gy.astype(np.float64) @ W64.T, 0.0) + 0.5 * c0
    # fp32-level: each product within 2^-23 of its magnitude (precision 6), fp32 accumulation
    assert_close(_n(y), ref_y, 1e-5, "y", floor=0.0)
    assert_close(_n(dx), ref_dx, 1e-5, "dx", floor=0.0)
    # a second call gives the same bits (no atomics, fixed order)
    y2 = F.gemm(xt, Wt, bias=_t(b, cuda), relu=True, precision=prec)
    assert torch.equal(y, y2)


# ---------------------------------------------------------------------------------------------
# weight-stationary split GEMM (gemm_ws.hip: the Dense layers' forward / dX when K, N are in
# {64, 128, 256} and the launch has >= 32768 rows, no addend / beta): against float64 at the split
# precision's bar, grouped launches bitwise their single launches, ragged row counts
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("G,M,K,N", [(2, 65536, 128, 256), (2, 65536, 256, 128), (2, 65536, 128, 64),
                                     (2, 65536, 64, 128), (1, 65536, 256, 256), (1, 40007, 128, 128),
                                     (2, 16411, 64, 64), (3, 33001, 256, 64), (4, 8200, 128, 256)])
def test_ws_gemm_forward_and_dx(cuda, prec, G, M, K, N):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(G * M + 7 * K + N + prec)
    xs = [rng.standard_normal((M, K)).astype(np.float32) for _ in range(G)]
    Ws = [(rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32) for _ in range(G)]
    bs = [rng.standard_normal(N).astype(np.float32) for _ in range(G)]
    gys = [rng.standard_normal((M, N)).astype(np.float32) for _ in range(G)]
    masks = [np.where(rng.random((M, K)) < 0.4, 0.0, rng.random((M, K)) + 0.1).astype(np.float32) for _ in range(G)]
    xt, Wt, bt = [_t(x, cuda) for x in xs], [_t(W, cuda) for W in Ws], [_t(b, cuda) for b in bs]
    gt, mt = [_t(g, cuda) for g in gys], [_t(m, cuda) for m in masks]
    ys = F.gemm_group(xt, Wt, bias=bt, relu=True, precision=prec)
    dxs = F.gemm_group(gt, Wt, trans_b=True, mask=mt, precision=prec)
    dxn = F.gemm_group(gt, Wt, trans_b=True, precision=prec)          # no mask (the input gradient)
    yl = F.gemm_group(xt, Wt, precision=prec)                         # linear, no bias (a top layer)
    torch.cuda.synchronize()
    for g in range(G):
        x64, W64, gy64 = xs[g].astype(np.float64), Ws[g].astype(np.float64), gys[g].astype(np.float64)
        assert_close(_n(ys[g]), np.maximum(x64 @ W64 + bs[g], 0.0), 1e-5, f"y {g}", floor=0.0)
        ref_dx = gy64 @ W64.T
        assert_close(_n(dxs[g]), np.where(masks[g] > 0, ref_dx, 0.0), 1e-5, f"dx {g}", floor=0.0)
        assert_close(_n(dxn[g]), ref_dx, 1e-5, f"dx unmasked {g}", floor=0.0)
        assert_close(_n(yl[g]), x64 @ W64, 1e-5, f"y linear {g}", floor=0.0)
    if G * M >= 32768 and M >= 32768:   # each problem alone also takes the kernel: same bits
        for g in range(G):
            assert torch.equal(ys[g], F.gemm(xt[g], Wt[g], bias=bt[g], relu=True, precision=prec)), g
            assert torch.equal(dxs[g], F.gemm(gt[g], Wt[g], trans_b=True, mask=mt[g], precision=prec)), g
    # a second call gives the same bits (no atomics, fixed order)
    assert torch.equal(ys[0], F.gemm_group(xt, Wt, bias=bt, relu=True, precision=prec)[0])


# ---------------------------------------------------------------------------------------------
# large-batch weight gradients (gemm_ws.hip wgrad_ws_kernel: dW + db when the batch has >= 8192
# rows and in, out are multiples of 64 with one a multiple of 128): against float64, grouped
# launches bitwise their single launches, the row-mapped form bitwise the expanded operand
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("G,K,M,N", [(2, 65536, 128, 256), (2, 65536, 256, 128), (2, 65536, 64, 128),
                                     (2, 65536, 128, 64), (1, 40007, 256, 256), (3, 8200, 128, 128),
                                     (2, 20011, 64, 256)])
def test_ws_wgrad(cuda, prec, G, K, M, N):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(G * K + 5 * M + N + prec)
    D = max(K // 7, 1)                  # distinct rows: batch row k reads row inv[k] of the table
    tabs = [rng.standard_normal((D, M)).astype(np.float32) for _ in range(G)]
    invs = [rng.integers(0, D, K).astype(np.int32) for _ in range(G)]
    xs = [t[i] for t, i in zip(tabs, invs)]
    gys = [rng.standard_normal((K, N)).astype(np.float32) for _ in range(G)]
    xt, gt = [_t(x, cuda) for x in xs], [_t(g, cuda) for g in gys]
    wg = F.gemm_wgrad_bias_group(xt, gt, prec)
    wr = F.gemm_wgrad_bias_group([_t(t, cuda) for t in tabs], gt, prec, x_rows=[_t(i, cuda) for i in invs])
    torch.cuda.synchronize()
    for g in range(G):
        x64, g64 = xs[g].astype(np.float64), gys[g].astype(np.float64)
        assert_close(_n(wg[g][0]), x64.T @ g64, 1e-5, f"dW {g}")
        assert_close(_n(wg[g][1]), g64.sum(0), 1e-5, f"db {g}")
        assert torch.equal(wr[g][0], wg[g][0]) and torch.equal(wr[g][1], wg[g][1]), g
        dW1, db1 = F.gemm_wgrad_bias(xt[g], gt[g], prec)
        assert torch.equal(dW1, wg[g][0]) and torch.equal(db1, wg[g][1]), g
    # a second call gives the same bits (no atomics, fixed order)
    assert torch.equal(wg[0][0], F.gemm_wgrad_bias_group(xt, gt, prec)[0][0])


@pytest.mark.parametrize("K", [8191, 8192, 8193, 12345])
@pytest.mark.parametrize("M,N", [(256, 64), (64, 256), (128, 128), (192, 128)])
def test_wgrad_envelope_edges(cuda, K, M, N):
    """Either side of the large-batch dW kernel's envelope (>= 8192 rows; in, out multiples of 64
    with one a multiple of 128): the split-K tile GEMM below it, the dW kernel at and above it with a
    ragged last slice, a 192-wide input (64-row tiles), all against float64 at the split bar; the
    single launch bitwise the grouped one and the l2 term folded in."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(K + 3 * M + N)
    xs = [rng.standard_normal((K, M)).astype(np.float32) for _ in range(2)]
    gs = [rng.standard_normal((K, N)).astype(np.float32) for _ in range(2)]
    xt, gt = [_t(x, cuda) for x in xs], [_t(g, cuda) for g in gs]
    wg = F.gemm_wgrad_bias_group(xt, gt, 6)
    W = rng.standard_normal((M, N)).astype(np.float32)
    sc = _t(np.array(0.5, dtype=np.float32), cuda)
    dW2, db2 = F.gemm_wgrad_bias(xt[0], gt[0], 6, W=_t(W, cuda), w_scale=2e-3, w_dscale=sc)
    torch.cuda.synchronize()
    for g in range(2):
        x64, g64 = xs[g].astype(np.float64), gs[g].astype(np.float64)
        assert_close(_n(wg[g][0]), x64.T @ g64, 1e-5, f"dW {g}")
        assert_close(_n(wg[g][1]), g64.sum(0), 1e-5, f"db {g}")
        dW1, db1 = F.gemm_wgrad_bias(xt[g], gt[g], 6)
        assert torch.equal(dW1, wg[g][0]) and torch.equal(db1, wg[g][1]), g
    assert_close(_n(dW2), xs[0].astype(np.float64).T @ gs[0].astype(np.float64) + 1e-3 * W, 1e-5, "dW + l2")
    assert torch.equal(db2, wg[0][1])


@pytest.mark.parametrize("ns", [[4096, 4096], [700, 0, 37, 2000, 129], [8192], [8193], [6000, 6000], [8193, 100]])
def test_sparse_adagrad_lds_sort(cuda, ns):
    """The one-workgroup LDS radix sort (n <= 8192 (table, id) keys below 2^32; several tables that
    each fit: one workgroup per table; a table of 8193 entries takes rocprim) against a float64
    restatement of the update (each table clipped by the norm of all its raw rows, invalid ids
    skipped, duplicates summed), on Zipf ids with heavy duplication, invalid ids and an empty table;
    and a second run bitwise the first. (The bitwise A/B against rocprim forced, RS_SORT_LDS=0, needs
    an -DRS_EXPERIMENTS build: the release library reads no switch.)"""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(sum(ns))
    D = 64
    V = [3000, 50, 7, 100000, 64][:len(ns)]
    ids = [(rng.zipf(1.2, n) % (v + 2) - 1).astype(np.int64) for v, n in zip(V, ns)]
    rows = [(rng.standard_normal((n, D)) * 0.05).astype(np.float32) for n in ns]
    tabs = [rng.standard_normal((v, D)).astype(np.float32) for v in V]
    it = torch.tensor(7, dtype=torch.int64, device=cuda)
    res = []
    for _ in range(2):
        tts = [_t(t, cuda) for t in tabs]
        tas = [torch.full((v, D), 0.1, device=cuda) for v in V]
        F.sparse_adagrad_multi(tts, tas, [_t(i, cuda) for i in ids], [_t(r, cuda) for r in rows], it, 0.05,
                               clipnorm=1.0)
        torch.cuda.synchronize()
        res.append([(t.cpu().numpy(), a.cpu().numpy()) for t, a in zip(tts, tas)])
    for k in range(len(ns)):
        assert np.array_equal(res[0][k][0], res[1][k][0]), k
        assert np.array_equal(res[0][k][1], res[1][k][1]), k
        P, A = tabs[k].astype(np.float64), np.full((V[k], D), 0.1)
        r64 = rows[k].astype(np.float64)
        nrm = np.sqrt((r64 ** 2).sum())
        g = r64 / max(nrm, 1.0)
        ok = (ids[k] >= 0) & (ids[k] < V[k])
        u, inv = np.unique(ids[k][ok], return_inverse=True)
        gs = np.zeros((len(u), D))
        np.add.at(gs, inv, g[ok])
        A[u] += gs * gs
        P[u] -= 0.05 * gs / np.sqrt(A[u] + 1e-7)
        assert_close(res[0][k][1], A, 1e-5, f"accumulator {k}")
        assert_close(res[0][k][0], P, 1e-5, f"table {k}")
