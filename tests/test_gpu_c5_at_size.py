"""Config 5 (DCN-v2 ranker) at the batches bench.py times: the plane-image cross
stack (rs_dcn_cross_mat_fwd/bwd_planes_f32: xgemm images, split-K dW over the batch) at
B = 16384 and B = 65536 with d = 3344 (26 x 128 + 13, padded), L = 4, and one DCNv2Ranker loss and
gradient step at B = 16384 with the 3 x 1024 deep tower, all against float64.

Truth:
* B = 16384: the oracle's own cross_matrix_forward / _backward and dcn2_ranker_loss_and_grads
  (numpy float64, every row).
* B = 65536: x_L and dL/dx0 are row-wise functions of (x0, g), so the oracle run on a sample of
  rows (first, last, random) gives their exact float64 values; dW_l = x_l^T t_l and db_l = sum t_l
  sum over all 65,536 rows, so they are checked against a host float64 GEMM of the GPU's own x_l
  (fp32 outputs of the forward, themselves checked) with the float64 gradient chain
  t_l = g_{l+1} * x0, g_l = t_l W_l^T + g_{l+1} (the oracle's backward, restated in torch float64 on
  the host; pinned to the oracle on the sampled rows first).

Bar: 1e-4 of each tensor's max magnitude (north_star's fp32 bar), as the smaller-size tests."""
import numpy as np
import pytest

from conftest import assert_close, oracle, pkg

pytestmark = pytest.mark.gpu

D_C5, L_C5 = 3344, 4


def _t(x, dev):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(x))
    if t.dtype == torch.float64:
        t = t.float()
    return t.to(dev)


def _n(t):
    return t.detach().double().cpu().numpy()


def _host_threads():
    import os
    import torch
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))


def _inputs(B, d, L, seed):
    """Cross-stack operands at the model's scale: x0 ~ N(0, 0.5^2), W ~ N(0, 1/d) per layer (so
    x_l stays O(1) through L layers), b ~ N(0, 0.1^2), an upstream gradient g and the deep tower's
    extra dL/dx0 term."""
    rng = np.random.default_rng(seed)
    x0 = (rng.standard_normal((B, d), dtype=np.float32) * 0.5)
    W = (rng.standard_normal((L, d, d), dtype=np.float32) / np.float32(np.sqrt(d)))
    b = (rng.standard_normal((L, d), dtype=np.float32) * 0.1)
    g = rng.standard_normal((B, d), dtype=np.float32)
    extra = rng.standard_normal((B, d), dtype=np.float32)
    return x0, W, b, g, extra


def _gpu_planes(cuda, x0, W, b, g, extra):
    import torch
    F = pkg("functional")
    tx0, tW, tb, tg, te = (_t(v, cuda) for v in (x0, W, b, g, extra))
    XS, US, ximg = F.dcn_cross_mat_fwd_planes(tx0, tW, tb, precision=6)
    GX0, GW, GB = F.dcn_cross_mat_bwd_planes(tx0, XS, US, tW, ximg, tg, te, precision=6)
    torch.cuda.synchronize()
    return XS, GX0, GW, GB


def test_cross_matrix_planes_b16384_against_oracle(cuda):
    """B = 16384 (bench.py --config c5): x_L, dL/dx0, dW and db of the plane path against the
    oracle's float64 cross stack over every row."""
    _host_threads()
    O = oracle()
    B, d, L = 16384, D_C5, L_C5
    x0, W, b, g, extra = _inputs(B, d, L, 16384)
    XS, GX0, GW, GB = _gpu_planes(cuda, x0, W, b, g, extra)
    x64, W64, b64 = x0.astype(np.float64), W.astype(np.float64), b.astype(np.float64)
    xL, xs = O.cross_matrix_forward(x64, W64, b64)
    assert_close(_n(XS[L - 1]), xL, 1e-4, "x_L", floor=0.0)
    for l in range(1, L):
        assert_close(_n(XS[l - 1]), xs[l], 1e-4, f"x_{l}", floor=0.0)
    gx0, gW, gb = O.cross_matrix_backward(x64, xs, W64, b64, g.astype(np.float64))
    del xs
    assert_close(_n(GX0), gx0 + extra, 1e-4, "g_x0", floor=0.0)
    for l in range(L):
        assert_close(_n(GW[l]), gW[l], 1e-4, f"g_W[{l}]", floor=0.0)
        assert_close(_n(GB[l]), gb[l], 1e-4, f"g_b[{l}]", floor=0.0)


def _sample_rows(B, n, seed):
    rng = np.random.default_rng(seed)
    mid = rng.choice(np.arange(1, B - 1), size=n - 2, replace=False)
    return np.unique(np.concatenate([[0, B - 1], mid]))


def _grad_chain_f64(x0, W, g):
    """The oracle's cross backward chain (recsys_oracle.cross_matrix_backward) without the forward
    terms, in torch float64 on the host: t_l = g_{l+1} * x0 and g_l = t_l W_l^T + g_{l+1} for
    l = L-1 .. 0; yields (l, t_l) from the top layer down."""
    import torch
    gg = g
    for l in range(W.shape[0] - 1, -1, -1):
        t = gg * x0
        yield l, t
        gg = torch.addmm(gg, t, W[l].T)


def test_cross_matrix_planes_b65536_sampled_rows_and_full_dw(cuda):
    """B = 65536 (north_star's batch, bench.py's c5_b65536): x_L and dL/dx0 on 64 sampled rows
    (incl. the first and last) against the oracle run on those rows; dW and db over all rows
    against a host float64 GEMM of the GPU's own x_l with the float64 gradient chain."""
    import torch
    _host_threads()
    O = oracle()
    B, d, L = 65536, D_C5, L_C5
    x0, W, b, g, extra = _inputs(B, d, L, 65536)
    XS, GX0, GW, GB = _gpu_planes(cuda, x0, W, b, g, extra)
    rows = _sample_rows(B, 64, 7)
    W64, b64 = W.astype(np.float64), b.astype(np.float64)
    xr = x0[rows].astype(np.float64)
    xL_r, xs_r = O.cross_matrix_forward(xr, W64, b64)
    it = torch.from_numpy(rows).to(cuda)
    assert_close(_n(XS[L - 1].index_select(0, it)), xL_r, 1e-4, "x_L rows", floor=0.0)
    gx0_r, gW_r, gb_r = O.cross_matrix_backward(xr, xs_r, W64, b64, g[rows].astype(np.float64))
    assert_close(_n(GX0.index_select(0, it)), gx0_r + extra[rows], 1e-4, "g_x0 rows", floor=0.0)
    # the torch float64 chain reproduces the oracle's dW / db on the sampled rows (pins the restatement)
    tx_r = [torch.from_numpy(a) for a in xs_r]
    tW = torch.from_numpy(W64)
    for l, t in _grad_chain_f64(torch.from_numpy(xr), tW, torch.from_numpy(g[rows].astype(np.float64))):
        assert_close((tx_r[l].T @ t).numpy(), gW_r[l], 1e-12, f"chain g_W[{l}] (sampled rows)", floor=0.0)
        assert_close(t.sum(0).numpy(), gb_r[l], 1e-12, f"chain g_b[{l}] (sampled rows)", floor=0.0)
    # every row: dW_l = x_l^T t_l with the GPU's own x_l (x_0 = the input), the chain in float64
    x0_64 = torch.from_numpy(x0).double()
    for l, t in _grad_chain_f64(x0_64, tW, torch.from_numpy(g).double()):
        xl = x0_64 if l == 0 else XS[l - 1].cpu().double()
        assert_close(_n(GW[l]), (xl.T @ t).numpy(), 1e-4, f"g_W[{l}]", floor=0.0)
        assert_close(_n(GB[l]), t.sum(0).numpy(), 1e-4, f"g_b[{l}]", floor=0.0)
        del xl


def test_dcn2_ranker_b16384_step_against_oracle(cuda):
    """One DCNv2Ranker loss + gradient step at bench.py's c5 batch (B = 16384; 26 tables x 128,
    13 dense features, d = 3344, 4 cross layers, 3 x 1024 deep tower, precision 6: the trunk node
    on the plane-pair GEMM) against oracle.dcn2_ranker_loss_and_grads in float64, under the GPU
    forward's ReLU gates (every gate that differs from the float64 sign sits within fp32 rounding
    of zero, asserted), every table's gradient rows and every dense gradient at 1e-4."""
    import torch
    _host_threads()
    models, F = pkg("models"), pkg("functional")
    O = oracle()
    nf, E, nd, L, B = 26, 128, 13, L_C5, 16384
    deep = [1024, 1024, 1024]
    vocab = [4093 + 17 * f for f in range(nf)]
    m = models.DCNv2Ranker(vocab, embedding_dim=E, num_dense=nd, cross_layers=L, deep_layers=deep, device=cuda,
                           precision=6, seed=16)
    d = m.d
    assert d == D_C5 and m.d_raw == 3341
    with torch.no_grad():                      # small live biases, a head that keeps p off 0 / 1
        gen = torch.Generator(device="cpu").manual_seed(17)
        m.cross_b.copy_((torch.rand(m.cross_b.shape, generator=gen) - 0.5) * 0.02)
        m.cross_b[:, m.d_raw:] = 0
        m.ctr_head.kernel.mul_(4.0)
    P = {k: v.detach().double().cpu().numpy() for k, v in m.state_dict().items()}
    rng = np.random.default_rng(1616)
    ids = np.stack([rng.integers(0, v + 1, B) for v in vocab]).astype(np.int64)
    dense = rng.standard_normal((B, nd)).astype(np.float32)
    y = (rng.random(B) < 0.3).astype(np.float32)
    with F.record_relu_gates() as rec:
        loss = m.compute_loss(_t(ids, cuda), _t(dense, cuda), _t(y, cuda))
        loss.backward()
    torch.cuda.synchronize()
    key = m.deep_nets[0].kernel.data_ptr()
    assert key in rec["fwd"], "the trunk node did not record its gates"
    masks = [gt.cpu().numpy() for gt in rec["fwd"][key]]
    assert len(masks) == len(deep)
    ref = O.dcn2_ranker_loss_and_grads(P, nf, E, d, deep, ids, dense.astype(np.float64), y.astype(np.float64),
                                       masks=masks)
    # gates against the float64 signs: a disagreement must be a rounding-size pre-activation
    flips = 0
    for j, mk in enumerate(masks):
        a = ref["acts"][j]
        Wj, bj = P[f"deep_nets.{j}.kernel"], P[f"deep_nets.{j}.bias"]
        pre = a @ Wj + bj
        flip = (pre > 0) != mk
        if flip.any():
            scale = np.abs(a) @ np.abs(Wj) + np.abs(bj)
            assert float(np.max(np.abs(pre[flip]) / scale[flip])) <= 1e-5, f"deep layer {j}: a gate flip past rounding"
            flips += int(flip.sum())
    print(f"C5 B={B}: {flips} deep-tower gates differ from the float64 sign (all within rounding)")
    assert abs(float(loss) - ref["loss"]) <= 1e-4 * max(1.0, abs(ref["loss"])), (float(loss), ref["loss"])
    named = dict(m.named_parameters())
    for k, gr in ref["grads"].items():
        if isinstance(gr, tuple):
            f = int(k.split(".")[1])
            gi, grow = m.tables[f].sink.gathered()
            assert np.array_equal(gi.cpu().numpy(), gr[0]), k
            assert_close(_n(grow), gr[1], 1e-4, k, floor=0.0)
        else:
            assert_close(_n(named[k].grad).reshape(gr.shape), gr, 1e-4, k, floor=0.0)
    gW = named["cross_W"].grad
    assert float(gW[:, m.d_raw:, :].abs().max()) == 0.0 and float(gW[:, :, m.d_raw:].abs().max()) == 0.0
