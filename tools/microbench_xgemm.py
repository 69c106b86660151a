"""The plane-pair GEMM (rs_xgemm_*) against the split-at-staging GEMM (rs_gemm_prec_f32 /
rs_gemm_splitk_prec_f32) on the c5 cross-stack shapes (B x 3344 x 3344 fwd, dX, dW) and the deep
layer, precision 6: checks the results against each other (both are fp32-level: max rel. diff is
printed) and times GEMM alone and image builds, interleaved over rounds in one process.
Usage: python tools/microbench_xgemm.py [B]"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
d = 3344
PEAK = 2500.0 / 6
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(0)
x = torch.randn(B, d, device=dev, generator=g) * 0.5
W = torch.randn(d, d, device=dev, generator=g) / d ** 0.5
gy = torch.randn(B, d, device=dev, generator=g)
Wd = torch.randn(d, 1024, device=dev, generator=g) / d ** 0.5


def ev_time(fn, reps=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


# images: fwd A = x [B][d], B = W^T (W stored [k][n] -> rows n: trans); dX: A = gy, B = W (rows k', contraction n);
# dW: A = x^T (rows k, contraction m: trans), B = gy^T (trans)
imgs = {}
cases = [
    ("fwd x W", B, d, d, lambda: F.gemm(x, W, precision=6),
     lambda: F.xgemm(imgs["x"], imgs["Wt"], B, d, d), [("x", x, False), ("Wt", W, True)]),
    ("dX g W^T", B, d, d, lambda: F.gemm(gy, W, trans_b=True, precision=6),
     lambda: F.xgemm(imgs["g"], imgs["W"], B, d, d), [("g", gy, False), ("W", W, False)]),
    ("dW x^T g", d, d, B, lambda: F.gemm_splitk(x, gy, trans_a=True, precision=6),
     lambda: F.xgemm_splitk(imgs["xT"], imgs["gT"], d, d, B), [("xT", x, True), ("gT", gy, True)]),
    ("deep x Wd", B, 1024, d, lambda: F.gemm(x, Wd, precision=6),
     lambda: F.xgemm(imgs["x"], imgs["Wdt"], B, 1024, d), [("x", x, False), ("Wdt", Wd, True)]),
]
for _, _, _, _, _, _, need in cases:
    for name, t, tr in need:
        imgs[name] = F.xgemm_image(t, tr)
torch.cuda.synchronize()
res = {}
for label, M, N, K, ref_fn, new_fn, need in cases:
    r = ref_fn()
    o = new_fn()
    torch.cuda.synchronize()
    err = float(((o - r).abs().max() / r.abs().max()).item())
    print(f"{label:10s} M={M} N={N} K={K}: max |xgemm - split GEMM| / max|C| = {err:.2e}", flush=True)
    assert err < 1e-5, label
for rnd in range(3):
    for label, M, N, K, ref_fn, new_fn, need in cases:
        res.setdefault((label, "split GEMM"), []).append(ev_time(ref_fn))
        res.setdefault((label, "xgemm"), []).append(ev_time(new_fn))
        res.setdefault((label, "images"), []).append(
            ev_time(lambda: [F.xgemm_image(t, tr) for _, t, tr in need]))
for label, M, N, K, _, _, _ in cases:
    fl = 2.0 * M * N * K
    line = f"{label:10s}"
    for kind in ("split GEMM", "xgemm", "images"):
        ms = float(np.median(res[(label, kind)]))
        line += f"  {kind} {ms:7.3f} ms" + (f" ({fl / ms / 1e9 / PEAK:.1%})" if kind != "images" else "")
    print(line, flush=True)
