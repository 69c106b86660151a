"""Interleaved A/B of the xgemm variants (RS_XGEMM_VAR = 0..7, read per launch) on the c5 GEMM shapes.
Usage: python tools/ab_xgemm.py [B] [variants, e.g. 0,1,2,3]"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
VARS = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2,3,4,5,6,7").split(",")]
d, PEAK = 3344, 2500.0 / 6
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(0)
x = torch.randn(B, d, device=dev, generator=g) * 0.5
W = torch.randn(d, d, device=dev, generator=g) / d ** 0.5
gy = torch.randn(B, d, device=dev, generator=g)
xi, wti, gi, wi = F.xgemm_image(x), F.xgemm_image(W, True), F.xgemm_image(gy), F.xgemm_image(W)
xti, gti = F.xgemm_image(x, True), F.xgemm_image(gy, True)
cases = [("fwd", B, d, d, lambda: F.xgemm(xi, wti, B, d, d)), ("dX", B, d, d, lambda: F.xgemm(gi, wi, B, d, d)),
         ("dW", d, d, B, lambda: F.xgemm_splitk(xti, gti, d, d, B))]
refs = {}
for v in VARS:
    os.environ["RS_XGEMM_VAR"] = str(v)
    for lab, M, N, K, fn in cases:
        o = fn()
        torch.cuda.synchronize()
        if lab in refs:
            assert float((o - refs[lab]).abs().max()) == 0.0, (v, lab)
        else:
            refs[lab] = o
res = {}
rng = np.random.default_rng(0)
for rnd in range(4):
    for v in rng.permutation(VARS):
        os.environ["RS_XGEMM_VAR"] = str(v)
        for lab, M, N, K, fn in cases:
            fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                fn()
            e.record()
            torch.cuda.synchronize()
            res.setdefault((lab, int(v)), []).append(s.elapsed_time(e) / 5)
for lab, M, N, K, _ in cases:
    fl = 2.0 * M * N * K
    print(lab, "  ".join(f"v{v}: {np.median(res[(lab, v)]):.3f} ms ({fl / np.median(res[(lab, v)]) / 1e9 / PEAK:.1%})"
                         for v in VARS), flush=True)
