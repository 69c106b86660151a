"""The config-5 cross stack (d = 3,344, 4 layers) on the plane-image path vs the split-at-staging
path: forward, backward and the per-GEMM kernels are in the rocprof stats; this prints stack
times and the fp32-equivalent rate against the split peak (2500 / 6 TF/s).
Usage: [RS_PGEMM_BM=256] python tools/microbench_dcn2_planes.py [B] [d] [L]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
d = int(sys.argv[2]) if len(sys.argv) > 2 else 3344
L = int(sys.argv[3]) if len(sys.argv) > 3 else 4
PEAK = 2500.0 / 6
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(0)
x0 = torch.randn(B, d, device=dev, generator=g) * 0.1
W = torch.randn(L, d, d, device=dev, generator=g) / d ** 0.5
b = torch.randn(L, d, device=dev, generator=g) * 0.01
gy = torch.randn(B, d, device=dev, generator=g)


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        out = fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps, out


gf = 2.0 * B * d * d * L
print(f"B={B} d={d} L={L} RS_PGEMM_BM={os.environ.get('RS_PGEMM_BM', '128')}", flush=True)
for name, fwd, bwd in (
        ("split-at-staging", lambda: F.dcn_cross_mat_fwd(x0, W, b, precision=6),
         lambda o: F.dcn_cross_mat_bwd(x0, o[0], o[1], W, gy, precision=6)),
        ("plane images", lambda: F.dcn_cross_mat_fwd_planes(x0, W, b, precision=6),
         lambda o: F.dcn_cross_mat_bwd_planes(x0, o[0], o[1], W, o[2], gy, precision=6))):
    tf, o = timed(fwd)
    tb, _ = timed(lambda: bwd(o))
    print(f"  {name:18s} fwd {tf:7.3f} ms ({gf / tf / 1e9 / PEAK:.1%})  bwd {tb:7.3f} ms ({2 * gf / tb / 1e9 / PEAK:.1%})"
          f"  stack {tf + tb:7.3f} ms ({3 * gf / (tf + tb) / 1e9 / PEAK:.1%} of the split peak)", flush=True)
