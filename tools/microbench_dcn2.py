"""Time the DCN-v2 matrix cross stack alone (config 5: d = 3,344, 4 layers) and its three GEMM
shapes, with a float64 spot check of one layer. Usage:
    python tools/microbench_dcn2.py [B] [d] [L]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
d = int(sys.argv[2]) if len(sys.argv) > 2 else 3344
L = int(sys.argv[3]) if len(sys.argv) > 3 else 4
PEAK = 157.3
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


def rep(name, ms, flops):
    tf = flops / ms / 1e9
    print(f"  {name:34s} {ms:8.3f} ms  {tf:7.1f} TF/s  ({tf / PEAK:.1%} of fp32 MFMA peak)", flush=True)


print(f"B={B} d={d} L={L}", flush=True)
gf = 2.0 * B * d * d
tf_, (xs, us) = timed(lambda: F.dcn_cross_mat_fwd(x0, W, b))
rep("cross stack fwd", tf_, gf * L)
tb_, (gx0, gW, gb) = timed(lambda: F.dcn_cross_mat_bwd(x0, xs, us, W, gy))
rep("cross stack bwd", tb_, 2 * gf * L)
rep("cross stack fwd+bwd", tf_ + tb_, 3 * gf * L)
ms, _ = timed(lambda: F.gemm(x0, W[0]))
rep("GEMM NN  [B,d]x[d,d]", ms, gf)
ms, _ = timed(lambda: F.gemm(x0, W[0], trans_b=True))
rep("GEMM NT  [B,d]x[d,d]^T", ms, gf)
ms, _ = timed(lambda: F.gemm_splitk(x0, gy))
rep("GEMM TN split-K [B,d]^T x [B,d]", ms, gf)

# float64 spot check of layer 0 on the first 256 rows and of dW_{L-1} on a 64x64 corner
n = 256
u_ref = x0[:n].double() @ W[0].double() + b[0].double()
x1_ref = x0[:n].double() * u_ref + x0[:n].double()
print("x1 max err", (xs[0, :n].double() - x1_ref).abs().max().item(),
      "rel", ((xs[0, :n].double() - x1_ref).norm() / x1_ref.norm()).item())
xin = xs[L - 2] if L >= 2 else x0
t = gy.double() * x0.double()
gW_ref = xin[:, :64].double().T @ t[:, :64]
print("gW corner rel err", ((gW[L - 1, :64, :64].double() - gW_ref).norm() / gW_ref.norm()).item())
