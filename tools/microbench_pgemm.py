"""The config-5 cross-stack GEMM shapes on the split GEMM (fp32 operands split at staging,
gemm_x3_kernel) vs the plane-image GEMM (pre-split operands streamed by LDS-DMA, pgemm_kernel),
plus the image builds. TF/s = fp32-equivalent 2 M N K / t. Usage: python tools/microbench_pgemm.py [B] [d]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
d = int(sys.argv[2]) if len(sys.argv) > 2 else 3344
PEAK = 2500.0 / 6
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(0)
x = torch.randn(B, d, device=dev, generator=g) * 0.1
t = torch.randn(B, d, device=dev, generator=g)
W = torch.randn(d, d, device=dev, generator=g) / d ** 0.5


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        out = fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps, out


def rep(name, ms, flops=None):
    if flops:
        tf = flops / ms / 1e9
        print(f"  {name:44s} {ms:8.3f} ms  {tf:7.1f} TF/s  ({tf / PEAK:.1%} of the split peak)", flush=True)
    else:
        print(f"  {name:44s} {ms:8.3f} ms", flush=True)


gf = 2.0 * B * d * d
print(f"B={B} d={d}", flush=True)
ms, xkc = timed(lambda: F.plane_image(x, F.PLANE_KC))
rep("image KC(x) [B,d]", ms)
ms, xkm = timed(lambda: F.plane_image(x, F.PLANE_KM))
rep("image KM(x) [B,d]", ms)
ms, wkm = timed(lambda: F.plane_image(W, F.PLANE_KM))
rep("image KM(W) [d,d]", ms)
wkc = F.plane_image(W, F.PLANE_KC)
tkc = F.plane_image(t, F.PLANE_KC)
tkm = F.plane_image(t, F.PLANE_KM)
ms, r0 = timed(lambda: F.gemm(x, W, precision=6))
rep("x3 NN  x W", ms, gf)
ms, r1 = timed(lambda: F.gemm_planes(xkc, wkm, B, d, d, precision=6))
rep("planes NN  x W", ms, gf)
print("    bitwise equal:", bool(torch.equal(r0, r1)), flush=True)
ms, r0 = timed(lambda: F.gemm(t, W, trans_b=True, precision=6))
rep("x3 NT  t W^T", ms, gf)
ms, r1 = timed(lambda: F.gemm_planes(tkc, wkc, B, d, d, trans_b=True, precision=6))
rep("planes NT  t W^T", ms, gf)
print("    bitwise equal:", bool(torch.equal(r0, r1)), flush=True)
ms, r0 = timed(lambda: F.gemm_splitk(x, t, trans_a=True, precision=6))
rep("x3 TN split-K  x^T t", ms, gf)
ms, r1 = timed(lambda: F.gemm_planes_splitk(xkm, tkm, d, d, B, True, False, precision=6))
rep("planes TN split-K  x^T t", ms, gf)
print("    max |diff| / max |ref|:", float((r0 - r1).abs().max() / r0.abs().max()), flush=True)
