"""Time rs_relu_bwd_colsum_f32 (ReLU backward mask + ordered column sums) on the C3 Dense-layer
shapes. Usage: python tools/microbench_colsum.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(0)
for M, N in [(65536, 256), (65536, 128), (65536, 64), (16384, 3344), (4096, 256)]:
    dy = torch.randn(M, N, device=dev, generator=g)
    y = torch.randn(M, N, device=dev, generator=g)
    for _ in range(3):
        gg, cs = F.relu_bwd_colsum(dy, y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        gg, cs = F.relu_bwd_colsum(dy, y)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    ref = torch.where(y > 0, dy, torch.zeros_like(dy))
    ok = torch.equal(gg, ref) and torch.allclose(cs.double(), ref.double().sum(0), rtol=1e-5, atol=1e-3)
    byts = 3 * M * N * 4
    print(f"M={M} N={N}: {us:7.1f} us  {byts / us / 1e3:6.0f} GB/s  ok={ok}", flush=True)
