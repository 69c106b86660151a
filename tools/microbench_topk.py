"""Time the exact inner-product top-k (rs_topk_ip_f32: scan + merge) over one C4 shard
(12.5M x 128 fp32 = 6.4 GB, the per-GPU share of 100M items at 8 GPUs) at Q in {1, 64, 1024},
k = 100, with an exactness check on a dyadic grid. Usage:
    python tools/microbench_topk.py [N] [k] [Q,...]
(env: PREC scan precision, GAUSS=1 Gaussian rows, ORDER=norm the bound-first scan's worst order)"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 100
Qs = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 64, 1024]
PREC = int(os.environ.get("PREC", "0"))   # scan contraction precision (0 = f32 MFMA, 6 / 9 split)
D = 128
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(7)
# dyadic grid: multiples of 1/8 in [-1, 1) -> every fp32 dot product of length 128 is exact
GAUSS = os.environ.get("GAUSS", "0") == "1"  # Gaussian data (few ties; the exactness check then uses fp32-rounded scores)
items = (torch.randint(-8, 8, (N, D), device=dev, generator=g).float() / 8).contiguous()
if GAUSS:
    items = torch.randn(N, D, device=dev, generator=g)
# ORDER=norm: the bound-first scan's adversarial order (row norms rising linearly from 0.01 to 1 down
# the table: every later range beats the earlier ranges' k-th score for thousands of its rows, the
# candidate slots overflow and the call reruns as the list scan)
if os.environ.get("ORDER") == "norm":
    items *= torch.linspace(0.01, 1.0, N, device=dev)[:, None]
for Q in Qs:
    q = (torch.randint(-8, 8, (Q, D), device=dev, generator=g).float() / 8).contiguous()
    if GAUSS:
        q = torch.randn(Q, D, device=dev, generator=g)
    F.topk_ip(q, items, k, precision=PREC)
    torch.cuda.synchronize()
    reps = 5 if Q <= 64 else 2
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        sc, ix = F.topk_ip(q, items, k, precision=PREC)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    byts = N * D * 4 + Q * D * 4
    fl = 2.0 * Q * N * D
    print(f"Q={Q:5d} N={N} k={k}: {ms:9.3f} ms  {byts / ms / 1e6:7.1f} GB/s ({byts / ms / 1e6 / 8000:.1%} of 8 TB/s)  "
          f"{fl / ms / 1e9:6.1f} TF/s ({fl / ms / 1e9 / 157.3:.1%} of fp32 MFMA)  "
          f"{Q * N / ms / 1e6:.3g} G dots/s", flush=True)
    # exactness on the first 16 queries: float64 scores (exact on the grid), stable (-score, index)
    nchk = min(Q, 16)
    S = q[:nchk].double() @ items.double().T
    order = torch.sort(-S, dim=1, stable=True).indices[:, :k]
    ok = torch.equal(order, ix[:nchk]) and torch.equal(S.gather(1, order).float(), sc[:nchk])
    print(f"   exact top-{k} indices+scores match float64 reference on {nchk} queries: {ok}", flush=True)
    del S, order
