"""Selection statistics of an instrumented top-k build (tools/build_topk_variants.sh
"stats:-DRS_TOPK_EXP_STATS"): compactions, cycles inside compaction vs total scan cycles, appends.
Usage: RECSYS_HIP_LIB=tools/_exp_topk_stats.so python tools/topk_stats.py [N] [k] [Q,...]"""
import ctypes
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
lib = ctypes.CDLL(os.environ["RECSYS_HIP_LIB"])
N = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 100
Qs = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 16, 64, 1024]
PREC = int(os.environ.get("PREC", "0"))
GAUSS = os.environ.get("GAUSS", "0") == "1"
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(7)
items = (torch.randint(-8, 8, (N, 128), device=dev, generator=g).float() / 8).contiguous()
if GAUSS:
    items = torch.randn(N, 128, device=dev, generator=g)
buf = (ctypes.c_ulonglong * 8)()
for Q in Qs:
    q = (torch.randint(-8, 8, (Q, 128), device=dev, generator=g).float() / 8).contiguous()
    if GAUSS:
        q = torch.randn(Q, 128, device=dev, generator=g)
    F.topk_ip(q, items, k, precision=PREC)
    torch.cuda.synchronize()
    lib.rs_topk_debug_stats(buf, 1)
    F.topk_ip(q, items, k, precision=PREC)
    torch.cuda.synchronize()
    lib.rs_topk_debug_stats(buf, 1)
    nc, cc, ap, sc, nw = list(buf)[:5]
    print(f"Q={Q}: waves={nw} compactions={nc} ({nc / max(nw, 1):.1f}/wave) appends={ap} "
          f"cycles/compaction={cc / max(nc, 1):.0f} compaction share of scan cycles={cc / max(sc, 1):.1%} "
          f"scan cycles/wave={sc / max(nw, 1):.3g}", flush=True)
