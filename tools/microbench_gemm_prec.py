"""Time the GEMM shapes of the c5 cross stack and the c3 towers at each contraction precision.
Usage: python tools/microbench_gemm_prec.py [precisions, e.g. 0,6,9]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")

precs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,6,9").split(",")]
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(0)
# (label, M, N, K, ta, tb, splitk)
SHAPES = [("c5 cross fwd NN", 16384, 3344, 3344, 0, 0, 0), ("c5 cross dX NT", 16384, 3344, 3344, 0, 1, 0),
          ("c5 cross dW TN splitk", 3344, 3344, 16384, 1, 0, 1), ("c5 deep fwd", 16384, 1024, 3344, 0, 0, 0),
          ("c3 tower fwd 128->256", 65536, 256, 128, 0, 0, 0), ("c3 tower dX 256->128", 65536, 128, 256, 0, 1, 0),
          ("c3 tower dW splitk", 128, 256, 65536, 1, 0, 1)]
ONLY = os.environ.get("SHAPES", "")   # label prefix filter, e.g. SHAPES=c5 (PMC passes)
BATCH = int(os.environ.get("C5_BATCH", "16384"))
SHAPES = [(lab, BATCH if (lab.startswith("c5") and M == 16384) else M, N,
           BATCH if (lab.startswith("c5") and K == 16384) else K, ta, tb, sk) for lab, M, N, K, ta, tb, sk in SHAPES]
for label, M, N, K, ta, tb, sk in SHAPES:
    if ONLY and not label.startswith(ONLY):
        continue
    A = torch.randn((K, M) if ta else (M, K), device=dev, generator=g)
    B = torch.randn((N, K) if tb else (K, N), device=dev, generator=g)
    ref = None
    line = f"{label:24s} M={M} N={N} K={K}:"
    for prec in precs:
        fn = (lambda: F.gemm_splitk(A, B, trans_a=bool(ta), trans_b=bool(tb), precision=prec)) if sk else \
             (lambda: F.gemm(A, B, trans_a=bool(ta), trans_b=bool(tb), precision=prec))
        out = fn()
        torch.cuda.synchronize()
        reps = 10
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        if ref is None:
            ref = out.double()
        err = (out.double() - ref).abs().max().item()
        line += f"  p{prec} {ms:.3f} ms {2.0 * M * N * K / ms / 1e9:.1f} TF/s (d vs p{precs[0]} {err:.1e})"
    print(line, flush=True)
