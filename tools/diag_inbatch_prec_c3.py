"""Diagnostic (round 5): the in-batch pair's column-sum errors at C3 (B = 65536, bench.py's first
Zipf(1.05) batch over 10M users / 1M items, tower-like rows: one row per distinct id, a common
per-column offset of 0.05 plus N(0, 0.03) noise, so the columns keep one sign as a tower output's
bias makes them) against float64 (torch fp64 on the GPU, in row chunks): the deduplicated pair (the
C3 step's default, running MFMA accumulation in its WK kernels) and the full pair (fresh per-tile
accumulators). colsum(dU), colsum(dC) are what the tower-top bias gradients sum.
Usage: python tools/diag_inbatch_prec_c3.py"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
from bench import zipf_ids  # noqa: E402

B, D, PREC = 65536, 128, 6
dev = torch.device("cuda")
rng = np.random.default_rng(1234)
uid = torch.from_numpy(zipf_ids(rng, B, 10_000_000)).to(dev)
iid = torch.from_numpy(zipf_ids(rng, B, 1_000_000)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(5)


def rows(ids, off):
    uniq, inv = torch.unique(ids, return_inverse=True)
    r = off + torch.randn((uniq.numel(), D), device=dev, generator=g) * 0.03
    return r[inv].contiguous()


U = rows(uid, 0.05 * torch.sign(torch.randn(D, device=dev, generator=g)))
C = rows(iid, 0.05 * torch.sign(torch.randn(D, device=dev, generator=g)))
U64, C64 = U.double(), C.double()
lse = torch.empty(B, dtype=torch.float64, device=dev)
for r0 in range(0, B, 4096):
    lse[r0:r0 + 4096] = torch.logsumexp(U64[r0:r0 + 4096] @ C64.T, dim=1)
dU_ref = torch.zeros((B, D), dtype=torch.float64, device=dev)
cs_dC = torch.zeros(D, dtype=torch.float64, device=dev)
for r0 in range(0, B, 4096):
    P = torch.exp(U64[r0:r0 + 4096] @ C64.T - lse[r0:r0 + 4096, None])
    dU_ref[r0:r0 + 4096] = P @ C64 - C64[r0:r0 + 4096]
    cs_dC += P.sum(0) @ C64 * 0   # placeholder keeps shapes; dC column sums below
# colsum(dC) = sum_j (sum_i P_ij U_i - U_j) = sum_i U_i (sum_j P_ij) - sum_j U_j
rowsumP = torch.zeros(B, dtype=torch.float64, device=dev)
for r0 in range(0, B, 4096):
    rowsumP[r0:r0 + 4096] = torch.exp(U64[r0:r0 + 4096] @ C64.T - lse[r0:r0 + 4096, None]).sum(1)
cs_dC = (U64 * rowsumP[:, None]).sum(0) - U64.sum(0)
cs_dU = dU_ref.sum(0)
scale = float(dU_ref.abs().sum(0).max())
print(f"|colsum dU| ref {cs_dU.abs().max():.3e}, |colsum dC| ref {cs_dC.abs().max():.3e}; "
      f"sum_rows |dU| per column up to {scale:.3e}", flush=True)
gs = torch.ones((), device=dev)
for name in ("dedup", "full"):
    S = F.inbatch_scores_buffer(B, dev)
    if name == "dedup":
        users, items = F.inbatch_dedup_plan(U, C, PREC, ids=(uid, iid, 10_000_001, 1_000_001))
        _, _, lg, dU1, _ = F.inbatch_softmax_fwd_dedup(U, C, users, items, S, PREC)
        dU, dC = F.inbatch_softmax_bwd_dedup(U, lg, users, items, S, PREC, gscale=gs, dU_unit=dU1)
    else:
        _, _, lg, dU1, _ = F.inbatch_softmax_fwd(U, C, scores=S, precision=PREC)
        dU, dC = F.inbatch_softmax_bwd(U, C, lg, gscale=gs, dU_unit=dU1, scores=S, precision=PREC)
    torch.cuda.synchronize()
    eu = float((dU.double().sum(0) - cs_dU).abs().max())
    ec = float((dC.double().sum(0) - cs_dC).abs().max())
    emax = float((dU.double() - dU_ref).abs().max())
    print(f"{name:6s}: colsum err dU {eu:.3e} dC {ec:.3e} (relative to the column's sum of |dU|: "
          f"{eu / scale:.2e}, {ec / scale:.2e}); max |dU - ref| {emax:.3e}", flush=True)
    del S
    torch.cuda.empty_cache()
