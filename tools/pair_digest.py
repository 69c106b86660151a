"""Bitwise digest of the deduplicated in-batch pair's outputs at the C3 shape (B = 65536, D = 128,
precision 6, Zipf(1.05) ids over 10M users / 1M items, tower rows equal per id; the same seeds as
tools/microbench_inbatch_dedup.py): total loss, per-row loss, lse, dU and dC as fp32 bit-pattern
sums, one line each, so that two library builds (RECSYS_HIP_LIB) can be compared with diff.
Usage: python tools/pair_digest.py"""
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
g = torch.Generator(device=dev)
g.manual_seed(5)


def tower_rows(vocab):
    ids = torch.from_numpy(zipf_ids(rng, B, vocab)).to(dev)
    uniq, inv = torch.unique(ids, return_inverse=True)
    rows = torch.randn((uniq.numel(), D), device=dev, generator=g) * 0.3
    return rows[inv].contiguous()


U = tower_rows(10_000_000)
C = tower_rows(1_000_000)
scores = F.inbatch_scores_buffer(B, dev)
users, items = F.inbatch_dedup_plan(U, C, PREC, force=True)
gs = torch.ones((), device=dev)
tot, row, lse, dU, _ = F.inbatch_softmax_fwd_dedup(U, C, users, items, scores, PREC)
out = F.inbatch_softmax_bwd_dedup(U, lse, users, items, scores, PREC, gscale=gs, dU_unit=dU)
dC = out[1] if isinstance(out, (tuple, list)) else out
torch.cuda.synchronize()


def digest(t):
    b = t.detach().reshape(-1).contiguous().view(torch.int32).to(torch.int64)
    return f"{int(b.sum())} {int((b * torch.arange(1, b.numel() + 1, device=b.device)).sum())}"


for name, t in (("loss", tot), ("row_loss", row), ("lse", lse), ("dU", dU), ("dC", dC)):
    print(name, tuple(t.shape), digest(t), flush=True)
