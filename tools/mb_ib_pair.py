"""Microbenchmark of the deduplicated in-batch pair at the C3 shape (bench.py's first C3 batch:
B = 65536, Zipf(1.05) ids over 10M users / 1M items, tower rows equal per id, precision 6): N
forward (row pass) and N backward (col pass) launches, each bracketed by HIP events on the launch
stream; prints the median and min per entry point. Usage: python tools/mb_ib_pair.py [N] [tag]"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
from bench import zipf_ids  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
tag = sys.argv[2] if len(sys.argv) > 2 else ""
B, D, PREC = 65536, 128, 6
dev = torch.device("cuda")
rng = np.random.default_rng(1234)
uid = torch.from_numpy(zipf_ids(rng, B, 10_000_000)).to(dev)
iid = torch.from_numpy(zipf_ids(rng, B, 1_000_000)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(5)


def rows(ids):
    uniq, inv = torch.unique(ids, return_inverse=True)
    return (torch.randn((uniq.numel(), D), device=dev, generator=g) * 0.3)[inv].contiguous()


U, C = rows(uid), rows(iid)
scores = F.inbatch_scores_buffer(B, dev)
users, items = F.inbatch_dedup_plan(U, C, PREC, ids=(uid, iid, 10_000_001, 1_000_001), device_counts=True)
ws = F.inbatch_workspace(B, D, dev, dedup=True)
gs = torch.ones((), device=dev)
fw, bw = [], []
for i in range(N + 2):
    a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    torch.cuda._sleep(200000)   # a GPU pre-roll: the host's launch work is not in the brackets
    a.record()
    tot, row, lse, dU, _ = F.inbatch_softmax_fwd_dedup(U, C, users, items, scores, PREC, workspace=ws)
    b.record()
    F.inbatch_softmax_bwd_dedup(U, lse, users, items, scores, PREC, gscale=gs, dU_unit=dU, workspace=ws)
    c.record()
    torch.cuda.synchronize()
    if i >= 2:
        fw.append(a.elapsed_time(b))
        bw.append(b.elapsed_time(c))
nu, nc = int(users[4][0]), int(items[4][2])
pairs = nu * nc
print(f"{tag:20s} row {np.median(fw):.4f} ms (min {min(fw):.4f})  col {np.median(bw):.4f} ms (min {min(bw):.4f})  "
      f"{nu} x {nc} = {pairs / 1e9:.3f} G pairs  frac row {4 * pairs * D / np.median(fw) / 1e9 / 416.7:.3f} "
      f"col {2 * pairs * D / np.median(bw) / 1e9 / 416.7:.3f} pair {6 * pairs * D / (np.median(fw) + np.median(bw)) / 1e9 / 416.7:.3f}",
      flush=True)
