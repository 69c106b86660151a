"""The deduplicated in-batch pair at the C3 shape (B = 65536, D = 128, precision 6; Zipf(1.05) ids
over 10M users / 1M items as bench.py draws them, tower rows equal per id): the pre-pass, then
N x (forward + backward) between two iteration_increment marker kernels, so that rocprofv3 --pmc
passes can be cut to the timed launches (tools/traffic_summary.py, tools/pmc_summary.py).
Usage: python tools/microbench_inbatch_dedup.py [N] [B]"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
from bench import zipf_ids  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
D, PREC = 128, 6
dev = torch.device("cuda")
rng = np.random.default_rng(1234)
g = torch.Generator(device=dev)
g.manual_seed(5)


def tower_rows(vocab):
    ids = torch.from_numpy(zipf_ids(rng, B, vocab)).to(dev)
    uniq, inv = torch.unique(ids, return_inverse=True)
    rows = torch.randn((uniq.numel(), D), device=dev, generator=g) * 0.3
    return rows[inv].contiguous(), uniq.numel()


U, nu = tower_rows(10_000_000)
C, nc = tower_rows(1_000_000)
scores = F.inbatch_scores_buffer(B, dev)
users, items = F.inbatch_dedup_plan(U, C, PREC, force=True)
gs = torch.ones((), device=dev)
mark = torch.zeros((), dtype=torch.int64, device=dev)


def run():
    tot, row, lse, dU, _ = F.inbatch_softmax_fwd_dedup(U, C, users, items, scores, PREC)
    F.inbatch_softmax_bwd_dedup(U, lse, users, items, scores, PREC, gscale=gs, dU_unit=dU)
    return tot


run()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
F.iteration_increment(mark)
s.record()
for _ in range(N):
    tot = run()
e.record()
F.iteration_increment(mark)
torch.cuda.synchronize()
ms = s.elapsed_time(e) / N
pairs = users[3] * items[3]
print(f"dedup pair B={B}: {nu} distinct users x {nc} distinct items ({pairs / 1e9:.3f} G pairs), "
      f"{ms:.3f} ms per fwd+bwd, loss {float(tot):.6g}", flush=True)
