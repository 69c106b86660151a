"""Embedding-gather bandwidth on the C3 tables (10M x 128 fp32 user table, Zipf(1.05) and
uniform ids). Algorithmic bytes per gathered row = 2*D*4 + 8 (read row + write row + int64 id,
SURVEY §8d). Usage: python tools/microbench_gather.py [rows_per_call ...]"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
bench = importlib.import_module("bench")

V, D = 10_000_000, 128
dev = torch.device("cuda")
table = torch.empty((V + 1, D), dtype=torch.float32, device=dev).uniform_(-0.05, 0.05)
rng = np.random.default_rng(1234)
sizes = [int(s) for s in sys.argv[1:]] or [65536, 1 << 20, 4 << 20]
for n in sizes:
    for dist_name in ("zipf", "uniform"):
        if dist_name == "zipf":
            ids = bench.zipf_ids(rng, n, V)
        else:
            ids = rng.integers(1, V + 1, n)
        ids_t = torch.from_numpy(ids).to(dev)
        out = F.embedding_gather(table, ids_t)
        torch.cuda.synchronize()
        reps = 20
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            F.embedding_gather(table, ids_t)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        gbs = n * (2 * D * 4 + 8) / (ms * 1e-3) / 1e9
        ok = torch.equal(out[:1000], table[ids_t[:1000]])
        print(f"gather n={n:>8} {dist_name:7s}: {ms * 1e3:8.1f} us  {gbs:7.0f} GB/s  "
              f"({gbs / 8000 * 100:.1f}% of 8 TB/s)  parity={ok}")
