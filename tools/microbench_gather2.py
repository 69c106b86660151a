"""Gather of the C3 step (user 10M x 128 + item 1M x 128 tables, B = 65536 each, one launch of
rs_embedding_gather_tables_f32) on FRESH id batches per launch (no MALL reuse between launches),
Zipf(1.05) vs uniform, as issued and with the ids pre-sorted (locality / hot-row probe).
Algorithmic bytes = 2 B (2 D 4 + 8)."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
bench = importlib.import_module("bench")

D, B, R = 128, int(sys.argv[1]) if len(sys.argv) > 1 else 65536, 12
dev = torch.device("cuda")
tabs = [torch.empty((n + 1, D), dtype=torch.float32, device=dev).uniform_(-0.05, 0.05) for n in (10_000_000, 1_000_000)]
rng = np.random.default_rng(1234)
nbytes = 2 * B * (2 * D * 4 + 8)
for dist in ("zipf", "uniform"):
    for order in ("as-issued", "sorted"):
        batches = []
        for _ in range(R):
            ids = []
            for t in tabs:
                v = t.shape[0] - 1
                x = bench.zipf_ids(rng, B, v) if dist == "zipf" else rng.integers(1, v + 1, B)
                if order == "sorted":
                    x = np.sort(x)
                ids.append(torch.from_numpy(x).to(dev))
            batches.append(ids)
        F.embedding_gather_tables(tabs, batches[0])
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(R)]
        for (s, e), ids in zip(ev, batches):
            s.record()
            F.embedding_gather_tables(tabs, ids)
            e.record()
        torch.cuda.synchronize()
        ms = np.array([s.elapsed_time(e) for s, e in ev])
        uniq = np.mean([len(np.unique(b[0].cpu().numpy())) / B for b in batches])
        print(f"{dist:8s} {order:9s}: median {np.median(ms)*1e3:6.1f} us  min {ms.min()*1e3:6.1f} us -> "
              f"{nbytes / (np.median(ms) * 1e-3) / 1e9:6.0f} GB/s ({nbytes / (np.median(ms) * 1e-3) / 8e12 * 100:.1f}% of 8 TB/s), "
              f"user-table unique {uniq:.2f}", flush=True)
