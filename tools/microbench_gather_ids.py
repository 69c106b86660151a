"""The C3 step's distinct-id lookup (rs_embedding_gather_tables_ids_f32: the id plan's ascending
distinct ids, -1 past the count) hipGraph-timed over 8 different batches in rotation (so a replay
does not re-read rows an earlier launch left in L2 / MALL), Zipf(1.05) and uniform ids over 10M users
/ 1M items, B = 65536 per side. Bytes: (2 D 4 + 8) per distinct row. Set RECSYS_HIP_LIB to time a
variant build. Usage: python tools/microbench_gather_ids.py"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
bench = importlib.import_module("bench")

B, D, NU, NI, NB, REPS = 65536, 128, 10_000_000, 1_000_000, 8, 4
dev = torch.device("cuda")
ut = torch.empty((NU + 1, D), device=dev).uniform_(-0.05, 0.05)
it = torch.empty((NI + 1, D), device=dev).uniform_(-0.05, 0.05)
rng = np.random.default_rng(7)
lib = os.environ.get("RECSYS_HIP_LIB", "release")

for law in ("zipf", "uniform"):
    sets, nrows = [], 0
    for _ in range(NB):
        if law == "zipf":
            uid = torch.from_numpy(bench.zipf_ids(rng, B, NU)).to(dev)
            iid = torch.from_numpy(bench.zipf_ids(rng, B, NI)).to(dev)
        else:
            uid = torch.from_numpy(rng.integers(1, NU + 1, B)).to(dev)
            iid = torch.from_numpy(rng.integers(1, NI + 1, B)).to(dev)
        pu, pi = F.inbatch_unique_ids_pair(uid, iid, NU + 1, NI + 1, order=True, dids=True)
        du, di = pu[6], pi[6]
        nrows += int((du >= 0).sum().item()) + int((di >= 0).sum().item())
        outs = [torch.empty((B, D), device=dev), torch.empty((B, D), device=dev)]
        sets.append((du, di, outs))
        # check: each written row is the table row of its id
        F.embedding_gather_tables_ids([ut, it], [du, di], out=outs)
        nu = int((du >= 0).sum().item())
        assert torch.equal(outs[0][:nu], ut[du[:nu]]), "user rows differ"
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            for _ in range(REPS):
                for du, di, outs in sets:
                    F.embedding_gather_tables_ids([ut, it], [du, di], out=outs)
    torch.cuda.current_stream().wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(5):
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / (REPS * NB))
    by = nrows / NB * (2 * D * 4 + 8)
    print(f"{lib}: {law:7s} {nrows / NB:8.0f} distinct rows/launch  {best:6.2f} us  {by / best / 1e3:6.0f} GB/s "
          f"frac {by / best / 1e3 / 8000:.3f}", flush=True)
