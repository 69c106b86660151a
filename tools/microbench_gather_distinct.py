"""The C3 step's table lookup three ways, hipGraph-timed (20 launches per replay): (a) the
distinct-row form the step runs (rs_embedding_gather_tables_rows_f32: representative batch row ->
id -> row, device counts), (b) the same distinct ids handed over compact (one dependent load
fewer), (c) the full-B lookup of every batch row. Zipf(1.05) ids over 10M users / 1M items, B =
65536 per side. Usage: python tools/microbench_gather_distinct.py"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
bench = importlib.import_module("bench")

B, D, NU, NI = 65536, 128, 10_000_000, 1_000_000
dev = torch.device("cuda")
ut = torch.empty((NU + 1, D), device=dev).uniform_(-0.05, 0.05)
it = torch.empty((NI + 1, D), device=dev).uniform_(-0.05, 0.05)
rng = np.random.default_rng(7)


def graph_us(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for law in ("zipf", "uniform"):
    if law == "zipf":
        uid = torch.from_numpy(bench.zipf_ids(rng, B, NU)).to(dev)
        iid = torch.from_numpy(bench.zipf_ids(rng, B, NI)).to(dev)
    else:
        uid = torch.from_numpy(rng.integers(1, NU + 1, B)).to(dev)
        iid = torch.from_numpy(rng.integers(1, NI + 1, B)).to(dev)
    pu, pi = F.inbatch_unique_ids_pair(uid, iid, NU + 1, NI + 1)
    cu, ci = pu[3][0:1], pi[3][0:1]
    nu, ni = int(cu.item()), int(ci.item())
    du = uid[pu[0][:nu].long()].contiguous()
    di = iid[pi[0][:ni].long()].contiguous()
    ta = graph_us(lambda: F.embedding_gather_tables_rows([ut, it], [uid, iid], [pu[0], pi[0]], [cu, ci]))
    tb = graph_us(lambda: F.embedding_gather_tables([ut, it], [du, di]))
    tc = graph_us(lambda: F.embedding_gather_tables([ut, it], [uid, iid]))
    ra = F.embedding_gather_tables_rows([ut, it], [uid, iid], [pu[0], pi[0]], [cu, ci])
    rb = F.embedding_gather_tables([ut, it], [du, di])
    same = torch.equal(ra[0][:nu], rb[0]) and torch.equal(ra[1][:ni], rb[1])
    bd = (nu + ni) * (2 * D * 4 + 8)
    bf = 2 * B * (2 * D * 4 + 8)
    print(f"{law:7s} distinct {nu}+{ni}: rows form {ta:6.1f} us ({bd / ta / 1e3:6.0f} GB/s)  compact ids "
          f"{tb:6.1f} us ({bd / tb / 1e3:6.0f} GB/s)  full B {tc:6.1f} us ({bf / tc / 1e3:6.0f} GB/s)  same={same}",
          flush=True)
