"""The N-independent sparse costs of the data-parallel C3 step on one GPU, hipGraph-
timed: (a) the local deduplication of each table's 65,536 raw gradient rows (rs_sparse_dedupe_f32,
what each rank runs before the all-gather), (b) the sparse Adagrad over the rows an 8-rank step
applies after the deduplicating exchange (8 ranks' distinct (id, row) pairs per table, rank order,
the exchanged norm), and for reference (c) the one-GPU update of the 2 x 65,536 raw rows in the
plan's order with its run heads (the single-GPU step's path) and (d) sorted by the update itself.
Zipf(1.05) ids over 10M users / 1M items, B = 65,536 per rank, D = 128.
Usage: python tools/microbench_dp_sparse.py [ranks=8] (prints one JSON line)"""
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
bench = importlib.import_module("bench")

R = int(sys.argv[1]) if len(sys.argv) > 1 else 8
B, D, NU, NI = 65536, 128, 10_000_000, 1_000_000
dev = torch.device("cuda")
tabs = [torch.empty((NU + 1, D), device=dev).uniform_(-0.05, 0.05),
        torch.empty((NI + 1, D), device=dev).uniform_(-0.05, 0.05)]
accs = [torch.full_like(t, 0.1) for t in tabs]
it = torch.zeros((), dtype=torch.int64, device=dev)
rng = np.random.default_rng(11)


def graph_us(fn, reps=10):
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


ranks = []
for r in range(R):
    uid = torch.from_numpy(bench.zipf_ids(rng, B, NU)).to(dev)
    iid = torch.from_numpy(bench.zipf_ids(rng, B, NI)).to(dev)
    ranks.append((uid, iid, torch.randn((B, D), device=dev) * 1e-3, torch.randn((B, D), device=dev) * 1e-3))
uid, iid, gu, gi = ranks[0]
out = {"ranks": R, "B_per_rank": B, "D": D}

# (a) one rank's local deduplication of both tables (each rank runs this; N-independent): sorting,
# and over the step's id plan (the product's path in the data-parallel step)
out["local_dedupe_sorting_us"] = round(graph_us(lambda: (F.sparse_dedupe(uid, gu, NU + 1),
                                                         F.sparse_dedupe(iid, gi, NI + 1))), 1)
plan = F.inbatch_unique_ids_pair(uid, iid, NU + 1, NI + 1, order=True, dids=True)
pls = [(p[5], p[7], p[6], p[3][0:1]) for p in plan]
out["local_dedupe_planned_us"] = round(graph_us(lambda: (F.sparse_dedupe(uid, gu, NU + 1, plan=pls[0]),
                                                         F.sparse_dedupe(iid, gi, NI + 1, plan=pls[1]))), 1)

# (b) the update an R-rank deduplicating exchange leaves: every rank's distinct pairs, rank order
ded = [[F.sparse_dedupe(r[0], r[2], NU + 1), F.sparse_dedupe(r[1], r[3], NI + 1)] for r in ranks]
torch.cuda.synchronize()
cat_ids, cat_rows, ssq = [], [], []
for t in range(2):
    cs = [int(d[t][2].item()) for d in ded]
    cat_ids.append(torch.cat([d[t][0][:c] for d, c in zip(ded, cs)]))
    cat_rows.append(torch.cat([d[t][1][:c] for d, c in zip(ded, cs)]))
    ssq.append(torch.stack([d[t][3] for d in ded]).sum().reshape(()))
out["dp_rows_per_table"] = [int(x.numel()) for x in cat_ids]
out["dp_rows_total"] = sum(out["dp_rows_per_table"])
out["dp_update_sorting_us"] = round(graph_us(lambda: F.sparse_adagrad_multi(
    tabs, accs, cat_ids, cat_rows, it, 0.05, 0.96, 1000, 1.0, 1e-7, sumsq=ssq, increment=True)), 1)
offs = [np.concatenate([[0], np.cumsum([int(d[t][2].item()) for d in ded])]).tolist() for t in range(2)]
out["dp_merge_order_us"] = round(graph_us(lambda: [F.merge_runs_order(cat_ids[t], offs[t]) for t in range(2)]), 1)
mo = [F.merge_runs_order(cat_ids[t], offs[t]) for t in range(2)]
out["dp_update_merged_us"] = round(graph_us(lambda: F.sparse_adagrad_multi(
    tabs, accs, cat_ids, cat_rows, it, 0.05, 0.96, 1000, 1.0, 1e-7, sumsq=ssq, increment=True, orders=mo)), 1)

# (c) / (d) the one-GPU step's update of the raw rows: the plan's order + run heads, and sorted
orders = [plan[0][5], plan[1][5]]
heads = [(plan[0][7], plan[0][6], plan[0][3][0:1]), (plan[1][7], plan[1][6], plan[1][3][0:1])]
out["one_gpu_update_planned_us"] = round(graph_us(lambda: F.sparse_adagrad_multi(
    tabs, accs, [uid, iid], [gu, gi], it, 0.05, 0.96, 1000, 1.0, 1e-7, increment=True, orders=orders, heads=heads)), 1)
out["one_gpu_update_ordered_us"] = round(graph_us(lambda: F.sparse_adagrad_multi(
    tabs, accs, [uid, iid], [gu, gi], it, 0.05, 0.96, 1000, 1.0, 1e-7, increment=True, orders=orders)), 1)
out["one_gpu_update_sorted_us"] = round(graph_us(lambda: F.sparse_adagrad_multi(
    tabs, accs, [uid, iid], [gu, gi], it, 0.05, 0.96, 1000, 1.0, 1e-7, increment=True)), 1)
print(json.dumps(out), flush=True)
