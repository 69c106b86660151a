"""HBM traffic probe for rocprofv3 --pmc passes: runs N launches of one measured entry point
between two marker dispatches (iteration_increment_kernel), so that the per-launch traffic is the
sum of the counters of the dispatches between the markers divided by N
(tools/traffic_summary.py). Workloads (the bench's shapes):
  c4        rs_topk_ip_prec_f32, 1024 N(0,1) queries over a 12.5M x 128 N(0,1) shard, k = 100, precision 6
  c5:<B>    the DCN-v2 cross stack on the plane path (d = 3344, L = 4): N x (forward + backward)
  gather:<zipf|uniform>  rs_embedding_gather_tables_f32 of the C3 step (10M + 1M rows, 2 x 65536 ids)
Usage: python tools/traffic_probe.py <workload> [N]"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
what = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(7)
mark = torch.zeros((), dtype=torch.int64, device=dev)

if what == "c4":
    items = torch.randn((12_500_000, 128), device=dev, generator=g)
    q = torch.randn((1024, 128), device=dev, generator=g)
    run = lambda: F.topk_ip(q, items, 100, precision=6)
elif what.startswith("c5"):
    B = int(what.split(":")[1]) if ":" in what else 16384
    d, L = 3344, 4
    x0 = torch.randn(B, d, device=dev, generator=g) * 0.1
    W = torch.randn(L, d, d, device=dev, generator=g) / d ** 0.5
    b = torch.randn(L, d, device=dev, generator=g) * 0.01
    gy = torch.randn(B, d, device=dev, generator=g)

    def run():
        o = F.dcn_cross_mat_fwd_planes(x0, W, b, precision=6)
        F.dcn_cross_mat_bwd_planes(x0, o[0], o[1], W, o[2], gy, precision=6)
elif what.startswith("gather"):
    kind = what.split(":")[1]
    tables = [torch.rand((10_000_001, 128), device=dev, generator=g), torch.rand((1_000_001, 128), device=dev, generator=g)]
    rng = np.random.default_rng(1234)
    B = 65536

    def ids_for(V):
        if kind == "uniform":
            return torch.randint(1, V, (B,), device=dev, generator=g)
        r = rng.zipf(1.05, B * 2)
        r = r[r <= V - 1][:B]
        return torch.from_numpy(((r.astype(np.int64) * (2654435761 % (V - 1))) % (V - 1)) + 1).to(dev)

    batches = [[ids_for(t.shape[0]) for t in tables] for _ in range(N + 1)]
    it = iter(batches)
    run = lambda: F.embedding_gather_tables(tables, next(it))
else:
    raise SystemExit(f"unknown workload {what}")

run()                              # warm-up (code objects, workspaces)
torch.cuda.synchronize()
F.iteration_increment(mark)        # start marker
for _ in range(N):
    run()
F.iteration_increment(mark)        # end marker
torch.cuda.synchronize()
print(f"{what}: {N} launches between the markers", flush=True)
