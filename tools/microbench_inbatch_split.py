"""Time the default C3 in-batch pair alone: the score-keeping row pass (forward) and the col pass
from the kept scores (backward) at contraction precision 6 (or argv[2]), B = argv[1] (65536).
TF/s = fp32-equivalent FLOP (4 B^2 D forward, 2 B^2 D backward) / time, against 2500 / 6."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
prec = int(sys.argv[2]) if len(sys.argv) > 2 else 6
D = 128
peak = 2500.0 / prec if prec else 157.3
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(0)
U = (torch.randn(B, D, device=dev, generator=g) * 0.3).contiguous()
C = (torch.randn(B, D, device=dev, generator=g) * 0.3).contiguous()
gs = torch.tensor(1.0, device=dev)
S = F.inbatch_scores_buffer(B, dev)
for _ in range(2):
    tot, row, lse, dU, _ = F.inbatch_softmax_fwd(U, C, scores=S, precision=prec)
    F.inbatch_softmax_bwd(U, C, lse, gscale=gs, dU_unit=dU, scores=S, precision=prec)
torch.cuda.synchronize()
reps = 5
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
ev[0].record()
for _ in range(reps):
    tot, row, lse, dU, _ = F.inbatch_softmax_fwd(U, C, scores=S, precision=prec)
ev[1].record()
for _ in range(reps):
    F.inbatch_softmax_bwd(U, C, lse, gscale=gs, dU_unit=dU, scores=S, precision=prec)
ev[2].record()
torch.cuda.synchronize()
tf, tb = ev[0].elapsed_time(ev[1]) / reps, ev[1].elapsed_time(ev[2]) / reps
ff, fb = 4.0 * B * B * D, 2.0 * B * B * D
print(f"B={B} prec={prec}: fwd {tf:.3f} ms ({ff / tf / 1e9:.1f} TF/s, {ff / tf / 1e9 / peak:.1%})  "
      f"bwd {tb:.3f} ms ({fb / tb / 1e9:.1f} TF/s, {fb / tb / 1e9 / peak:.1%})  "
      f"pair {(ff + fb) / (tf + tb) / 1e9 / peak:.1%}", flush=True)
