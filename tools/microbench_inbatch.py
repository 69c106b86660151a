"""Time the in-batch softmax fwd (row pass + dU) and bwd (col pass) alone, plus a parity spot
check against float64 torch on a slice. Usage: python tools/microbench_inbatch.py [B] [D]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
D = int(sys.argv[2]) if len(sys.argv) > 2 else 128
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(0)
U = (torch.randn(B, D, device=dev, generator=g) * 0.3).contiguous()
C = (torch.randn(B, D, device=dev, generator=g) * 0.3).contiguous()
gs = torch.tensor(1.0, device=dev)

ONLY_STORED = len(sys.argv) > 3 and sys.argv[3] == "stored"
reps = 5
if ONLY_STORED:   # (PMC passes: only the score-storing pair)
    reps = 0
for _ in range(0 if ONLY_STORED else 2):
    tot, row, lse, dU, _ = F.inbatch_softmax_fwd(U, C)
    F.inbatch_softmax_bwd(U, C, lse, gscale=gs, dU_unit=dU)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
ev[0].record()
for _ in range(reps):
    tot, row, lse, dU, _ = F.inbatch_softmax_fwd(U, C)
ev[1].record()
for _ in range(reps):
    dUs, dC = F.inbatch_softmax_bwd(U, C, lse, gscale=gs, dU_unit=dU)
ev[2].record()
torch.cuda.synchronize()
fl = 4.0 * B * B * D
tf = ev[0].elapsed_time(ev[1]) / max(reps, 1)
tb = ev[1].elapsed_time(ev[2]) / max(reps, 1)
if reps:
    print(f"B={B} D={D}: fwd {tf:.3f} ms ({fl / tf / 1e9:.1f} TF/s)  bwd {tb:.3f} ms ({fl / tb / 1e9:.1f} TF/s)")
reps = 5

# score-storing pair: forward keeps U C^T (B x B fp32), backward reads it
Sbuf = F.inbatch_scores_buffer(B, dev)
for _ in range(2):
    tot, row, lse, dU, _ = F.inbatch_softmax_fwd(U, C, scores=Sbuf)
    F.inbatch_softmax_bwd(U, C, lse, gscale=gs, dU_unit=dU, scores=Sbuf)
torch.cuda.synchronize()
ev[0].record()
for _ in range(reps):
    tot, row, lse, dU, _ = F.inbatch_softmax_fwd(U, C, scores=Sbuf)
ev[1].record()
for _ in range(reps):
    dUs2, dC2 = F.inbatch_softmax_bwd(U, C, lse, gscale=gs, dU_unit=dU, scores=Sbuf)
ev[2].record()
torch.cuda.synchronize()
tf2 = ev[0].elapsed_time(ev[1]) / reps
tb2 = ev[1].elapsed_time(ev[2]) / reps
print(f"stored scores ({Sbuf.numel() * 4 / 1e9:.1f} GB): fwd {tf2:.3f} ms ({fl / tf2 / 1e9:.1f} TF/s)  "
      f"bwd {tb2:.3f} ms ({fl / 2 / tb2 / 1e9:.1f} TF/s on its 2 B^2 D)  total {tf2 + tb2:.3f} vs {tf + tb:.3f} ms",
      flush=True)
del Sbuf

# spot parity on the first 512 rows (float64 torch reference over the full batch of candidates)
n = 512
S = U[:n].double() @ C.double().T
lse_ref = torch.logsumexp(S, 1)
P = torch.exp(S - lse_ref[:, None])
dU_ref = P @ C.double() - C[:n].double()
print("lse max err", (lse[:n].double() - lse_ref).abs().max().item(),
      "dU max err", (dU[:n].double() - dU_ref).abs().max().item())
Sc = U.double() @ C[:n].double().T           # columns 0..n-1 for dC
Pc = torch.exp(Sc - lse.double()[:, None])
dC_ref = Pc.T @ U.double() - U[:n].double()
print("dC max err", (dC2[:n].double() - dC_ref).abs().max().item())
