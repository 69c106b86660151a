"""Time the score-storing in-batch pair at each contraction precision (0 = f32 MFMA, 6 / 9 =
split bf16 terms) and report the error of each against a float64 reference on a row slice.
Usage: python tools/microbench_inbatch_prec.py [B] [precisions, e.g. 0,6,9]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
precs = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,6,9").split(",")]
D = 128
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(0)
U = (torch.randn(B, D, device=dev, generator=g) * 0.3).contiguous()
C = (torch.randn(B, D, device=dev, generator=g) * 0.3).contiguous()
gs = torch.tensor(1.0, device=dev)
Sbuf = F.inbatch_scores_buffer(B, dev)
fl = 2.0 * B * B * D
# float64 reference on 256 rows: lse, dU rows; dC on 256 columns
R = 256
U64, C64 = U.double(), C.double()
S64 = U64[:R] @ C64.T
lse64 = torch.logsumexp(S64, 1)
P64 = torch.exp(S64 - lse64[:, None])
dU64 = P64 @ C64 - C64[:R]
lse_all = torch.logsumexp(U64 @ C64[:R].T, 1) if B <= 8192 else None
for prec in precs:
    for _ in range(2):
        tot, row, lse, dU, _ = F.inbatch_softmax_fwd(U, C, scores=Sbuf, precision=prec)
        F.inbatch_softmax_bwd(U, C, lse, gscale=gs, dU_unit=dU, scores=Sbuf, precision=prec)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    reps = 5
    ev[0].record()
    for _ in range(reps):
        tot, row, lse, dU, _ = F.inbatch_softmax_fwd(U, C, scores=Sbuf, precision=prec)
    ev[1].record()
    for _ in range(reps):
        dUs, dC = F.inbatch_softmax_bwd(U, C, lse, gscale=gs, dU_unit=dU, scores=Sbuf, precision=prec)
    ev[2].record()
    torch.cuda.synchronize()
    tf = ev[0].elapsed_time(ev[1]) / reps
    tb = ev[1].elapsed_time(ev[2]) / reps
    e_lse = (lse[:R].double() - lse64).abs().max().item()
    e_du = (dU[:R].double() - dU64).abs().max().item()
    bits = lambda x: int(x.contiguous().view(torch.int32).long().mul(torch.arange(1, x.numel() + 1, device=x.device).view(x.shape) % 1000003).sum().item())
    sv = Sbuf.view(torch.int32)
    s_all = sum(int(sv[i:i + (1 << 27)].to(torch.int64).sum().item()) for i in range(0, sv.numel(), 1 << 27))
    print(f"prec={prec} bitsum lse {bits(lse)} dU {bits(dU)} dC {bits(dC)} S {bits(Sbuf[:1 << 24])} "
          f"Slast {bits(Sbuf[-(1 << 24):])} Sall {s_all}")
    print(f"prec={prec} B={B}: fwd {tf:.3f} ms ({2 * fl / tf / 1e9:.1f} TF/s fp32-equiv)  "
          f"bwd {tb:.3f} ms ({fl / tb / 1e9:.1f} TF/s)  max|err| lse {e_lse:.3e} dU {e_du:.3e}", flush=True)
