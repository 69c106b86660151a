"""Diagnostic (round 5): the in-batch pair alone at C2 (B = 4096, D = 128) on the C2 model's own
tower outputs, at contraction precision 0 / 6 / 9 against float64: lse (signed mean and RMS error),
the implied P row sums, dU, dC and their column sums (the tower-top bias gradients' retrieval part,
which cancel to ~0 in exact arithmetic and so expose any error common to the rows).
Usage: python tools/diag_inbatch_prec.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import pkg  # noqa: E402
import oracle.recsys_oracle as O  # noqa: E402

dev = torch.device("cuda")
cfgm, models, F = pkg("config"), pkg("models"), pkg("functional")
nu, ni, B = 6040, 3706, 4096
ocfg = O.OracleConfig(embedding_dim=128, cross_layers=3, learning_rate_retrieval=0.01)
P = O.init_params(ocfg, nu + 1, ni + 1, seed=11, dtype=np.float32, bias_scale=0.05)
rng = np.random.default_rng(4096)
uid = rng.integers(0, nu + 1, B)
iid = rng.integers(0, ni + 1, B)
cfg = cfgm.ModelConfig(embedding_dim=128, cross_layers=3, batch_size=B, contraction_precision=6)
model = models.MultiTaskModel(cfg, nu, ni, {}, device=dev)
model.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
with torch.no_grad():
    emb = model.encoder({"user_id": torch.from_numpy(uid).to(dev), "movie_id": torch.from_numpy(iid).to(dev)})
U, C = emb["user_embedding"].contiguous(), emb["item_embedding"].contiguous()
U64, C64 = U.double().cpu().numpy(), C.double().cpu().numpy()
S = U64 @ C64.T
lse = O.logsumexp_rows(S)
Pm = np.exp(S - lse[:, None])
dU_ref = Pm @ C64 - C64
dC_ref = Pm.T @ U64 - U64
scale_u = np.abs(dU_ref).max()
print(f"U {np.abs(U64).max():.3e} C {np.abs(C64).max():.3e} S [{S.min():.4f}, {S.max():.4f}] lse [{lse.min():.4f}, {lse.max():.4f}]")
print(f"colsum ref: dU {np.abs(dU_ref.sum(0)).max():.3e} dC {np.abs(dC_ref.sum(0)).max():.3e}; "
      f"sum |dU| {np.abs(dU_ref).sum(0).max():.3e} sum |dC| {np.abs(dC_ref).sum(0).max():.3e}")
g = torch.ones((), device=dev)
for prec in (0, 6, 9):
    buf = F.inbatch_scores_buffer(B, dev)
    tot, row, lse_g, dU_unit, tot64 = F.inbatch_softmax_fwd(U, C, scores=buf, precision=prec)
    dU, dC = F.inbatch_softmax_bwd(U, C, lse_g, gscale=g, dU_unit=dU_unit, scores=buf, precision=prec)
    torch.cuda.synchronize()
    lg = lse_g.double().cpu().numpy()
    e = lg - lse
    rs = np.exp(S - lg[:, None]).sum(1) - 1
    dUg, dCg = dU.double().cpu().numpy(), dC.double().cpu().numpy()
    cu = np.abs(dUg.sum(0) - dU_ref.sum(0)).max()
    cc = np.abs(dCg.sum(0) - dC_ref.sum(0)).max()
    print(f"prec {prec}: lse err mean {e.mean():+.3e} rms {np.sqrt((e**2).mean()):.3e} | rowsum-1 mean {rs.mean():+.3e} "
          f"rms {np.sqrt((rs**2).mean()):.3e} | dU max {np.abs(dUg-dU_ref).max():.3e} dC max {np.abs(dCg-dC_ref).max():.3e} | "
          f"colsum err dU {cu:.3e} dC {cc:.3e}")
    # where the dC column-sum error comes from: with the GPU's own lse in the fp64 P
    Pg = np.exp(S - lg[:, None])
    dCl = Pg.T @ U64 - U64
    dUl = Pg @ C64 - C64
    print(f"          fp64 with the GPU lse: colsum err dU {np.abs(dUl.sum(0)-dU_ref.sum(0)).max():.3e} "
          f"dC {np.abs(dCl.sum(0)-dC_ref.sum(0)).max():.3e}")
