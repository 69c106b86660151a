"""Diagnostic: accuracy of the in-batch backward dC on C2-shaped tower outputs (B = 4096, D = 128)
vs float64, beside numpy fp32; splits the error into the lse part (row normalisation) and the
P^T U accumulation."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib  # noqa: E402

O = importlib.import_module("oracle.recsys_oracle")
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
dev = torch.device("cuda")
nu, ni, B = 6040, 3706, 4096
ocfg = O.OracleConfig(embedding_dim=128, cross_layers=3)
P = O.init_params(ocfg, nu + 1, ni + 1, seed=11, dtype=np.float32, bias_scale=0.05)
rng = np.random.default_rng(4096)
uid = rng.integers(0, nu + 1, B)
iid = rng.integers(0, ni + 1, B)
c = O.forward({k: v.astype(np.float64) for k, v in P.items()}, ocfg, uid, iid)
for scale in (1.0, 4.0):
    U32 = (c["U"] * scale).astype(np.float32)
    C32 = (c["C"] * scale).astype(np.float32)
    U, C = U32.astype(np.float64), C32.astype(np.float64)
    _, _, lse = O.retrieval_loss(U, C)
    dU, dC = O.retrieval_grads(U, C, lse)
    _, _, lse32 = O.retrieval_loss(U32, C32)
    dU32, dC32 = O.retrieval_grads(U32, C32, lse32)
    S64 = U @ C.T
    print(f"scale {scale}: |U| {np.abs(U).max():.3f} S range [{S64.min():.3f}, {S64.max():.3f}] lse mean {lse.mean():.3f}")
    for prec in (0, 6):
        for stored in (False, True):
            Sb = F.inbatch_scores_buffer(B, dev) if stored else None
            tU, tC = torch.from_numpy(U32).to(dev), torch.from_numpy(C32).to(dev)
            T, ROW, LSE, DU, T64 = F.inbatch_softmax_fwd(tU, tC, scores=Sb, precision=prec if stored else 0)
            DUs, DC = F.inbatch_softmax_bwd(tU, tC, LSE, gscale=torch.tensor(1.0, device=dev), dU_unit=DU, scores=Sb,
                                            precision=prec if stored else 0)
            lg = LSE.double().cpu().numpy()
            dcg = DC.double().cpu().numpy()
            # dC recomputed in fp64 from the GPU's lse: isolates the lse (normalisation) error
            Pg = np.exp(S64 - lg[:, None])
            dC_lse = (Pg - np.eye(B)).T @ U
            rs = Pg.sum(1) - 1.0
            m = np.abs(dC).max()
            print(f"  prec {prec} stored {stored}: lse err {np.abs(lg - lse).max():.2e} rowsum-1 max {np.abs(rs).max():.2e} "
                  f"| dC err {np.abs(dcg - dC).max() / m:.2e} (np32 {np.abs(dC32 - dC).max() / m:.2e}, "
                  f"from-lse-only {np.abs(dC_lse - dC).max() / m:.2e}) | colsum err {np.abs(dcg.sum(0) - dC.sum(0)).max():.2e} "
                  f"(np32 {np.abs(dC32.sum(0) - dC.sum(0)).max():.2e}, from-lse-only {np.abs(dC_lse.sum(0) - dC.sum(0)).max():.2e})"
                  f" | dU err {np.abs(DU.double().cpu().numpy() - dU).max() / np.abs(dU).max():.2e} "
                  f"(np32 {np.abs(dU32 - dU).max() / np.abs(dU).max():.2e})")
