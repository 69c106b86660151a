"""Diagnostic: the C2 step's gradient errors against the float64 oracle under the GPU's ReLU gates,
per parameter, at contraction precision 6 and 0, next to the float32 oracle's own error (numpy sgemm
accumulation). Usage: python tools/diag_c2_grad_err.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import gpu_relu_masks, mask_flips, pkg, rel_err  # noqa: E402
import oracle.recsys_oracle as O  # noqa: E402

torch.set_num_threads(16)
dev = torch.device("cuda")
cfgm, models = pkg("config"), pkg("models")
nu, ni, B = 6040, 3706, 4096
ocfg = O.OracleConfig(embedding_dim=128, cross_layers=3, learning_rate_retrieval=0.01)
P = O.init_params(ocfg, nu + 1, ni + 1, seed=11, dtype=np.float32, bias_scale=0.05)
P64 = {k: v.astype(np.float64) for k, v in P.items()}
rng = np.random.default_rng(4096)
uid = rng.integers(0, nu + 1, B)
iid = rng.integers(0, ni + 1, B)
rating = rng.integers(1, 6, B).astype(np.float32)
yi = (rating >= 4).astype(np.float32)
cw = {0: 1.6, 1: 0.73}
data = ({"user_id": torch.from_numpy(uid).to(dev), "movie_id": torch.from_numpy(iid).to(dev)},
        {"rating": torch.from_numpy(rating).to(dev), "y_implicit": torch.from_numpy(yi).to(dev)})
rows = {}
for prec in (6, 0, 9):
    cfg = cfgm.ModelConfig(embedding_dim=128, cross_layers=3, batch_size=B, learning_rate_retrieval=0.01,
                           contraction_precision=prec)
    model = models.MultiTaskModel(cfg, nu, ni, {}, class_weights=cw, device=dev)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    F = pkg("functional")
    with F.record_relu_gates() as rec:
        loss = model.compute_loss(data)
        (loss + sum(model.losses)).backward()
    gm = gpu_relu_masks(model, rec)
    flips = mask_flips(O, P64, ocfg, uid, iid, gm)
    ref = O.loss_and_grads(P64, ocfg, uid, iid, rating.astype(np.float64), yi.astype(np.float64), cw, masks=gm)
    if prec == 6:
        r32 = O.loss_and_grads(P, ocfg, uid, iid, rating, yi, cw, masks=gm)
    named = dict(model.named_parameters())
    print(f"precision {prec}: flips {flips}", flush=True)
    for k, g in ref["grads"].items():
        if isinstance(g, tuple):
            emb = model.encoder.user_embedding if "user" in k else model.encoder.item_embedding
            got, g = emb.sink.gathered()[1].double().cpu().numpy(), g[1]
            g32 = r32["grads"][k][1]
        else:
            got = named[k].grad.double().cpu().numpy().reshape(g.shape)
            g32 = r32["grads"][k]
        rows.setdefault(k, {})[prec] = rel_err(got, g, 0.0)
        rows[k]["f32"] = rel_err(g32, g, 0.0)
print(f"{'parameter':45s} {'prec6':>9s} {'prec0':>9s} {'prec9':>9s} {'np-f32':>9s}")
for k, r in rows.items():
    print(f"{k:45s} {r[6]:9.2e} {r[0]:9.2e} {r[9]:9.2e} {r['f32']:9.2e}")
