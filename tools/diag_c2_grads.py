"""Diagnostic: per-gradient error (max|a-b|/max|b|) of the C2 reference-dims step vs the fp64
oracle, at contraction precision 0 / 6 / 9, beside the numpy-fp32 oracle's own error."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib  # noqa: E402

PKG = "recommendation-system-maang-nvidia-_amd"
O = importlib.import_module("oracle.recsys_oracle")
cfgm = importlib.import_module(PKG + ".config")
models = importlib.import_module(PKG + ".models")
torch.set_num_threads(16)
nu, ni, B = 6040, 3706, int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dev = torch.device("cuda")
ocfg = O.OracleConfig(embedding_dim=128, cross_layers=3)
P = O.init_params(ocfg, nu + 1, ni + 1, seed=11, dtype=np.float32, bias_scale=0.05)
cw = {0: 1.6, 1: 0.73}
rng = np.random.default_rng(4096)
uid = rng.integers(0, nu + 1, B)
iid = rng.integers(0, ni + 1, B)
rating = rng.integers(1, 6, B).astype(np.float32)
yi = (rating >= 4).astype(np.float32)
P64 = {k: v.astype(np.float64) for k, v in P.items()}
r64 = O.loss_and_grads(P64, ocfg, uid, iid, rating.astype(np.float64), yi.astype(np.float64), cw)
r32 = O.loss_and_grads(P, ocfg, uid, iid, rating, yi, cw)


def errs(grads):
    out = {}
    for k, g in r64["grads"].items():
        a = grads[k]
        if isinstance(g, tuple):
            a, g = a[1], g[1]
        out[k] = np.abs(np.asarray(a, np.float64).reshape(g.shape) - g).max() / np.abs(g).max()
    return out


table = {"np32": errs(r32["grads"])}
for prec in (0, 6, 9):
    cfg = cfgm.ModelConfig(embedding_dim=128, cross_layers=3, contraction_precision=prec)
    m = models.MultiTaskModel(cfg, nu, ni, {}, class_weights=cw, device=dev)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    feats = {"user_id": torch.from_numpy(uid).to(dev), "movie_id": torch.from_numpy(iid).to(dev)}
    labels = {"rating": torch.from_numpy(rating).to(dev), "y_implicit": torch.from_numpy(yi).to(dev)}
    loss = m.compute_loss((feats, labels))
    (loss + sum(m.losses)).backward()
    named = dict(m.named_parameters())
    g = {}
    for k in r64["grads"]:
        if k.endswith("embedding.weight"):
            emb = m.encoder.user_embedding if "user" in k else m.encoder.item_embedding
            g[k] = (None, emb.sink.gathered()[1].double().cpu().numpy())
        else:
            g[k] = named[k].grad.double().cpu().numpy()
    table[f"p{prec}"] = errs(g)
    print(f"p{prec} loss {float(loss):.6f} oracle {r64['loss']:.6f}")
keys = sorted(r64["grads"], key=lambda k: -table["p6"][k])
print(f"{'grad':45s} " + " ".join(f"{c:>9s}" for c in table))
for k in keys:
    print(f"{k:45s} " + " ".join(f"{table[c][k]:9.2e}" for c in table))
