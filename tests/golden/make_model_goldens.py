"""Model-side golden vectors (SURVEY §8c "golden vectors (2)"): the oracle's restatement of the
reference arithmetic on fixed seeded weights in Keras layout, frozen as data.

    python tests/golden/make_model_goldens.py

TensorFlow is absent, so these vectors come from the numpy restatement (model side "parity
unpinned" at the TF boundary); freezing them pins the restatement against drift
(tests/test_oracle.py) and gives the GPU tests a fixed target independent of the live oracle
(tests/test_gpu_model.py). Written: model_goldens.npz (inputs, weights, activations, the B x B
scores, per-row retrieval loss, loss parts, every gradient, one Adagrad step).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle.recsys_oracle as O  # noqa: E402

CFG = dict(embedding_dim=16, user_tower_dims=[32, 16], item_tower_dims=[32, 16], cross_layers=2,
           dnn_dims=[16, 8])
NU, NI, B, SEED = 30, 20, 24, 11
CW = {0: 0.8, 1: 1.4}


def make():
    cfg = O.OracleConfig(**CFG)
    P = O.init_params(cfg, NU + 1, NI + 1, seed=SEED, dtype=np.float32, bias_scale=0.05)
    P = {k: v.astype(np.float64) for k, v in P.items()}
    rng = np.random.default_rng(SEED)
    uid = rng.integers(0, NU + 1, B)
    iid = rng.integers(0, NI + 1, B)
    rating = rng.integers(1, 6, B).astype(np.float64)
    yi = (rating >= 4).astype(np.float64)
    cache = O.forward(P, cfg, uid, iid)
    row, tot, lse = O.retrieval_loss(cache["U"], cache["C"])
    out = O.loss_and_grads(P, cfg, uid, iid, rating, yi, CW, ctr_mode=0)
    g = {}
    for k, v in out["grads"].items():
        if isinstance(v, tuple):
            g[f"gids::{k}"] = np.asarray(v[0])
            g[f"grows::{k}"] = v[1]
        else:
            g[f"g::{k}"] = v
    P1 = {k: v.copy() for k, v in P.items()}
    A1 = O.init_accumulators(P1)
    O.adagrad_apply(P1, A1, out["grads"], 0, 0.02, clipnorm=1.0)
    arrays = {"uid": uid, "iid": iid, "rating": rating, "y_implicit": yi,
              "U": cache["U"], "C": cache["C"], "x0": cache["x0"], "xL": cache["xL"], "h": cache["h"],
              "r": cache["r"], "p": cache["p"], "S": cache["U"] @ cache["C"].T, "row_loss": row, "lse": lse,
              "loss": np.array(out["loss"]), "loss_retrieval": np.array(out["retrieval"]),
              "loss_rating": np.array(out["rating"]), "loss_ctr": np.array(out["ctr"]), "reg": np.array(out["reg"]),
              "total_loss": np.array(out["total_loss"])}
    arrays.update({f"P::{k}": v for k, v in P.items()})
    arrays.update(g)
    arrays.update({f"P1::{k}": v for k, v in P1.items()})
    return arrays


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "model_goldens.npz"), **make())
    print("wrote", os.path.join(HERE, "model_goldens.npz"))
