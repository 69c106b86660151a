"""Helper of tests/test_gpu_env_switches.py (run as a subprocess, never collected): a fixed set of
product calls whose kernel choice the former RS_* switches used to steer, printed as one sha256 of
every output byte. Run once with and once without the switches set; the release library must give
the same digest."""
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.conftest import pkg  # noqa: E402

dev = torch.device("cuda")
cfgm, models, optim, F = pkg("config"), pkg("models"), pkg("optim"), pkg("functional")
h = hashlib.sha256()


def eat(*ts):
    for t in ts:
        h.update(t.detach().contiguous().cpu().numpy().tobytes())


torch.manual_seed(0)
# MultiTaskModel steps: B = 4096 (one-launch stacks), B = 20000 (per-layer skinny GEMMs, id plan,
# deduplicated in-batch pair with stream-K splits, plan-ordered sparse update)
for B, nu, ni in ((4096, 3000, 2000), (20000, 30000, 6000)):
    cfg = cfgm.ModelConfig(embedding_dim=128, cross_layers=3, batch_size=B)
    model = models.MultiTaskModel(cfg, nu, ni, {}, class_weights={0: 0.8, 1: 1.3}, device=dev, seed=3)
    opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(), 0.05, clipnorm=1.0)
    rng = np.random.default_rng(B)
    for step in range(2):
        uid = torch.from_numpy(np.minimum(rng.zipf(1.3, B), nu)).to(dev)
        iid = torch.from_numpy(np.minimum(rng.zipf(1.3, B), ni)).to(dev)
        rating = torch.from_numpy(rng.integers(1, 6, B).astype(np.float32)).to(dev)
        data = ({"user_id": uid, "movie_id": iid}, {"rating": rating, "y_implicit": (rating >= 4).float()})
        opt.zero_grad()
        loss = model.compute_loss(data)
        (loss + sum(model.losses)).backward()
        opt.step()
        eat(loss)
    eat(*model.state_dict().values())
# DCN-v2 ranker (plane-pair GEMMs, split-K weight gradients)
rk = models.DCNv2Ranker([5000] * 4, embedding_dim=128, num_dense=13, cross_layers=2, deep_layers=[256, 256],
                        device=dev, seed=5)
opt = optim.Adagrad(rk.dense_parameters(), rk.embedding_modules(), 0.05, clipnorm=1.0)
rng = np.random.default_rng(7)
B = 4096
for step in range(2):
    ids = torch.from_numpy(rng.integers(0, 5001, (4, B))).to(dev)
    dense = torch.from_numpy(rng.standard_normal((B, 13)).astype(np.float32)).to(dev)
    y = torch.from_numpy((rng.random(B) < 0.3).astype(np.float32)).to(dev)
    opt.zero_grad()
    loss = rk.compute_loss(ids, dense, y)
    loss.backward()
    opt.step()
    eat(loss)
eat(*rk.state_dict().values())
# exact top-k: the bound-first scan (> 64 queries over >= 2^20 rows) and the list scan
items = torch.randn((1 << 20, 128), device=dev)
for Q in (16, 256):
    s, i = F.topk_ip(torch.randn((Q, 128), device=dev), items, 100, precision=6)
    eat(s, i)
torch.cuda.synchronize()
print("DIGEST", h.hexdigest())
