"""The oracle checks itself against independent derivations before it is trusted:
  * every gradient of the full MultiTask objective vs torch.autograd in float64 (CPU);
  * finite differences on a few coordinates;
  * the Keras optimizer semantics it restates (sparse == dense when ids are unique, dedupe sums,
    clip over un-deduplicated values, staircase schedule);
  * top-K ordering and the data-parallel aggregation rule.
"""
import math

import numpy as np
import pytest
import torch

from conftest import oracle


def small_setup(seed=0, D=8, nu=20, ni=15, B=24, L=2):
    O = oracle()
    cfg = O.OracleConfig(embedding_dim=D, user_tower_dims=[16, 12], item_tower_dims=[16, 12],
                         cross_layers=L, dnn_dims=[16, 8])
    P = O.init_params(cfg, nu + 1, ni + 1, seed=seed, bias_scale=0.1)
    rng = np.random.default_rng(seed)
    uid = rng.integers(0, nu + 1, B)
    iid = rng.integers(0, ni + 1, B)
    rating = rng.integers(1, 6, B).astype(np.float64)
    yi = (rating >= 4).astype(np.float64)
    return O, cfg, P, uid, iid, rating, yi


def torch_objective(P, cfg, uid, iid, rating, yi, cw, mode):
    """Independent torch restatement of the same objective (autograd reference)."""
    T = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in P.items()}
    u = T["encoder.user_embedding.weight"][torch.tensor(uid)]
    it = T["encoder.item_embedding.weight"][torch.tensor(iid)]

    def tower(x, name, n):
        for j in range(n):
            x = x @ T[f"encoder.{name}.layers.{j}.kernel"] + T[f"encoder.{name}.layers.{j}.bias"]
            if j < n - 1:
                x = torch.relu(x)
        return x

    U = tower(u, "user_tower", len(cfg.user_tower_dims) + 1)
    C = tower(it, "item_tower", len(cfg.item_tower_dims) + 1)
    S = U @ C.T
    ret = (torch.logsumexp(S, 1) - torch.diagonal(S)).sum()
    x0 = torch.cat([U, C], 1)
    xl = x0
    for l in range(cfg.cross_layers):
        xl = x0 * (xl @ T["dcn.cross_w"][l])[:, None] + T["dcn.cross_b"][l] + xl
    h = x0
    for j in range(len(cfg.dnn_dims)):
        h = torch.relu(h @ T[f"dcn.deep_nets.{j}.kernel"] + T[f"dcn.deep_nets.{j}.bias"])
    z = torch.cat([xl, h], 1)
    r = (z @ T["rating_head.kernel"] + T["rating_head.bias"])[:, 0]
    p = torch.sigmoid(z @ T["ctr_head.kernel"] + T["ctr_head.bias"])[:, 0]
    y, yt = torch.tensor(rating), torch.tensor(yi)
    mse = ((r - y) ** 2).mean()
    eps = 1e-7
    pc = torch.clamp(p, eps, 1 - eps)
    bce = -(yt * torch.log(pc + eps) + (1 - yt) * torch.log(1 - pc + eps))
    sw = torch.where(yt == 1, torch.tensor(cw[1], dtype=torch.float64), torch.tensor(cw[0], dtype=torch.float64))
    ctr = (sw * bce).mean() if mode == 0 else bce.mean() * sw.mean()
    reg = cfg.l2_reg * sum((T[f"dcn.deep_nets.{j}.kernel"] ** 2).sum() for j in range(len(cfg.dnn_dims)))
    total = cfg.retrieval_weight * ret + cfg.rating_weight * mse + cfg.ctr_weight * ctr + reg
    total.backward()
    return float(total), {k: t.grad.numpy() for k, t in T.items()}


@pytest.mark.parametrize("mode", [0, 1])
def test_oracle_grads_match_torch_autograd(mode):
    O, cfg, P, uid, iid, rating, yi = small_setup()
    cw = {0: 0.7, 1: 1.6}
    out = O.loss_and_grads(P, cfg, uid, iid, rating, yi, cw, ctr_mode=mode)
    tot, G = torch_objective(P, cfg, uid, iid, rating, yi, cw, mode)
    assert abs(out["total_loss"] - tot) < 1e-10 * max(1, abs(tot))
    for k, g in out["grads"].items():
        if isinstance(g, tuple):
            dense = np.zeros_like(P[k])
            np.add.at(dense, g[0], g[1])
            g = dense
        assert np.allclose(g, G[k], rtol=1e-8, atol=1e-11), k


def test_oracle_finite_differences():
    O, cfg, P, uid, iid, rating, yi = small_setup(seed=3)
    cw = {0: 1.0, 1: 1.0}
    G = O.loss_and_grads(P, cfg, uid, iid, rating, yi, cw)["grads"]
    rng = np.random.default_rng(0)
    for name in ("dcn.cross_w", "encoder.user_tower.layers.0.kernel", "ctr_head.kernel"):
        for _ in range(3):
            idx = tuple(rng.integers(0, s) for s in P[name].shape)
            h = 1e-6
            P[name][idx] += h
            lp = O.loss_and_grads(P, cfg, uid, iid, rating, yi, cw, with_grads=False)["total_loss"]
            P[name][idx] -= 2 * h
            lm = O.loss_and_grads(P, cfg, uid, iid, rating, yi, cw, with_grads=False)["total_loss"]
            P[name][idx] += h
            fd = (lp - lm) / (2 * h)
            assert abs(fd - G[name][idx]) < 1e-5 * max(1.0, abs(fd)), (name, idx, fd, G[name][idx])


def test_sparse_adagrad_equals_dense_when_ids_unique():
    O = oracle()
    rng = np.random.default_rng(1)
    V, D = 30, 4
    ids = rng.permutation(V)[:10]
    rows = rng.standard_normal((10, D))
    P1 = {"e": rng.standard_normal((V, D))}
    P2 = {"e": P1["e"].copy()}
    A1 = {"e": np.full((V, D), 0.1)}
    A2 = {"e": np.full((V, D), 0.1)}
    O.adagrad_apply(P1, A1, {"e": (ids, rows)}, 0, 0.1, clipnorm=None)
    dense = np.zeros((V, D))
    dense[ids] = rows
    # dense Adagrad touches every row's accumulator with g = 0: the result is identical
    O.adagrad_apply(P2, A2, {"e": dense}, 0, 0.1, clipnorm=None)
    assert np.allclose(P1["e"], P2["e"]) and np.allclose(A1["e"], A2["e"])


def test_sparse_adagrad_dedupes_and_clips_over_raw_values():
    O = oracle()
    V, D = 5, 2
    rows = np.array([[3.0, 0.0], [4.0, 0.0]])      # ||values|| = 5 -> scale 1/5
    P = {"e": np.zeros((V, D))}
    A = {"e": np.full((V, D), 0.1)}
    O.adagrad_apply(P, A, {"e": (np.array([2, 2]), rows)}, 0, 1.0, clipnorm=1.0)
    gs = (3.0 + 4.0) / 5.0                         # deduplicated AFTER clipping
    assert np.isclose(A["e"][2, 0], 0.1 + gs * gs)
    assert np.isclose(P["e"][2, 0], -gs / math.sqrt(0.1 + gs * gs + 1e-7))
    assert np.all(P["e"][[0, 1, 3, 4]] == 0)


def test_learning_rate_staircase():
    O = oracle()
    assert O.learning_rate(0, 1e-3) == 1e-3
    assert O.learning_rate(999, 1e-3) == 1e-3
    assert np.isclose(O.learning_rate(1000, 1e-3), 0.96e-3)
    assert np.isclose(O.learning_rate(2500, 1e-3), 1e-3 * 0.96 ** 2)


def test_topk_order_is_score_desc_then_index():
    O = oracle()
    q = np.array([[1.0, 0.0]])
    items = np.array([[0.5, 1], [1.0, 0], [0.5, 2], [1.0, 5], [-1, 0]])
    sc, idx = O.topk_ip(q, items, 4)
    assert idx.tolist() == [[1, 3, 0, 2]]
    assert sc.tolist() == [[1.0, 1.0, 0.5, 0.5]]


def test_data_parallel_rule_sums_dense_and_concatenates_sparse():
    O, cfg, P, uid, iid, rating, yi = small_setup(seed=5, B=16)
    shards = [(uid[:8], iid[:8], rating[:8], yi[:8]), (uid[8:], iid[8:], rating[8:], yi[8:])]
    G = O.data_parallel_grads(P, cfg, shards)
    g0 = O.loss_and_grads(P, cfg, *shards[0])["grads"]
    g1 = O.loss_and_grads(P, cfg, *shards[1])["grads"]
    assert np.allclose(G["dcn.cross_w"], g0["dcn.cross_w"] + g1["dcn.cross_w"])
    ids, rows = G["encoder.user_embedding.weight"]
    assert np.array_equal(ids, np.concatenate([uid[:8], uid[8:]]))
    assert rows.shape == (16, cfg.embedding_dim)
    # per-replica in-batch negatives: NOT the same as one 16-row batch
    full = O.loss_and_grads(P, cfg, uid, iid, rating, yi)["grads"]
    assert not np.allclose(full["dcn.cross_w"], G["dcn.cross_w"])


def test_matrix_cross_grads_match_torch_autograd():
    O = oracle()
    rng = np.random.default_rng(8)
    B, d, L = 9, 12, 3
    x0 = rng.standard_normal((B, d))
    W = rng.standard_normal((L, d, d)) * 0.2
    b = rng.standard_normal((L, d)) * 0.1
    g = rng.standard_normal((B, d))
    xL, xs = O.cross_matrix_forward(x0, W, b)
    gx0, gW, gb = O.cross_matrix_backward(x0, xs, W, b, g)
    tx0, tW, tb = (torch.tensor(a, requires_grad=True) for a in (x0, W, b))
    xl = tx0
    for l in range(L):
        xl = tx0 * (xl @ tW[l] + tb[l]) + xl
    (xl * torch.tensor(g)).sum().backward()
    assert np.allclose(xL, xl.detach().numpy())
    assert np.allclose(gx0, tx0.grad.numpy()) and np.allclose(gW, tW.grad.numpy()) and np.allclose(gb, tb.grad.numpy())


def test_metric_suite_known_answers():
    """Hand-computed values of the src/evaluation.py definitions (first occurrence, 1/len(top_k)
    precision, ideal DCG 1, duplicates in lists, unknown truths, coverage over the union)."""
    O = oracle()
    preds = [["a", "b", "a", "c"], ["c"], [], ["d", "e"]]
    truth = ["a", "x", "q", "e"]
    r = O.metric_suite(preds, truth, [1, 3], 5)
    # k = 1: hits only for list 0 (rank 1)
    assert r[0:4] == [0.25, 0.25, 0.25, 0.25]
    # k = 3: list 0 hit at rank 1 (precision 1/3), list 3 hit at rank 2 (precision 1/2)
    assert np.allclose(r[4:8], [0.5, (1 / 3 + 1 / 2) / 4, (1 + 1 / np.log2(3)) / 4, (1 + 0.5) / 4])
    assert np.isclose(r[8], (1 + 0.5) / 4)                      # mrr
    assert np.isclose(r[9], (3 / 4 + 0 + 0 + 1) / 4)            # diversity
    assert np.isclose(r[10], 5 / 5)                             # coverage: {a,b,c,d,e}
    assert O.metric_suite([], [], [5], 3) == [0.0] * 7


def test_oracle_reproduces_committed_model_goldens():
    """tests/golden/model_goldens.npz froze the restatement; it must not drift."""
    import importlib.util
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    spec = importlib.util.spec_from_file_location("mmg", os.path.join(here, "make_model_goldens.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    fresh = mod.make()
    gold = np.load(os.path.join(here, "model_goldens.npz"))
    assert set(fresh) == set(gold.files)
    for k in gold.files:
        a, b = np.asarray(fresh[k]), gold[k]
        if a.dtype.kind in "iu":
            assert np.array_equal(a, b), k
        else:
            assert np.allclose(a, b, rtol=1e-12, atol=1e-14), k


def test_oracle_relu_gates_instrument():
    """The masks= instrument (used to compare the GPU step under its own ReLU gates): the oracle's
    own gates reproduce the plain evaluation exactly; a flipped gate changes the result like the
    ReLU with that unit's sign flipped would (finite differences under fixed gates)."""
    O, cfg, P, uid, iid, rating, yi = small_setup(seed=5)
    cw = {0: 1.0, 1: 1.3}
    base = O.loss_and_grads(P, cfg, uid, iid, rating, yi, cw)
    c = base["cache"]
    own = {"user_tower": [a > 0 for a in c["u_acts"][1:-1]], "item_tower": [a > 0 for a in c["i_acts"][1:-1]],
           "deep": [a > 0 for a in c["d_acts"][1:]]}
    same = O.loss_and_grads(P, cfg, uid, iid, rating, yi, cw, masks=own)
    assert same["total_loss"] == base["total_loss"]
    for k, g in base["grads"].items():
        g2 = same["grads"][k]
        assert np.array_equal(g[1] if isinstance(g, tuple) else g, g2[1] if isinstance(g2, tuple) else g2), k
    # flip one item-tower gate: the masked objective is smooth in the weights, and its gradient is
    # the finite difference of the masked loss
    flipped = {k: [m.copy() for m in v] for k, v in own.items()}
    flipped["item_tower"][0][3, 2] = ~flipped["item_tower"][0][3, 2]
    G = O.loss_and_grads(P, cfg, uid, iid, rating, yi, cw, masks=flipped)["grads"]
    name, idx, h = "encoder.item_tower.layers.0.bias", (2,), 1e-6
    P[name][idx] += h
    lp = O.loss_and_grads(P, cfg, uid, iid, rating, yi, cw, with_grads=False, masks=flipped)["total_loss"]
    P[name][idx] -= 2 * h
    lm = O.loss_and_grads(P, cfg, uid, iid, rating, yi, cw, with_grads=False, masks=flipped)["total_loss"]
    P[name][idx] += h
    fd = (lp - lm) / (2 * h)
    assert abs(fd - G[name][idx]) < 1e-5 * max(1.0, abs(fd))
    assert abs(G[name][idx] - base["grads"][name][idx]) > 1e-8      # the flip mattered
