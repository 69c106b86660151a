"""Parity at the sizes the bench runs (BASELINE.json configs 1, 2, 3 and 5), HIP vs the oracle.

The oracle cannot materialise everything at full size in a test's time, so each check picks
what is size-independent or sampled, always including the last rows / columns / tiles (the
ones at the largest byte offsets):

* C3 in-batch retrieval (B = 65536, D = 128, contraction precision 6, scores kept: a 17.2 GB
  buffer): lse, per-row loss and dU on sampled rows; dC on sampled columns (every row's lse is
  needed there: computed on the host in row chunks); the fp64 total against sum(lse) - sum(diag);
  kept score tiles at the start and at the end of the buffer (offsets > 2^32 bytes).
  Reference: tfrs.tasks.Retrieval (src/models.py:116,137), SURVEY Appendix A.6.
* C3 Dense weight gradient: split-K dW at K = 65536 (the tower shapes), every precision.
* C2 MultiTaskModel at the reference dims (D = 128, towers 256-128-64, dnn 256-128, L = 3) at
  B = 4096: loss, every gradient and one Adagrad step (src/models.py:105-148,
  src/trainer.py:157-163).
* C5 DCNv2Ranker at full width (26 x 128 + 13 -> d = 3344, L = 4, deep 3 x 1024) at B = 512.
* C1: the scripts/train.py-equivalent CLI at --embedding_dim 32 --batch_size 1024 on a
  reference-preprocessed pickle; its first training step against the oracle.
Tolerances are the north-star 1e-4 (conftest.assert_close: max |a - b| / max(1, max |b|), or
scale-relative with floor=0 for gradients).
"""
import os

import numpy as np
import pytest

from conftest import (assert_close, assert_flips_are_rounding, gpu_relu_masks, mask_flips, oracle, pkg, rel_err,
                      score_tiles)

pytestmark = pytest.mark.gpu

HOST_THREADS = 16          # the GPU box's CPU share


def _t(x, dev, dtype=None):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    elif t.dtype == torch.float64:
        t = t.float()
    return t.to(dev)


def _n(t):
    return t.detach().double().cpu().numpy()


def _host_threads():
    import torch
    torch.set_num_threads(max(1, min(HOST_THREADS, os.cpu_count() or 1)))


# ---------------------------------------------------------------------------------------------
# C3: in-batch softmax at B = 65536
# ---------------------------------------------------------------------------------------------
def _all_lse(U32, C32, chunk=2048):
    """lse_i = log sum_j exp(U_i . C_j) for every row: fp32 host GEMM per row chunk, the
    exponential sum in float64 (error ~1e-6, far inside the 1e-4 bar)."""
    import torch
    Ut, Ct = torch.from_numpy(U32), torch.from_numpy(C32)
    B = U32.shape[0]
    out = np.empty(B, np.float64)
    for r0 in range(0, B, chunk):
        S = Ut[r0:r0 + chunk] @ Ct.T
        m = S.max(dim=1, keepdim=True).values
        s = torch.exp(S - m).sum(dim=1, dtype=torch.float64)
        out[r0:r0 + chunk] = (m[:, 0].double() + torch.log(s)).numpy()
    return out


def _tile(S_buf, NT, it, ut):
    """32 x 32 kept-score tile (item tile it, user tile ut) -> M[user_local, item_local]
    (conftest.score_tiles)."""
    off = (it * NT + ut) * 1024
    return score_tiles(S_buf[off:off + 1024].cpu().numpy())


def test_inbatch_c3_full_batch_sampled_rows_and_columns(cuda):
    import torch
    _host_threads()
    F = pkg("functional")
    B, D, prec = 65536, 128, 6
    rng = np.random.default_rng(65536)
    U32 = (rng.standard_normal((B, D)) * 0.35).astype(np.float32)
    C32 = (rng.standard_normal((B, D)) * 0.35).astype(np.float32)
    U, C = U32.astype(np.float64), C32.astype(np.float64)
    tU, tC = _t(U32, cuda), _t(C32, cuda)
    S_buf = F.inbatch_scores_buffer(B, cuda)
    assert S_buf.numel() * 4 > (1 << 32)
    T, ROW, LSE, DU, T64 = F.inbatch_softmax_fwd(tU, tC, scores=S_buf, precision=prec)
    g = 0.75
    DUs, DC = F.inbatch_softmax_bwd(tU, tC, LSE, gscale=torch.tensor(g, device=cuda), dU_unit=DU,
                                    scores=S_buf, precision=prec)
    torch.cuda.synchronize()
    rows = np.unique(np.concatenate([np.arange(64), rng.choice(B, 192, replace=False), np.arange(B - 64, B)]))
    cols = np.unique(np.concatenate([np.arange(64), rng.choice(B, 192, replace=False), np.arange(B - 64, B)]))

    # sampled rows: lse, row loss, dU (fp64 truth)
    S_r = U[rows] @ C.T
    m = S_r.max(1, keepdims=True)
    lse_r = (m + np.log(np.exp(S_r - m).sum(1, keepdims=True)))[:, 0]
    P_r = np.exp(S_r - lse_r[:, None])
    dU_r = P_r @ C - C[rows]
    assert_close(_n(LSE)[rows], lse_r, 1e-4, "lse")
    assert_close(_n(ROW)[rows], lse_r - np.einsum("ij,ij->i", U[rows], C[rows]), 1e-4, "row loss")
    assert_close(_n(DU)[rows], dU_r, 1e-4, "dU (unit)", floor=0.0)
    assert_close(_n(DUs)[rows], g * dU_r, 1e-4, "dU", floor=0.0)

    # sampled columns: dC_j = g (sum_i P_ij U_i - U_j) needs every row's lse
    lse_all = _all_lse(U32, C32)
    assert np.abs(lse_all[rows] - lse_r).max() < 1e-5           # the chunked host lse itself
    P_c = np.exp(U @ C[cols].T - lse_all[:, None])
    dC_c = g * (P_c.T @ U - U[cols])
    assert_close(_n(DC)[cols], dC_c, 1e-4, "dC", floor=0.0)

    # whole-batch total (fp64 accumulation on the device) vs the host
    tot = float(lse_all.sum() - np.einsum("ij,ij->i", U, C).sum())
    assert abs(float(T64.item()) - tot) <= 1e-4 * max(1.0, abs(tot)), (float(T64.item()), tot)
    assert abs(float(T.item()) - tot) <= 1e-4 * max(1.0, abs(tot))

    # kept scores: first and last tiles of the 17.2 GB buffer
    NT = B // 32
    for it, ut in ((0, 0), (NT - 1, 0), (0, NT - 1), (NT - 1, NT - 1), (NT // 2, NT // 3)):
        M = _tile(S_buf, NT, it, ut)
        ref = U[32 * ut:32 * ut + 32] @ C[32 * it:32 * it + 32].T
        assert np.abs(M - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max()), (it, ut)


# ---------------------------------------------------------------------------------------------
# C3: split-K weight gradients at K = 65536
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("prec", [0, 6, 9])
@pytest.mark.parametrize("M,N", [(128, 128), (256, 128), (128, 256), (128, 64)])
def test_splitk_weight_grad_k65536(cuda, M, N, prec):
    F = pkg("functional")
    K = 65536
    rng = np.random.default_rng(M * 7 + N + prec)
    x = rng.standard_normal((K, M)).astype(np.float32)
    g = (rng.standard_normal((K, N)) * np.where(rng.random((K, 1)) < 0.5, 0.0, 1.0)).astype(np.float32)
    ref = x.astype(np.float64).T @ g.astype(np.float64)
    dW = F.gemm_splitk(_t(x, cuda), _t(g, cuda), trans_a=True, precision=prec)
    assert_close(_n(dW), ref, 1e-4, "dW", floor=0.0)


# ---------------------------------------------------------------------------------------------
# C2: the reference MultiTaskModel at the reference dims, B = 4096
# ---------------------------------------------------------------------------------------------
def test_multitask_reference_dims_b4096_step(cuda):
    import torch
    _host_threads()
    O = oracle()
    cfgm, models, optim, tr = pkg("config"), pkg("models"), pkg("optim"), pkg("trainer")
    nu, ni, B = 6040, 3706, 4096                                    # ML-1M shaped (config 2)
    cfg = cfgm.ModelConfig(embedding_dim=128, cross_layers=3, batch_size=B, learning_rate_retrieval=0.01)
    ocfg = O.OracleConfig(embedding_dim=128, cross_layers=3, learning_rate_retrieval=0.01)
    assert cfg.user_tower_dims == [256, 128, 64] and cfg.dnn_dims == [256, 128]
    P = O.init_params(ocfg, nu + 1, ni + 1, seed=11, dtype=np.float32, bias_scale=0.05)
    cw = {0: 1.6, 1: 0.73}
    model = models.MultiTaskModel(cfg, nu, ni, {}, class_weights=cw, device=cuda)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    P64 = {k: v.astype(np.float64) for k, v in P.items()}
    rng = np.random.default_rng(4096)
    uid = rng.integers(0, nu + 1, B)
    iid = rng.integers(0, ni + 1, B)
    rating = rng.integers(1, 6, B).astype(np.float32)
    yi = (rating >= 4).astype(np.float32)
    data = ({"user_id": _t(uid, cuda), "movie_id": _t(iid, cuda)},
            {"rating": _t(rating, cuda), "y_implicit": _t(yi, cuda)})
    # the step's own ReLU gates (recorded from its forward, checked against its backward) and the
    # float64 units that disagree with them
    F = pkg("functional")
    with F.record_relu_gates() as rec:
        loss, parts = model.compute_loss(data, return_parts=True)
        reg = sum(model.losses)
        (loss + reg).backward()
    gmasks = gpu_relu_masks(model, rec)
    flips = mask_flips(O, P64, ocfg, uid, iid, gmasks)
    assert_flips_are_rounding(flips)
    ref = O.loss_and_grads(P64, ocfg, uid, iid, rating.astype(np.float64), yi.astype(np.float64), cw)
    refm = O.loss_and_grads(P64, ocfg, uid, iid, rating.astype(np.float64), yi.astype(np.float64), cw, masks=gmasks)
    for got, want in ((loss, ref["loss"]), (parts["retrieval"], ref["retrieval"]), (parts["rating"], ref["rating"]),
                      (parts["ctr"], ref["ctr"])):
        assert abs(float(got) - want) <= 1e-4 * max(1.0, abs(want)), (float(got), want)
    assert abs(float(reg) - ref["reg"]) <= 1e-6
    named = dict(model.named_parameters())
    n_flips = sum(n for layers in flips.values() for n, _ in layers)
    explained = {}
    for k, gm in refm["grads"].items():
        gr = ref["grads"][k]
        if isinstance(gm, tuple):
            emb = model.encoder.user_embedding if "user" in k else model.encoder.item_embedding
            ids, got = emb.sink.gathered()
            assert np.array_equal(ids.cpu().numpy(), gm[0])
            got, gm, gr = _n(got), gm[1], gr[1]
        else:
            got = _n(named[k].grad).reshape(gm.shape)
        # the north-star 1e-4 of the gradient's scale against the float64 oracle under the GPU's
        # gates; against the oracle's own gates a miss must come with flipped units
        assert_close(got, gm, 1e-4, k, floor=0.0)
        e = rel_err(got, gr, 0.0)
        if e > 1e-4:
            assert n_flips > 0, f"{k}: {e:.3e} past 1e-4 with no flipped gate"
            explained[k] = e
    print("C2 flipped gates:", flips, "gradients past 1e-4 without the shared gates:",
          {k: f"{e:.2e}" for k, e in explained.items()} or "none")
    # the same step through the trainer's train_step + Adagrad (fresh gradients), against the
    # float64 step under the same gates
    model.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                        optim.ExponentialDecay(0.01, 1000, 0.96, True), clipnorm=1.0)
    with F.record_relu_gates() as rec2:
        out = tr.ProductionTrainer.train_step(model, opt, data)
    g2 = gpu_relu_masks(model, rec2)
    for key in gmasks:                      # the same forward: the same gates
        assert all(np.array_equal(a_, b_) for a_, b_ in zip(gmasks[key], g2[key])), key
    A = O.init_accumulators(P64)
    O.adagrad_apply(P64, A, refm["grads"], 0, ocfg.learning_rate_retrieval, clipnorm=1.0)
    assert abs(float(out["loss"]) - ref["loss"]) <= 1e-4 * max(1.0, abs(ref["loss"]))
    sd = model.state_dict()
    for k, v in P64.items():
        assert_close(_n(sd[k]), v, 1e-4, k)


# ---------------------------------------------------------------------------------------------
# C5: DCNv2Ranker at full width
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("prec", [6, 0])
def test_dcn2_ranker_full_width(cuda, prec):
    import torch
    _host_threads()
    models = pkg("models")
    O = oracle()
    nf, E, nd, L, B = 26, 128, 13, 4, 512
    deep = [1024, 1024, 1024]
    vocab = [997 + 13 * f for f in range(nf)]
    m = models.DCNv2Ranker(vocab, embedding_dim=E, num_dense=nd, cross_layers=L, deep_layers=deep, device=cuda,
                           precision=prec, seed=5)
    d = m.d
    assert d == 3344 and m.d_raw == 3341
    with torch.no_grad():                      # Keras-like small biases so every term is live
        g = torch.Generator(device="cpu").manual_seed(9)
        m.cross_b.copy_((torch.rand(m.cross_b.shape, generator=g) - 0.5) * 0.02)
        m.cross_b[:, m.d_raw:] = 0
        m.ctr_head.kernel.mul_(4.0)
    P = {k: v.detach().double().cpu().numpy() for k, v in m.state_dict().items()}
    rng = np.random.default_rng(55)
    ids = np.stack([rng.integers(0, v + 1, B) for v in vocab]).astype(np.int64)
    dense = rng.standard_normal((B, nd)).astype(np.float32)
    y = (rng.random(B) < 0.3).astype(np.float32)
    loss = m.compute_loss(_t(ids, cuda), _t(dense, cuda), _t(y, cuda))
    loss.backward()
    ref = O.dcn2_ranker_loss_and_grads(P, nf, E, d, deep, ids, dense.astype(np.float64), y.astype(np.float64))
    assert abs(float(loss) - ref["loss"]) <= 1e-4 * max(1.0, abs(ref["loss"])), (float(loss), ref["loss"])
    named = dict(m.named_parameters())
    for k, gr in ref["grads"].items():
        if isinstance(gr, tuple):
            f = int(k.split(".")[1])
            gi, grow = m.tables[f].sink.gathered()
            assert np.array_equal(gi.cpu().numpy(), gr[0])
            assert_close(_n(grow), gr[1], 1e-4, k, floor=0.0)
        else:
            assert_close(_n(named[k].grad).reshape(gr.shape), gr, 1e-4, k, floor=0.0)


# ---------------------------------------------------------------------------------------------
# C1: the training CLI (scripts/train.py flags) on a reference-preprocessed pickle
# ---------------------------------------------------------------------------------------------
def test_train_cli_c1_first_step_matches_oracle(cuda, tmp_path, monkeypatch):
    """tools/train.py --embedding_dim 32 --batch_size 1024 (config 1) on the train / val split
    that the reference's own preprocessing produced (tests/golden/data_goldens.npz); the first
    training step's loss and updated weights are checked against the oracle on the same batch
    and initial weights, then the run's artefacts are checked."""
    import importlib.util
    import json
    import sys

    import pandas as pd
    import torch
    O = oracle()
    tr = pkg("trainer")
    here = os.path.dirname(os.path.abspath(__file__))
    gold = np.load(os.path.join(here, "golden", "data_goldens.npz"))
    train = pd.DataFrame({"user_id": gold["train_user_id"], "movie_id": gold["train_movie_id"],
                          "rating": gold["train_rating"].astype(np.int64),
                          "y_implicit": gold["train_y_implicit"].astype(np.int64),
                          "timestamp": np.zeros(len(gold["train_user_id"]), np.int64)})
    val = pd.DataFrame({"user_id": gold["val_user_id"], "movie_id": gold["val_movie_id"],
                        "rating": gold["val_rating"].astype(np.int64),
                        "y_implicit": gold["val_y_implicit"].astype(np.int64),
                        "timestamp": np.zeros(len(gold["val_user_id"]), np.int64)})
    pkl = tmp_path / "processed_data.pkl"
    pd.to_pickle({"train_ratings": train, "val_ratings": val, "test_ratings": val,
                  "user_features": {}, "movie_features": {}}, pkl)

    seen = {}
    orig = tr.ProductionTrainer.train_step

    def spy(model, opt, batch):
        if not seen:
            seen["P"] = {k: v.detach().double().cpu().numpy() for k, v in model.state_dict().items()}
            seen["batch"] = [{k: v.cpu().numpy() for k, v in part.items()} for part in batch]
            seen["cw"] = dict(model.class_weights)
            seen["cfg"] = model.config
            out = orig(model, opt, batch)
            seen["loss"] = float(out["loss"])
            seen["P1"] = {k: v.detach().double().cpu().numpy() for k, v in model.state_dict().items()}
            return out
        return orig(model, opt, batch)

    monkeypatch.setattr(tr.ProductionTrainer, "train_step", staticmethod(spy))
    spec = importlib.util.spec_from_file_location("train_cli", os.path.join(os.path.dirname(here), "tools", "train.py"))
    cli = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cli)
    out_dir = tmp_path / "out"
    monkeypatch.setattr(sys, "argv", ["train.py", "--data", str(pkl), "--output_dir", str(out_dir),
                                      "--embedding_dim", "32", "--batch_size", "1024", "--epochs", "1"])
    cli.main()

    cfg = seen["cfg"]
    assert cfg.embedding_dim == 32 and cfg.batch_size == 1024 and cfg.cross_layers == 1   # CLI defaults
    assert seen["cw"] == pytest.approx({0: float(gold["class_weights"][0]), 1: float(gold["class_weights"][1])})
    feats, labels = seen["batch"]
    assert feats["user_id"].shape == (1024,)
    ocfg = O.OracleConfig(embedding_dim=32, cross_layers=1, learning_rate_retrieval=cfg.learning_rate_retrieval,
                          ctr_weight=cfg.ctr_weight, rating_weight=cfg.rating_weight)
    P = seen["P"]
    A = O.init_accumulators(P)
    ref = O.train_step(P, A, ocfg, 0, feats["user_id"], feats["movie_id"], labels["rating"].astype(np.float64),
                       labels["y_implicit"].astype(np.float64), seen["cw"])
    assert abs(seen["loss"] - ref["loss"]) <= 1e-4 * max(1.0, abs(ref["loss"])), (seen["loss"], ref["loss"])
    for k, v in P.items():
        assert_close(seen["P1"][k], v, 1e-4, k)
    for f in ("best_model.pt", "training_log.csv", "metrics.json", "encoder.pt", "vocabs.json", "config.json",
              "config_ext.json", "faiss.idx", "item_map.json"):
        assert (out_dir / f).exists(), f
    # config.json keeps the reference schema: ModelConfig(**json) of the reference's fields
    cj = json.load(open(out_dir / "config.json"))
    assert set(cj) == set(pkg("config").REFERENCE_FIELDS)
    torch.cuda.synchronize()
