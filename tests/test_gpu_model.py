"""Model-level parity on the GPU: the reference constructor API (MultiTaskModel / MultiTowerModel
/ DeepCrossNetwork / ProductionTrainer) running on the HIP kernels vs the CPU oracle with the
same weights and inputs (fp32; tolerance 1e-4 on logits/losses, scaled as conftest.assert_close).
"""
import numpy as np
import pytest

from conftest import assert_close, oracle, pkg

pytestmark = pytest.mark.gpu


def build(cuda, D=32, L=2, nu=60, ni=45, seed=1, mode="per_sample", towers=None, dnn=None):
    import torch
    O = oracle()
    cfgm = pkg("config")
    models = pkg("models")
    towers = towers or [64, 48, 32]
    dnn = dnn or [64, 32]
    cfg = cfgm.ModelConfig(embedding_dim=D, cross_layers=L, user_tower_dims=list(towers),
                           item_tower_dims=list(towers), dnn_dims=list(dnn), ctr_loss_mode=mode)
    ocfg = O.OracleConfig(embedding_dim=D, cross_layers=L, user_tower_dims=list(towers),
                          item_tower_dims=list(towers), dnn_dims=list(dnn))
    P = O.init_params(ocfg, nu + 1, ni + 1, seed=seed, dtype=np.float32, bias_scale=0.05)
    cw = {0: 0.75, 1: 1.5}
    model = models.MultiTaskModel(cfg, [str(i) for i in range(nu)], [str(i) for i in range(ni)], {},
                                  class_weights=cw, device=cuda)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    P64 = {k: v.astype(np.float64) for k, v in P.items()}
    return O, cfg, ocfg, model, P64, cw


def batch(cuda, B, nu, ni, seed=0):
    import torch
    rng = np.random.default_rng(seed)
    uid = rng.integers(0, nu + 1, B)
    iid = rng.integers(0, ni + 1, B)
    rating = rng.integers(1, 6, B).astype(np.float32)
    yi = (rating >= 4).astype(np.float32)
    feats = {"user_id": torch.from_numpy(uid).to(cuda), "movie_id": torch.from_numpy(iid).to(cuda)}
    labels = {"rating": torch.from_numpy(rating).to(cuda), "y_implicit": torch.from_numpy(yi).to(cuda)}
    return (feats, labels), (uid, iid, rating.astype(np.float64), yi.astype(np.float64))


def n(t):
    return t.detach().double().cpu().numpy()


@pytest.mark.parametrize("B", [1, 37, 256])
def test_forward_matches_oracle(cuda, B):
    O, cfg, ocfg, model, P, cw = build(cuda)
    data, (uid, iid, _, _) = batch(cuda, B, 60, 45, seed=B)
    out = model(data)
    c = O.forward(P, ocfg, uid, iid)
    assert_close(n(out["user_embedding"]), c["U"], 1e-5, "U")
    assert_close(n(out["item_embedding"]), c["C"], 1e-5, "C")
    assert_close(n(out["rating_prediction"]), c["r"], 1e-5, "rating")
    assert_close(n(out["ctr_prediction"]), c["p"], 1e-5, "ctr")


@pytest.mark.parametrize("mode", ["per_sample", "keras3"])
@pytest.mark.parametrize("B,D", [(64, 32), (300, 64), (129, 128)])
def test_loss_and_all_gradients_match_oracle(cuda, mode, B, D):
    O, cfg, ocfg, model, P, cw = build(cuda, D=D, mode=mode)
    data, (uid, iid, rating, yi) = batch(cuda, B, 60, 45, seed=D + B)
    loss, parts = model.compute_loss(data, return_parts=True)
    reg = sum(model.losses)
    (loss + reg).backward()
    ref = O.loss_and_grads(P, ocfg, uid, iid, rating, yi, cw, ctr_mode=0 if mode == "per_sample" else 1)
    assert abs(float(loss) - ref["loss"]) <= 1e-4 * max(1.0, abs(ref["loss"]))
    assert abs(float(parts["retrieval"]) - ref["retrieval"]) <= 1e-4 * max(1.0, abs(ref["retrieval"]))
    assert abs(float(parts["rating"]) - ref["rating"]) <= 1e-4 * max(1.0, ref["rating"])
    assert abs(float(parts["ctr"]) - ref["ctr"]) <= 1e-4 * max(1.0, ref["ctr"])
    assert abs(float(reg) - ref["reg"]) <= 1e-6
    named = dict(model.named_parameters())
    for k, g in ref["grads"].items():
        if isinstance(g, tuple):
            emb = model.encoder.user_embedding if "user" in k else model.encoder.item_embedding
            ids, rows = emb.sink.gathered()
            assert np.array_equal(ids.cpu().numpy(), g[0])
            assert_close(n(rows), g[1], 1e-4, k, floor=0.0)
            assert named[k].grad is None          # never a dense [V, D] gradient
        else:
            assert_close(n(named[k].grad).reshape(g.shape), g, 1e-4, k, floor=0.0)


def test_three_train_steps_match_oracle(cuda):
    optim = pkg("optim")
    tr = pkg("trainer")
    O, cfg, ocfg, model, P, cw = build(cuda, D=64, L=3)
    opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                        optim.ExponentialDecay(0.05, 1000, 0.96, True), clipnorm=1.0)
    A = O.init_accumulators(P)
    ocfg.learning_rate_retrieval = 0.05
    for step in range(3):
        data, (uid, iid, rating, yi) = batch(cuda, 200, 60, 45, seed=100 + step)
        out = tr.ProductionTrainer.train_step(model, opt, data)
        ref = O.train_step(P, A, ocfg, step, uid, iid, rating, yi, cw)
        assert abs(float(out["loss"]) - ref["loss"]) <= 1e-4 * max(1.0, abs(ref["loss"]))
    sd = model.state_dict()
    for k, v in P.items():
        assert_close(n(sd[k]), v, 1e-4, k)
    assert int(opt.iterations.item()) == 3


def test_string_ids_equal_int_fast_path(cuda):
    import torch
    O, cfg, ocfg, model, P, cw = build(cuda)
    users = np.array(["3", "17", "unknown", "59", "0"])
    items = np.array(["44", "1", "2", "nope", "10"])
    a = model.encoder({"user_id": users, "movie_id": items})
    ids_u = torch.tensor([4, 18, 0, 60, 1], device=cuda)        # 1 + position; OOV -> 0
    ids_i = torch.tensor([45, 2, 3, 0, 11], device=cuda)
    b = model.encoder({"user_id": ids_u, "movie_id": ids_i})
    assert np.array_equal(n(a["user_embedding"]), n(b["user_embedding"]))
    assert np.array_equal(n(a["item_embedding"]), n(b["item_embedding"]))
    only_user = model.encoder({"user_id": users})
    assert only_user["item_embedding"] is None


def test_deep_cross_network_standalone_api(cuda):
    import torch
    O = oracle()
    models = pkg("models")
    dcn = models.DeepCrossNetwork(cross_layers=2, deep_layers=[64, 32], l2_reg=1e-5, device=cuda)
    x = torch.randn(50, 128, device=cuda) * 0.2
    y = dcn(x)                                   # builds lazily like Keras (d = 128)
    assert y.shape == (50, 128 + 32)
    xn = n(x)
    xl, _, _ = O.cross_forward(xn, n(dcn.cross_w), n(dcn.cross_b))
    h, _ = O.mlp_forward(xn, [(n(l.kernel), n(l.bias)) for l in dcn.deep_nets], relu_last=True)
    assert_close(n(y), np.concatenate([xl, h], 1), 1e-5, "dcn")
    assert dcn.cross_weight(1).shape == (128, 1)
    assert dcn.get_config()["deep_layers"] == [64, 32]


def test_training_is_bitwise_deterministic(cuda):
    import torch
    optim = pkg("optim")
    tr = pkg("trainer")
    finals = []
    for _ in range(2):
        O, cfg, ocfg, model, P, cw = build(cuda, D=128, L=3, nu=500, ni=300)
        opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(), 0.05, clipnorm=1.0)
        for step in range(3):
            data, _ = batch(cuda, 1024, 500, 300, seed=step)
            tr.ProductionTrainer.train_step(model, opt, data)
        torch.cuda.synchronize()
        finals.append({k: v.clone() for k, v in model.state_dict().items()})
    for k in finals[0]:
        assert torch.equal(finals[0][k], finals[1][k]), k


def test_brute_force_index_cosine_and_recall(cuda):
    import torch
    O = oracle()
    retrieval = pkg("retrieval")
    rng = np.random.default_rng(0)
    items = rng.integers(-8, 9, (2000, 64)).astype(np.float32) / 16
    q = rng.integers(-8, 9, (20, 64)).astype(np.float32) / 16
    idx = retrieval.BruteForceIndex(64, "ip", cuda)
    idx.add(items)
    s, i = idx.search(q, 50)
    _, oi = O.topk_ip(q, items, 50)
    assert np.array_equal(i.cpu().numpy(), oi)
    true = oi[:, 7].copy()
    true[:5] = 1999 - true[:5]                # some misses
    rec = retrieval.recall_at_k(torch.from_numpy(items).to(cuda), torch.from_numpy(q).to(cuda), true, [5, 10, 50])
    for k in (5, 10, 50):
        expect = np.mean([(true[r] in oi[r, :k]) for r in range(20)])
        assert rec[f"recall@{k}"] == pytest.approx(expect)
    cos = retrieval.BruteForceIndex(64, "cosine", cuda)
    cos.add(items)
    _, ci = cos.search(q, 10)
    nrm = items / np.maximum(np.linalg.norm(items, axis=1, keepdims=True), 1e-12)
    qn = q / np.linalg.norm(q, axis=1, keepdims=True)
    sims = qn.astype(np.float64) @ nrm.T.astype(np.float64)
    for r in range(20):  # cosine scores are not dyadic: compare score sets, allow near-ties
        top = np.sort(sims[r])[::-1][:10]
        got = sims[r][ci[r].cpu().numpy()]
        assert np.allclose(np.sort(got)[::-1], top, atol=1e-6)


def test_trainer_end_to_end(cuda, tmp_path):
    import json
    import pandas as pd
    cfgm = pkg("config")
    tr = pkg("trainer")
    rng = np.random.default_rng(0)
    n_rows = 6000

    def frame(k, seed):
        r = np.random.default_rng(seed)
        return pd.DataFrame({"user_id": r.integers(0, 300, k), "movie_id": r.integers(0, 200, k),
                             "rating": r.integers(1, 6, k), "timestamp": r.integers(0, 10 ** 9, k)})

    train = frame(n_rows, 1)
    train["y_implicit"] = (train["rating"] >= 4).astype(int)
    val = frame(800, 2)
    val["y_implicit"] = (val["rating"] >= 4).astype(int)
    pkl = tmp_path / "processed.pkl"
    pd.to_pickle({"train_ratings": train, "val_ratings": val, "test_ratings": val,
                  "user_features": {}, "movie_features": {}}, pkl)
    cfg = cfgm.ModelConfig(embedding_dim=32, cross_layers=1, batch_size=512, epochs_retrieval=3,
                           ctr_weight=0.2, rating_weight=0.2)
    trainer = tr.ProductionTrainer(cfg, str(tmp_path / "out"))
    model, history = trainer.train(str(pkl))
    assert len(history.history["loss"]) == 3 and len(history.history["val_loss"]) == 3
    assert all(np.isfinite(history.history["val_loss"]))
    out = tmp_path / "out"
    for f in ("best_model.pt", "training_log.csv", "metrics.json", "encoder.pt", "vocabs.json", "config.json",
              "faiss.idx", "item_map.json", "detailed_metrics.json"):
        assert (out / f).exists(), f
    metrics = json.load(open(out / "metrics.json"))
    assert set(metrics) == {"recall@5", "recall@10", "recall@20", "recall@50"}
    vocabs = json.load(open(out / "vocabs.json"))
    assert vocabs["users"] == sorted(vocabs["users"])
    assert json.load(open(out / "config.json"))["embedding_dim"] == 32


@pytest.mark.parametrize("packed", [False, True])
def test_graphed_train_step_is_bitwise_identical_to_eager(cuda, packed):
    import torch
    optim = pkg("optim")
    tr = pkg("trainer")
    graphs = pkg("graphs")
    finals = []
    mk = (lambda s: graphs.pack_batch(batch(cuda, 512, 400, 300, seed=s)[0])) if packed else \
        (lambda s: batch(cuda, 512, 400, 300, seed=s)[0])
    for mode in ("eager", "graph"):
        O, cfg, ocfg, model, P, cw = build(cuda, D=64, L=3, nu=400, ni=300)
        opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                            optim.ExponentialDecay(0.05, 2, 0.5, True), clipnorm=1.0)  # lr decays every 2 steps
        step = lambda b: tr.ProductionTrainer.train_step(model, opt, b)  # noqa: E731
        runner = graphs.GraphedTrainStep(step, mk(0)) if mode == "graph" else step
        if mode == "graph":   # the packed static copy (one memcpy per replay) only for pack_batch batches
            assert (graphs._packed_storage(runner.static) is not None) == packed
        losses = []
        for i in range(5):
            out = runner(mk(i))
            losses.append(float(out["loss"]))
        torch.cuda.synchronize()
        assert int(opt.iterations.item()) == 5
        finals.append(({k: v.clone() for k, v in model.state_dict().items()}, losses))
    assert finals[0][1] == finals[1][1]
    for k in finals[0][0]:
        assert torch.equal(finals[0][0][k], finals[1][0][k]), k


def test_model_matches_committed_goldens(cuda):
    """The GPU path against the frozen model-side golden vectors (tests/golden/model_goldens.npz):
    activations, scores, losses, every gradient and one Adagrad step."""
    import os
    import torch
    cfgm = pkg("config")
    models = pkg("models")
    optim = pkg("optim")
    gold = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "model_goldens.npz"))
    P = {k[3:]: gold[k] for k in gold.files if k.startswith("P::")}
    nu = P["encoder.user_embedding.weight"].shape[0] - 1
    ni = P["encoder.item_embedding.weight"].shape[0] - 1
    cfg = cfgm.ModelConfig(embedding_dim=16, user_tower_dims=[32, 16], item_tower_dims=[32, 16], cross_layers=2,
                           dnn_dims=[16, 8])
    model = models.MultiTaskModel(cfg, [str(i) for i in range(nu)], [str(i) for i in range(ni)], {},
                                  class_weights={0: 0.8, 1: 1.4}, device=cuda)
    model.load_state_dict({k: torch.from_numpy(v.astype(np.float32)) for k, v in P.items()})
    feats = {"user_id": torch.from_numpy(gold["uid"]).to(cuda), "movie_id": torch.from_numpy(gold["iid"]).to(cuda)}
    labels = {"rating": torch.from_numpy(gold["rating"].astype(np.float32)).to(cuda),
              "y_implicit": torch.from_numpy(gold["y_implicit"].astype(np.float32)).to(cuda)}
    out = model(feats)
    assert_close(n(out["user_embedding"]), gold["U"], 1e-4, "U")
    assert_close(n(out["item_embedding"]), gold["C"], 1e-4, "C")
    assert_close(n(out["rating_prediction"]), gold["r"], 1e-4, "rating")
    assert_close(n(out["ctr_prediction"]), gold["p"], 1e-4, "ctr")
    loss, parts = model.compute_loss((feats, labels), return_parts=True)
    reg = sum(model.losses)
    assert abs(float(loss) - float(gold["loss"])) <= 1e-4 * max(1.0, abs(float(gold["loss"])))
    assert abs(float(parts["retrieval"]) - float(gold["loss_retrieval"])) <= 1e-4 * max(1.0, float(gold["loss_retrieval"]))
    assert abs(float(reg) - float(gold["reg"])) <= 1e-6
    opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(), 0.02, clipnorm=1.0)
    opt.zero_grad()
    (loss + reg).backward()
    named = dict(model.named_parameters())
    for k in gold.files:
        if k.startswith("g::"):
            name = k[3:]
            assert_close(n(named[name].grad).reshape(gold[k].shape), gold[k], 1e-4, name, floor=0.0)
        elif k.startswith("gids::"):
            name = k[6:]
            emb = model.encoder.user_embedding if "user" in name else model.encoder.item_embedding
            ids, rows = emb.sink.gathered()
            assert np.array_equal(ids.cpu().numpy(), gold[k])
            assert_close(n(rows), gold["grows::" + name], 1e-4, name, floor=0.0)
    opt.step()
    for k in gold.files:
        if k.startswith("P1::"):
            assert_close(n(dict(model.state_dict())[k[4:]]), gold[k], 1e-4, k, floor=0.0)


@pytest.mark.parametrize("graphed", [False, True])
def test_deferred_reductions_bitwise_equal(cuda, graphed):
    """Adagrad(defer_reductions=True): the gradient reductions of the backward (Dense stacks,
    DCN-v1 cross, heads) are queued in the optimizer's own ReductionQueue and run as one launch at
    the top of step(); five training steps end bitwise equal to the undeferred steps, eager and
    graph-captured, and the queue is empty after every step."""
    import torch
    optim = pkg("optim")
    tr = pkg("trainer")
    graphs = pkg("graphs")
    finals = []
    for defer in (False, True):
        O, cfg, ocfg, model, P, cw = build(cuda, D=64, L=3, nu=400, ni=300)
        opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                            optim.ExponentialDecay(0.05, 2, 0.5, True), clipnorm=1.0, defer_reductions=defer)
        assert (opt._rq is not None) == defer
        step = lambda b: tr.ProductionTrainer.train_step(model, opt, b)  # noqa: E731
        runner = graphs.GraphedTrainStep(step, batch(cuda, 512, 400, 300, seed=0)[0]) if graphed else step
        losses = []
        for i in range(5):
            if i == 0 and defer and not graphed:   # the backward (on autograd's worker thread) queues
                b0 = batch(cuda, 512, 400, 300, seed=0)[0]
                opt.zero_grad()
                loss = model.compute_loss(b0, training=True)
                (loss + model.losses[0]).backward()
                assert opt._rq.pending() >= 8   # Dense stacks, cross, heads
                opt.step()
                losses.append(float(loss))
            else:
                out = runner(batch(cuda, 512, 400, 300, seed=i)[0])
                losses.append(float(out["loss"]))
            if defer:
                assert opt._rq.pending() == 0
        torch.cuda.synchronize()
        finals.append(({k: v.clone() for k, v in model.state_dict().items()}, losses))
    assert finals[0][1] == finals[1][1]
    for k in finals[0][0]:
        assert torch.equal(finals[0][0][k], finals[1][0][k]), k


def test_deferred_reductions_queue_and_errors(cuda):
    """Queued reductions write exactly the immediate result at the flush; an op given a closed
    queue (or none) launches at once; a flush with nothing queued is a no-op; flushing on another
    stream than the jobs' is refused."""
    import torch
    F = pkg("functional")
    native = pkg("_native")
    rng = np.random.default_rng(2)
    x = torch.from_numpy(rng.standard_normal((3000, 64)).astype(np.float32)).to(cuda)
    g = torch.from_numpy(rng.standard_normal((3000, 96)).astype(np.float32)).to(cuda)
    ref_w, ref_b = F.gemm_wgrad_bias(x, g, 6)
    q = F.ReductionQueue()
    F.gemm_wgrad_bias(x, g, 6, queue=q)                  # closed queue: launched at once
    assert q.pending() == 0
    q.open()
    dW, db = F.gemm_wgrad_bias(x, g, 6, queue=q)
    assert q.pending() == 1
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        with pytest.raises(native.NativeError, match="another stream"):
            native.call("rs_reduction_queue_flush", q.handle, F._stream())
    q.flush()
    assert q.pending() == 0 and not q.active
    assert torch.equal(dW, ref_w) and torch.equal(db, ref_b)
    q.flush()


def test_deferred_reductions_each_op_bitwise(cuda):
    """Every deferrable reduction, queued together and flushed once, equals its immediate form
    bitwise: the towers' grouped dW + db, the deep net's dW + db with the l2 addend, ReLU-masked
    column sums, the DCN-v1 cross and the heads' parameter gradients."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(12)
    t = lambda *s: torch.from_numpy(rng.standard_normal(s).astype(np.float32)).to(cuda)  # noqa: E731
    B = 2048
    x, g, W, dsc = t(B, 64), t(B, 96), t(64, 96), t(1).reshape(())
    xs, gs = [t(B, 128), t(B, 128)], [t(B, 64), t(B, 64)]
    dy, y = t(B, 72), t(B, 72)
    x0, s_, w, b, gxl = t(B, 128), t(B, 3), t(3, 128), t(3, 128), t(B, 128)
    xl, h, wr, wc, p, gr, gp = t(B, 128), t(B, 64), t(192, 1), t(192, 1), t(B, 1).sigmoid(), t(B, 1), t(B, 1)

    def run(q=None):
        out = list(F.gemm_wgrad_bias(x, g, 6, W=W, w_scale=0.3, w_dscale=dsc, queue=q))
        for a_, b_ in F.gemm_wgrad_bias_group(xs, gs, 6, queue=q):
            out += [a_, b_]
        out += list(F.relu_bwd_colsum(dy, y, queue=q))
        out += list(F.dcn_cross_bwd(x0, s_, w, b, gxl, queue=q))
        out += list(F.heads_bwd(xl, h, wr, wc, p, g_r=gr, g_p=gp, queue=q))
        return out
    ref = [o.clone() for o in run()]
    torch.cuda.synchronize()
    q = F.ReductionQueue()
    q.open()
    got = run(q)
    assert q.pending() == 1 + 1 + 1 + 2 + 4
    q.flush()
    torch.cuda.synchronize()
    for i, (a_, b_) in enumerate(zip(got, ref)):
        assert torch.equal(a_, b_), i


def test_two_models_two_streams_defer_concurrently(cuda):
    """Two MultiTaskModels, each with its own deferring Adagrad, trained on two streams with their
    steps interleaved (model A's backward queued, then model B's zero_grad / backward / step on the
    other stream, then A's step): each ends bitwise equal to the same model trained alone and
    undeferred. The queues are the optimizers' own, so neither ever sees the other's jobs."""
    import torch
    optim = pkg("optim")
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def make(seed, defer):
        O, cfg, ocfg, model, P, cw = build(cuda, D=64, L=3, nu=400, ni=300, seed=seed)
        opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                            optim.ExponentialDecay(0.05, 2, 0.5, True), clipnorm=1.0, defer_reductions=defer)
        return model, opt

    def fwd_bwd(model, opt, b):
        opt.zero_grad()
        loss = model.compute_loss(b, training=True)
        (loss + model.losses[0]).backward()
        return loss

    alone = []
    for seed in (1, 2):
        model, opt = make(seed, False)
        for i in range(3):
            fwd_bwd(model, opt, batch(cuda, 512, 400, 300, seed=10 * seed + i)[0])
            opt.step()
        torch.cuda.synchronize()
        alone.append({k: v.clone() for k, v in model.state_dict().items()})

    (ma, oa), (mb, ob) = make(1, True), make(2, True)
    assert oa._rq is not ob._rq
    for i in range(3):
        ba, bb = batch(cuda, 512, 400, 300, seed=10 + i)[0], batch(cuda, 512, 400, 300, seed=20 + i)[0]
        for st in streams:
            st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(streams[0]):
            fwd_bwd(ma, oa, ba)
        na = oa._rq.pending()
        assert na >= 8
        with torch.cuda.stream(streams[1]):
            fwd_bwd(mb, ob, bb)
            assert ob._rq.pending() == na and oa._rq.pending() == na   # B queued into its own queue
            ob.step()
        assert ob._rq.pending() == 0 and oa._rq.pending() == na
        with torch.cuda.stream(streams[0]):
            oa.step()
        assert oa._rq.pending() == 0
        for st in streams:
            torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    for ref, model in zip(alone, (ma, mb)):
        sd = model.state_dict()
        for k in ref:
            assert torch.equal(ref[k], sd[k]), k


def test_abandoned_deferring_optimizer_never_holds_gradients(cuda):
    """a deferring Adagrad whose step was abandoned after zero_grad() (its queue left
    open) is replaced by a new optimizer, deferring or not, for the same model: training then ends
    bitwise equal to a model that never had the abandoned optimizer (no gradient is queued into the
    orphaned queue), and the replacement raises no error."""
    import torch
    optim = pkg("optim")
    tr = pkg("trainer")
    finals = []
    for case in ("plain", "after_deferring", "after_plain_replacement"):
        O, cfg, ocfg, model, P, cw = build(cuda, D=64, L=3, nu=400, ni=300)
        if case != "plain":
            old = optim.Adagrad(model.dense_parameters(), model.embedding_modules(), 0.05, clipnorm=1.0,
                                defer_reductions=True)
            old.zero_grad()                  # the queue is open; the step never comes
            assert old._rq.active
        opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(), 0.05, clipnorm=1.0,
                            defer_reductions=(case == "after_deferring"))
        if case != "plain":
            assert not old._rq.active
        for i in range(3):
            tr.ProductionTrainer.train_step(model, opt, batch(cuda, 512, 400, 300, seed=i)[0])
        if case != "plain":
            assert old._rq.pending() == 0
        torch.cuda.synchronize()
        finals.append({k: v.clone() for k, v in model.state_dict().items()})
    for other in finals[1:]:
        for k in finals[0]:
            assert torch.equal(finals[0][k], other[k]), k


def test_deferred_step_peak_memory_not_above_undeferred(cuda):
    """While reductions are deferred only the workspaces of queued jobs are held to the flush (the
    in-batch, gather and forward workspaces go back to the caching allocator at once): a deferred
    step's peak device memory is the undeferred step's within 2 %, at a C3-like batch."""
    import torch
    optim = pkg("optim")
    cfgm, models = pkg("config"), pkg("models")
    B = 16384
    rng = np.random.default_rng(8)
    feats = {"user_id": torch.from_numpy(((rng.zipf(1.1, B) * 7919) % 200000 + 1).astype(np.int64)).to(cuda),
             "movie_id": torch.from_numpy(((rng.zipf(1.1, B) * 104729) % 50000 + 1).astype(np.int64)).to(cuda)}
    rating = torch.from_numpy(rng.integers(1, 6, B).astype(np.float32)).to(cuda)
    data = (feats, {"rating": rating, "y_implicit": (rating >= 4).float()})
    peaks = {}
    for defer in (False, True):
        model = models.MultiTaskModel(cfgm.ModelConfig(embedding_dim=128), 200000, 50000, {}, seed=3, device=cuda)
        opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(), 0.01, clipnorm=1.0,
                            defer_reductions=defer)
        for i in range(2):
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats()
            base = torch.cuda.memory_allocated()
            opt.zero_grad()
            loss = model.compute_loss(data, training=True)
            (loss + model.losses[0]).backward()
            opt.step()
            torch.cuda.synchronize()
            peaks[defer] = torch.cuda.max_memory_allocated() - base
        del model, opt, loss
        torch.cuda.empty_cache()
    assert peaks[True] <= 1.02 * peaks[False], peaks


@pytest.mark.parametrize("with_ctr", [True, False])
def test_loss_node_with_regularization_equals_separate_add(cuda, with_ctr):
    """compute_loss(with_regularization=True) forms loss + sum(model.losses) inside the loss node
    (rs_ranking_losses_combine_f32 / rs_heads_bwd_combine_f32); its (loss, total, reg) and every
    gradient equal the separate `loss + reg` backward bitwise, with and without CTR labels."""
    import torch
    res = []
    for fused in (False, True):
        O, cfg, ocfg, model, P, cw = build(cuda, D=64, L=3, nu=400, ni=300)
        data, _ = batch(cuda, 700, 400, 300, seed=9)
        if not with_ctr:
            data = (data[0], {"rating": data[1]["rating"]})
        if fused:
            loss, total, reg = model.compute_loss(data, training=True, with_regularization=True)
        else:
            loss = model.compute_loss(data, training=True)
            reg = model.losses[0]
            total = loss + reg
        total.backward()
        g = {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
        g.update({f"sink{j}": e.sink.gathered()[1].clone() for j, e in enumerate(model.embedding_modules())})
        res.append((loss.detach().clone(), total.detach().clone(), reg.detach().clone(), g))
    for j in range(3):
        assert torch.equal(res[0][j], res[1][j]), j
    assert res[0][3].keys() == res[1][3].keys()
    for k in res[0][3]:
        assert torch.equal(res[0][3][k], res[1][3][k]), k


def test_deep_top_relu_masked_in_heads_backward(cuda, monkeypatch):
    """The heads backward masks the deep net's top-layer gradient by h > 0 (RS_HEADS_RELU_H), so the
    deep net's MLPFn backward launches no relu_bwd_colsum: every gradient bitwise equal to the
    unfolded backward (heads unmasked + relu_bwd_colsum), and no relu_bwd_colsum call left."""
    import torch
    F = pkg("functional")
    orig_apply = F.HeadsLossTotalFn.apply
    calls = []
    orig_rbc = F.relu_bwd_colsum

    def counting_rbc(*a, **k):
        calls.append(1)
        return orig_rbc(*a, **k)

    monkeypatch.setattr(F, "relu_bwd_colsum", counting_rbc)
    res, ncalls = [], []
    for fold in (False, True):
        if fold:
            monkeypatch.setattr(F.HeadsLossTotalFn, "apply", orig_apply)
        else:
            monkeypatch.setattr(F.HeadsLossTotalFn, "apply", lambda *a: orig_apply(*a[:-1], False))
        calls.clear()
        O, cfg, ocfg, model, P, cw = build(cuda, D=64, L=3, nu=400, ni=300)
        data, _ = batch(cuda, 700, 400, 300, seed=11)
        loss, total, reg = model.compute_loss(data, training=True, with_regularization=True)
        total.backward()
        g = {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
        g.update({f"sink{j}": e.sink.gathered()[1].clone() for j, e in enumerate(model.embedding_modules())})
        res.append((total.detach().clone(), g))
        ncalls.append(len(calls))
    assert ncalls == [1, 0], ncalls
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][1].keys() == res[1][1].keys()
    for k in res[0][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k


def test_prepared_stack_images_bitwise(cuda, monkeypatch):
    """compute_loss builds the towers' and the deep net's weight images in one launch
    (functional.prepare_mlp_images) and each stack node takes its own: two training steps end
    bitwise equal to the per-node image builds, and no prepared image outlives its forward."""
    import torch
    optim = pkg("optim")
    tr = pkg("trainer")
    F = pkg("functional")
    finals, taken = [], []
    real = F.mlp_weight_image

    def spy(W_lists):
        taken.append(F._image_key(W_lists) in F._PREPARED_IMAGES)
        return real(W_lists)
    monkeypatch.setattr(F, "mlp_weight_image", spy)
    for prep in (False, True):
        monkeypatch.setattr(F, "MLP_PREPARE", prep)
        taken.clear()
        O, cfg, ocfg, model, P, cw = build(cuda, D=64, L=3, nu=400, ni=300, towers=[128, 64, 64], dnn=[64, 64])
        opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                            optim.ExponentialDecay(0.05, 2, 0.5, True), clipnorm=1.0)
        for i in range(2):
            tr.ProductionTrainer.train_step(model, opt, batch(cuda, 512, 400, 300, seed=i)[0])
        torch.cuda.synchronize()
        assert not F._PREPARED_IMAGES
        assert taken and all(t == prep for t in taken), taken
        finals.append({k: v.clone() for k, v in model.state_dict().items()})
    for k in finals[0]:
        assert torch.equal(finals[0][k], finals[1][k]), k
