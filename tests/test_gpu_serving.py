"""the GPU ranking-metric suite (metrics.hip) and the serving path
(RecommendationService on the trainer's artefacts, cosine BruteForceIndex) vs the oracle."""
import numpy as np
import pytest

from conftest import oracle, pkg

pytestmark = pytest.mark.gpu


def _lists(rng, U, n_items, kmax, ragged=True):
    out = []
    for _ in range(U):
        L = int(rng.integers(0, kmax + 1)) if ragged else kmax
        out.append([int(v) for v in rng.integers(0, n_items, L)])   # duplicates included
    return out


@pytest.mark.parametrize("U,n_items,kmax", [(1, 5, 3), (300, 50, 20), (1000, 5000, 100), (37, 8, 130)])
def test_rank_metrics_match_oracle(cuda, U, n_items, kmax):
    import torch
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(U + n_items)
    lists = _lists(rng, U, n_items, kmax)
    truths = [int(v) for v in rng.integers(-1, n_items, U)]
    ks = [1, 5, 10, 50]
    K = max(max(len(l) for l in lists), 1)
    pred = np.full((U, K), -3, np.int64)
    for u, l in enumerate(lists):
        pred[u, :len(l)] = l
    lens = torch.tensor([len(l) for l in lists], dtype=torch.int32, device=cuda)
    tr = torch.tensor([t if t >= 0 else -2 for t in truths], dtype=torch.int64, device=cuda)
    got = F.rank_metrics(torch.from_numpy(pred).to(cuda), tr, ks, n_items, lens).cpu().numpy()
    ref = O.metric_suite(lists, truths, ks, n_items)
    assert np.allclose(got, ref, rtol=0, atol=1e-12), (got, ref)


def test_advanced_metrics_reference_api_on_strings(cuda):
    M = pkg("metrics").AdvancedMetrics
    O = oracle()
    rng = np.random.default_rng(5)
    names = [f"m{i}" for i in range(40)]
    preds = [[names[j] for j in rng.integers(0, 40, int(rng.integers(0, 12)))] for _ in range(200)]
    truth = [names[j] if j < 40 else "unknown" for j in rng.integers(0, 45, 200)]
    ref = O.metric_suite(preds, truth, [10], 40)
    assert M.recall_at_k(preds, truth, 10) == pytest.approx(ref[0], abs=1e-12)
    assert M.precision_at_k(preds, truth, 10) == pytest.approx(ref[1], abs=1e-12)
    assert M.ndcg_at_k(preds, truth, 10) == pytest.approx(ref[2], abs=1e-12)
    assert M.map_at_k(preds, truth, 10) == pytest.approx(ref[3], abs=1e-12)
    assert M.mrr(preds, truth) == pytest.approx(ref[4], abs=1e-12)
    assert M.diversity(preds) == pytest.approx(ref[5], abs=1e-12)
    assert M.coverage(preds, names) == pytest.approx(ref[6], abs=1e-12)
    assert M.recall_at_k([], [], 5) == 0.0 and M.coverage(preds, []) == 0.0


def test_l2_normalize_rows(cuda):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(2)
    for D in (32, 128, 200):
        x = rng.standard_normal((300, D)).astype(np.float32)
        x[7] = 0.0
        y = F.l2_normalize_rows(torch.from_numpy(x).to(cuda)).cpu().numpy().astype(np.float64)
        ref = x.astype(np.float64) / np.maximum(np.linalg.norm(x.astype(np.float64), axis=1, keepdims=True), 1e-30)
        ref[7] = 0.0
        assert np.abs(y - ref).max() < 1e-6


def test_recommendation_service_end_to_end(cuda, tmp_path):
    import pandas as pd
    import torch
    cfgm = pkg("config")
    tr = pkg("trainer")
    serving = pkg("serving")
    O = oracle()

    def frame(k, seed):
        r = np.random.default_rng(seed)
        return pd.DataFrame({"user_id": r.integers(0, 200, k), "movie_id": r.integers(0, 150, k),
                             "rating": r.integers(1, 6, k), "timestamp": r.integers(0, 10 ** 9, k)})

    train, val = frame(4000, 1), frame(500, 2)
    for d in (train, val):
        d["y_implicit"] = (d["rating"] >= 4).astype(int)
    pkl = tmp_path / "processed.pkl"
    pd.to_pickle({"train_ratings": train, "val_ratings": val, "test_ratings": val,
                  "user_features": {}, "movie_features": {}}, pkl)
    cfg = cfgm.ModelConfig(embedding_dim=32, cross_layers=1, batch_size=512, epochs_retrieval=1)
    out = tmp_path / "out"
    model, _ = tr.ProductionTrainer(cfg, str(out)).train(str(pkl))

    svc = serving.RecommendationService(str(out))
    assert not svc.is_ready()
    svc.load()
    assert svc.is_ready()
    info = svc.get_model_info()
    assert info["faiss_index_items"] == len(svc.item_map) and info["num_users"] == len(svc.user_vocab)

    user = svc.user_vocab[3]
    recs = svc.recommend(user, k=10)
    assert [r["rank"] for r in recs] == list(range(1, 11))
    # oracle: cosine top-10 of the same (normalised) vectors in float64
    with torch.no_grad():
        u = model.encoder({"user_id": [user]})["user_embedding"].cpu().numpy().astype(np.float64)
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    items = svc.faiss_index.items.cpu().numpy().astype(np.float64)
    sc, idx = O.topk_ip(u, items, 10)
    got_items = [r["item_id"] for r in recs]
    ref_items = [svc.item_map[str(i)] for i in idx[0]]
    got_scores = np.array([r["score"] for r in recs])
    assert np.abs(got_scores - sc[0]).max() < 1e-5
    gap = np.diff(sc[0]).min() if len(sc[0]) > 1 else -1
    if -gap > 1e-5:   # no near-ties: identical order
        assert got_items == ref_items
    # batched recommend, cold start, score
    batch = svc.recommend_batch([user, "nobody"], k=5)
    assert [r["item_id"] for r in batch[0]] == got_items[:5]
    assert batch[1] == svc._get_popular_items(5) == svc.recommend("nobody", k=5)
    assert batch[1][0]["score"] == 1.0 and batch[1][1]["score"] == pytest.approx(0.95)
    some = [svc.item_map[str(i)] for i in (0, 4, 9)]
    s = svc.score(user, some)
    with torch.no_grad():
        e = model.encoder({"user_id": [user], "movie_id": some})
    ref = e["item_embedding"].cpu().double().numpy() @ e["user_embedding"].cpu().double().numpy()[0]
    assert np.allclose([s[i] for i in some], ref, atol=1e-5)
    with pytest.raises(ValueError):
        svc.score("nobody", some)
    # the HTTP routes (api.py, app/main.py:132-196) over the loaded service: the same answers
    from fastapi.testclient import TestClient
    api = pkg("api")
    with TestClient(api.create_app(service=svc)) as client:
        h = client.get("/health").json()
        assert h == {"status": "healthy", "model_loaded": True, "model_version": svc.version}
        r = client.post("/recommend", json={"user_id": user, "k": 10}).json()
        assert r["count"] == 10 and [x["item_id"] for x in r["recommendations"]] == got_items
        assert np.abs(np.array([x["score"] for x in r["recommendations"]]) - got_scores).max() < 1e-6
        sr = client.post("/score", json={"user_id": user, "item_ids": some})
        assert sr.status_code == 200 and sr.json()["scores"] == pytest.approx(s, abs=1e-6)
        assert client.post("/score", json={"user_id": "nobody", "item_ids": some}).status_code == 404
        assert client.get("/model/info").json()["faiss_index_items"] == info["faiss_index_items"]

    # second serving variant (app/model_service.py): raw inner product over the item tower
    ms = pkg("model_service").RecommendationService(str(out))
    assert not ms.is_ready()
    ms.load_model()
    assert ms.is_ready() and ms.get_version() == "1.0.0"
    info = ms.get_model_info()
    assert info["num_items"] == len(ms.item_vocab) and info["embedding_dim"] == 32
    with torch.no_grad():
        ie = model.encoder({"movie_id": ms.item_vocab})["item_embedding"].cpu().numpy().astype(np.float64)
        ue = model.encoder({"user_id": [user]})["user_embedding"].cpu().numpy().astype(np.float64)
    assert np.abs(ms.item_embeddings.cpu().numpy() - ie).max() < 1e-5
    recs2 = ms.recommend(user, k=7)
    sc2, idx2 = O.topk_ip(ue, ms.item_embeddings.cpu().numpy().astype(np.float64), 7)
    assert [r["rank"] for r in recs2] == list(range(1, 8))
    assert np.abs(np.array([r["score"] for r in recs2]) - sc2[0]).max() < 1e-5
    if len(sc2[0]) < 2 or -np.diff(sc2[0]).min() > 1e-5:
        assert [r["item_id"] for r in recs2] == [ms.item_vocab[i] for i in idx2[0]]
    b2 = ms.recommend_batch([user, "nobody", user], k=7)
    assert [x["status"] for x in b2] == ["success"] * 3 and b2[0]["recommendations"] == recs2
    assert b2[1]["recommendations"] == ms._get_popular_items(7) and b2[1]["recommendations"][1]["score"] == 0.5
    assert b2[2]["user_id"] == user and b2[2]["recommendations"] == recs2
    s2 = ms.score(user, some + ["not-an-item"])
    assert set(s2) == set(some) and np.allclose([s2[i] for i in some], ref, atol=1e-5)
    with pytest.raises(ValueError):
        ms.score(user, ["not-an-item"])
    with pytest.raises(FileNotFoundError):
        pkg("model_service").RecommendationService(str(tmp_path / "missing")).load_model()
