"""The HTTP layer (api.py) over a stand-in service: the reference's routes, schemas and status
codes (app/main.py:132-196) — 503 until a model is loaded, 404 for an unknown user on /score,
request validation (k in 1..100, 1..100 item ids), the cold-start answer passed through. The GPU
service behind the same routes is tested in tests/test_gpu_serving.py."""
import pytest

from conftest import pkg

fastapi = pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402


class FakeService:
    version = "test-1"

    def __init__(self, ready=True):
        self.ready = ready

    def is_ready(self):
        return self.ready

    def recommend(self, user_id, k=10):
        if user_id == "boom":
            raise RuntimeError("kernel failure")
        return [{"item_id": f"i{j}", "score": 1.0 - 0.1 * j, "rank": j + 1} for j in range(k)]

    def score(self, user_id, item_ids):
        if user_id != "u1":
            raise ValueError(f"User '{user_id}' not found in vocabulary.")
        return {i: float(len(i)) for i in item_ids}

    def get_model_info(self):
        return {"version": self.version, "model_path": "mem", "num_users": 1, "faiss_index_items": 3}


def test_routes_over_a_ready_service():
    api = pkg("api")
    with TestClient(api.create_app(service=FakeService())) as c:
        assert c.get("/").json()["status"] == "running"
        assert c.get("/health").json() == {"status": "healthy", "model_loaded": True, "model_version": "test-1"}
        r = c.post("/recommend", json={"user_id": "u1", "k": 3})
        assert r.status_code == 200
        body = r.json()
        assert body["count"] == 3 and body["model_version"] == "test-1"
        assert [x["rank"] for x in body["recommendations"]] == [1, 2, 3]
        assert c.post("/recommend", json={"user_id": "u1"}).json()["count"] == 10      # default k
        assert c.post("/recommend", json={"user_id": "u1", "k": 0}).status_code == 422
        assert c.post("/recommend", json={"user_id": "u1", "k": 101}).status_code == 422
        assert c.post("/recommend", json={"user_id": "boom", "k": 2}).status_code == 500
        s = c.post("/score", json={"user_id": "u1", "item_ids": ["a", "bb"]})
        assert s.status_code == 200 and s.json() == {"user_id": "u1", "scores": {"a": 1.0, "bb": 2.0}}
        assert c.post("/score", json={"user_id": "x", "item_ids": ["a"]}).status_code == 404
        assert c.post("/score", json={"user_id": "u1", "item_ids": []}).status_code == 422
        assert c.get("/model/info").json()["faiss_index_items"] == 3


def test_routes_answer_503_until_loaded_and_after_a_failed_load():
    api = pkg("api")

    def failing_loader(path):
        raise FileNotFoundError(path)
    for app in (api.create_app(service=FakeService(ready=False)),
                api.create_app(model_dir="/nonexistent", loader=failing_loader)):
        with TestClient(app) as c:
            assert c.get("/health").json() == {"status": "degraded", "model_loaded": False, "model_version": None}
            assert c.post("/recommend", json={"user_id": "u1", "k": 3}).status_code == 503
            assert c.post("/score", json={"user_id": "u1", "item_ids": ["a"]}).status_code == 503
            assert c.get("/model/info").status_code == 503


def test_startup_loads_through_the_loader():
    api = pkg("api")
    seen = []

    def loader(path):
        seen.append(path)
        return FakeService()
    with TestClient(api.create_app(model_dir="some/dir", loader=loader)) as c:
        assert c.get("/health").json()["model_loaded"] is True
    assert seen == ["some/dir"]
