"""API contract tests: FastAPI TestClient over a tmp "PVC" filled by the job."""
import pickle
import threading
import time

import numpy as np
import pytest
from fastapi.testclient import TestClient

from kubernetes_machine_learning_server_amd.job import main as job
from kubernetes_machine_learning_server_amd.models import oracle
from kubernetes_machine_learning_server_amd.serve.app import create_app
from kubernetes_machine_learning_server_amd.serve.matcher import NO_RECOMMENDATIONS
from tests.helpers import api_settings, job_settings, make_datasets


@pytest.fixture()
def pvc(tmp_path):
    make_datasets(tmp_path)
    job.run(job_settings(tmp_path))
    return tmp_path


def rec_dict(root):
    with open(root / "api-data" / "pickles" / "recommendations.pickle", "rb") as f:
        return pickle.load(f)


def best_names(root):
    with open(root / "api-data" / "pickles" / "best_tracks.pickle", "rb") as f:
        return [b["track_name"] for b in pickle.load(f)]


def test_openapi_contract(pvc):
    with TestClient(create_app(api_settings(pvc))) as c:
        spec = c.get("/openapi.json").json()
        assert spec["info"]["title"] == "Music Recommendation API"
        assert spec["info"]["version"] == "V-test"
        assert spec["info"]["summary"] == "Kubernetes based deployment with fpgrowth recommendations"
        assert spec["tags"] == [{"name": "recommend", "description": "Song recommendation service"}]
        op = spec["paths"]["/api/recommend/"]["post"]
        assert op["operationId"] == "get_recommendations_api_recommend__post"
        assert op["tags"] == ["recommend"]
        ex = op["requestBody"]["content"]["application/json"]["examples"]
        assert set(ex) == {"normal", "uncommon", "absent"}
        assert ex["normal"]["value"] == {"songs": ["Gold Digger", "Closer"]}
        assert "/test" not in spec["paths"] and "/" not in spec["paths"]
        r = c.get("/test", follow_redirects=False)
        assert r.status_code == 307
        assert r.headers["location"] == "/docs#/recommend/get_recommendations_api_recommend__post"
        assert c.get("/docs").status_code == 200


def test_recommend_matches_reference_semantics(pvc):
    rec = rec_dict(pvc)
    keys = list(rec)
    rng = np.random.default_rng(0)
    with TestClient(create_app(api_settings(pvc))) as c:
        for _ in range(60):
            n = int(rng.integers(1, 5))
            seeds = [keys[int(i)] for i in rng.integers(0, len(keys), n)]
            if rng.random() < 0.3:
                seeds.append("definitely not a song")
            r = c.post("/api/recommend/", json={"songs": seeds})
            assert r.status_code == 200
            body = r.json()
            assert body["version"] == "V-test"
            assert body["model_date"] == (pvc / "api-data" / "last_execution.txt").read_text()
            assert body["songs"] == oracle.recommend_oracle(rec, seeds, 10)


def test_empty_unknown_and_redirect(pvc):
    with TestClient(create_app(api_settings(pvc))) as c:
        r = c.post("/api/recommend/", json={"songs": []})
        assert r.status_code == 400 and r.json() == {"detail": "The songs list cannot be empty."}
        assert c.post("/api/recommend/", json={"nope": 1}).status_code == 422
        r1 = c.post("/api/recommend/", json={"songs": ["Evidencias", "Esse cara sou eu"]}).json()
        r2 = c.post("/api/recommend/", json={"songs": ["Esse cara sou eu", "Evidencias"]}).json()
        assert r1["songs"] == r2["songs"]  # deterministic, order-insensitive seed
        assert len(r1["songs"]) == 10 and set(r1["songs"]) <= set(best_names(pvc))
        r = c.post("/api/recommend", json={"songs": ["x"]}, follow_redirects=False)
        assert r.status_code == 307
        page = c.get("/")
        assert page.status_code == 200 and page.text.count('type="checkbox"') == 10
        assert c.get("/healthz").json() == {"status": "ok"}
        assert c.get("/readyz").json()["ready"] is True
        m = c.get("/metrics").text
        assert "kmls_recommend_requests_total" in m and "kmls_index_keys" in m


def test_key_with_empty_row_returns_empty_list(tmp_path):
    pk = tmp_path / "api-data" / "pickles"
    pk.mkdir(parents=True)
    (pk / "recommendations.pickle").write_bytes(pickle.dumps({"A": {}, "B": {"C": 0.5}, "C": {"B": 0.5}}))
    (pk / "best_tracks.pickle").write_bytes(pickle.dumps(
        [{"track_name": f"t{i}", "count": 10 - i} for i in range(12)]))
    (tmp_path / "api-data" / "last_execution.txt").write_text("2025-01-01 00:00:00")
    with TestClient(create_app(api_settings(tmp_path))) as c:
        assert c.post("/api/recommend/", json={"songs": ["A"]}).json()["songs"] == []
        assert c.post("/api/recommend/", json={"songs": ["A", "B"]}).json()["songs"] == ["C"]
        # seeds are not excluded from their own recommendations (Appendix B.12)
        assert c.post("/api/recommend/", json={"songs": ["B", "C"]}).json()["songs"] == ["C", "B"]


def test_tie_order_follows_pickle_insertion_order(tmp_path):
    """Stable sort over dict insertion order (rest_api/app/main.py:250) — reproduced exactly."""
    pk = tmp_path / "api-data" / "pickles"
    pk.mkdir(parents=True)
    rec = {"s1": {"z": 0.2, "a": 0.2, "m": 0.3}, "s2": {"q": 0.2, "a": 0.25, "z": 0.1},
           "z": {}, "a": {}, "m": {}, "q": {}}
    (pk / "recommendations.pickle").write_bytes(pickle.dumps(rec))
    (pk / "best_tracks.pickle").write_bytes(pickle.dumps([{"track_name": "a", "count": 1}]))
    with TestClient(create_app(api_settings(tmp_path))) as c:
        for seeds in (["s1"], ["s2"], ["s1", "s2"], ["s2", "s1"], ["s2", "s2", "s1"]):
            got = c.post("/api/recommend/", json={"songs": seeds}).json()["songs"]
            assert got == oracle.recommend_oracle(rec, seeds, 10), seeds
        # fewer best tracks than K: clamped instead of the reference's ValueError
        assert c.post("/api/recommend/", json={"songs": ["??"]}).json()["songs"] == ["a"]


def test_not_loaded_placeholder_then_reload(tmp_path):
    make_datasets(tmp_path)
    cfg = api_settings(tmp_path)
    app = create_app(cfg)
    with TestClient(app) as c:
        r = c.post("/api/recommend/", json={"songs": ["x"]})
        assert r.json()["songs"] == [NO_RECOMMENDATIONS] and r.json()["model_date"] is None
        assert c.get("/readyz").status_code == 503
        job.run(job_settings(tmp_path))
        assert app.state.mgr.reload_data_if_required() is True
        assert c.get("/readyz").status_code == 200
        marker = (tmp_path / "api-data" / "last_execution.txt").read_text()
        assert c.post("/api/recommend/", json={"songs": ["x"]}).json()["model_date"] == marker
        assert app.state.mgr.reload_data_if_required() is False  # not stale
        # next job run (dataset 2) → marker changes → reload picks up the new model
        time.sleep(1.1)
        job.run(job_settings(tmp_path))
        assert app.state.mgr.reload_data_if_required() is True
        assert app.state.mgr.reload_counter == 2
        new_marker = (tmp_path / "api-data" / "last_execution.txt").read_text()
        assert c.post("/api/recommend/", json={"songs": ["x"]}).json()["model_date"] == new_marker


def test_failed_reload_keeps_old_model_and_retries(pvc):
    app = create_app(api_settings(pvc))
    with TestClient(app) as c:
        mgr = app.state.mgr
        old = mgr.cache_value
        best = pvc / "api-data" / "pickles" / "best_tracks.pickle"
        saved = best.read_bytes()
        best.unlink()
        (pvc / "api-data" / "last_execution.txt").write_text("2099-01-01 00:00:00")
        assert mgr.reload_data_if_required() is False
        assert mgr.cache_value == old  # still serving the previous snapshot
        assert c.post("/api/recommend/", json={"songs": ["x"]}).status_code == 200
        best.write_bytes(saved)
        assert mgr.reload_data_if_required() is True  # retried because the marker is unconsumed
        assert mgr.cache_value == "2099-01-01 00:00:00"


def test_concurrent_requests_during_reloads(pvc):
    """Stress: hammer /recommend while reloading (the reference's acknowledged race)."""
    app = create_app(api_settings(pvc))
    rec = rec_dict(pvc)
    keys = list(rec)
    errors = []
    with TestClient(app) as c:
        stop = threading.Event()

        def reloader():
            i = 0
            while not stop.is_set():
                (pvc / "api-data" / "last_execution.txt").write_text(f"2030-01-01 00:00:{i % 60:02d}")
                app.state.mgr.reload_data_if_required()
                i += 1

        def client(seed):
            rng = np.random.default_rng(seed)
            for _ in range(40):
                seeds = [keys[int(j)] for j in rng.integers(0, len(keys), 3)]
                r = c.post("/api/recommend/", json={"songs": seeds})
                if r.status_code != 200 or r.json()["songs"] != oracle.recommend_oracle(rec, seeds, 10):
                    errors.append(r.text)

        th = [threading.Thread(target=reloader)] + [threading.Thread(target=client, args=(s,)) for s in range(4)]
        for t in th:
            t.start()
        for t in th[1:]:
            t.join()
        stop.set()
        th[0].join()
    assert not errors
    assert app.state.mgr.reload_counter > 1


def test_corrupt_rule_index_falls_back_to_pickle(pvc):
    """rules.idx is written atomically; a corrupt/truncated one (crash of a foreign writer) is
    skipped in favour of recommendations.pickle, so a fresh replica still becomes ready."""
    import os
    idx = pvc / "api-data" / "pickles" / "rules.idx"
    assert idx.exists()
    idx.write_bytes(idx.read_bytes()[:100])  # truncated
    t = (pvc / "api-data" / "pickles" / "recommendations.pickle").stat().st_mtime
    os.utime(idx, (t + 5, t + 5))  # newer than the pickle: the loader tries it first
    with TestClient(create_app(api_settings(pvc))) as c:
        assert c.get("/readyz").status_code == 200
        rec = rec_dict(pvc)
        seed = next(k for k, v in rec.items() if v)
        got = c.post("/api/recommend/", json={"songs": [seed]}).json()["songs"]
        assert got == oracle.recommend_oracle(rec, [seed], 10)


class _FakeGpuIndex:
    """Stands in for _native.GpuRuleIndex (CPU-only tests): answers with the C++ matcher and
    counts the batches it was given."""

    def __init__(self, index):
        self.host = index.native()
        self.calls = 0

    def query_batch(self, q_ptr, seeds, k):
        self.calls += 1
        return self.host.query_batch(q_ptr, seeds, k)


@pytest.mark.parametrize("backend,expect_gpu", [("auto", False), ("hip", True)])
def test_router_uses_gpu_only_past_the_measured_crossover(pvc, monkeypatch, backend, expect_gpu):
    """SERVE_BACKEND=auto sends work to the HIP matcher only when enough requests are in flight
    to fill a batch at least as large as the crossover measured on the index; one-at-a-time
    traffic never touches it.  SERVE_BACKEND=hip forces every request through it."""
    from kubernetes_machine_learning_server_amd.serve import app as app_mod
    from kubernetes_machine_learning_server_amd.serve import state as state_mod
    made = []

    def factory(cfg):
        def build(index):
            g = _FakeGpuIndex(index)
            made.append(g)
            return g
        return build
    monkeypatch.setattr(app_mod, "_gpu_factory", factory)
    monkeypatch.setattr(state_mod, "measure_crossover", lambda index, g: (256, {256: (47.0, 33.0)}))
    rec = rec_dict(pvc)
    seeds = [k for k, v in rec.items() if v][:20]
    with TestClient(create_app(api_settings(pvc, serve_backend=backend))) as c:
        ready = c.get("/readyz").json()
        assert ready["gpu_index"] and ready["gpu_min_batch"] == (1 if backend == "hip" else 256)
        for sd in seeds:
            got = c.post("/api/recommend/", json={"songs": [sd]}).json()["songs"]
            assert got == oracle.recommend_oracle(rec, [sd], 10)
    assert made and (made[-1].calls > 0) == expect_gpu
