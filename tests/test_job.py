"""Job pipeline tests (SURVEY §7.6 unit + artifact contract §2.F, failure handling §5.3)."""
import pickle

import numpy as np
import pytest

from kubernetes_machine_learning_server_amd.job import main as job
from kubernetes_machine_learning_server_amd.job import preprocess as pp
from kubernetes_machine_learning_server_amd.job import rotation as rot
from kubernetes_machine_learning_server_amd.models import oracle
from kubernetes_machine_learning_server_amd.serve.index import RuleIndexData
from tests.helpers import job_settings, make_datasets


@pytest.fixture()
def pvc(tmp_path):
    make_datasets(tmp_path)
    return tmp_path


def load(p):
    with open(p, "rb") as f:
        return pickle.load(f)


def test_job_artifacts_and_rotation(pvc, capsys):
    cfg = job_settings(pvc)
    s1 = job.run(cfg)
    assert s1["dataset_index"] == 1
    pk = cfg.pickles_folder
    rec = load(pk / "recommendations.pickle")
    best = load(pk / "best_tracks.pickle")
    artists = load(pk / "artistsMapping.pickle")
    info = load(pk / "trackIdsToInfo.pickle")
    assert isinstance(rec, dict) and all(isinstance(v, dict) for v in rec.values())
    assert all(isinstance(x, float) for row in rec.values() for x in row.values())
    assert isinstance(best, list) and set(best[0]) == {"track_name", "count"}
    assert [b["count"] for b in best] == sorted([b["count"] for b in best], reverse=True)
    assert all(isinstance(v, str) for v in artists.values())
    assert set(next(iter(info.values()))) == {"track_name", "artist_name", "album_name"}
    marker = (cfg.base_dir / "last_execution.txt").read_text()
    assert len(marker) == 19 and marker[4] == "-" and marker[13] == ":"
    hist = (cfg.base_dir / "dataset_history.csv").read_text().splitlines()
    assert hist[0] == "time,dataset_index,dataset_file" and hist[1].split(",")[1] == "1"
    lst = (cfg.base_dir / "datasets_list.txt").read_text().splitlines()
    assert lst == sorted(lst) and len(lst) == 2
    # second run → dataset 2, third wraps to 1
    assert job.run(cfg)["dataset_index"] == 2
    assert job.run(cfg)["dataset_index"] == 1
    out = capsys.readouterr().out
    assert "Songs without recommendations:" in out and "Time elapsed in rule generation:" in out


def test_rule_map_matches_oracle(pvc):
    """recommendations.pickle == the reference rule loop over mlxtend-faithful itemsets."""
    cfg = job_settings(pvc, min_support=0.05)
    job.run(cfg)
    rec = load(cfg.pickles_folder / "recommendations.pickle")
    t = pp.clean_df(pp.read_tracks(str(pvc / "datasets" / "2023_spotify_ds1.csv"), verbose=False))
    txl = pp.group_tracks_by_playlist(t).as_lists()
    X, cols = oracle.transaction_encode(txl)
    ref = oracle.rule_map_from_itemsets(oracle.fpgrowth_oracle(X, 0.05, cols))
    assert set(rec) == set(ref)
    for k in ref:
        assert rec[k] == ref[k]
    # rules.idx round-trips to the same dict
    idx = RuleIndexData.load(cfg.pickles_folder / "rules.idx")
    assert idx.to_rec_dict() == rec


@pytest.mark.parametrize("mode", ["pairs", "full"])
def test_rules_modes_identical(pvc, mode):
    cfg = job_settings(pvc, rules_mode=mode)
    job.run(cfg)
    rec = load(cfg.pickles_folder / "recommendations.pickle")
    cfg2 = job_settings(pvc, miner="oracle")
    cfg2.base_dir = pvc / "api-oracle"
    cfg2.pickles_folder = cfg2.base_dir / "pickles"
    job.run(cfg2)
    assert rec == load(cfg2.pickles_folder / "recommendations.pickle")


def test_history_malformed_and_wrap(pvc):
    cfg = job_settings(pvc)
    cfg.base_dir.mkdir(parents=True)
    ds = ["a.csv", "b.csv", "c.csv"]
    assert rot.get_next_run_index(cfg, ds) == 1
    cfg.dataset_history_file.write_text("time,dataset_index,dataset_file\n2025,3,c.csv\n")
    assert rot.get_next_run_index(cfg, ds) == 1  # wrap
    cfg.dataset_history_file.write_text("time,dataset_index,dataset_file\n2025,2,b.csv\n")
    assert rot.get_next_run_index(cfg, ds) == 3
    cfg.dataset_history_file.write_text("time,dataset_index,dataset_file\ngarbage\n")
    assert rot.get_next_run_index(cfg, ds) == 1


def test_no_datasets_raises(tmp_path):
    cfg = job_settings(tmp_path)
    with pytest.raises(FileNotFoundError):
        rot.get_dataset_list(cfg)


def test_dist_mode_validated(tmp_path, monkeypatch):
    """'local' would put every itemset N times into the distributed job's rule map."""
    from kubernetes_machine_learning_server_amd.config import JobSettings
    monkeypatch.setenv("KMLS_DIST_MODE", "local")
    with pytest.raises(ValueError, match="KMLS_DIST_MODE"):
        JobSettings.from_env(dotenv=False)
    monkeypatch.setenv("KMLS_DIST_MODE", "Shard")
    assert JobSettings.from_env(dotenv=False).dist_mode == "shard"


def test_artist_validation_raises(tmp_path):
    ds = tmp_path / "datasets"
    ds.mkdir()
    (ds / "2023_spotify_ds1.csv").write_text(
        "pid,track_uri,track_name,artist_name,artist_uri,album_name,album_uri,duration_ms\n"
        "0,u1,Song A,Artist X,ax1,Al,al,1\n0,u2,Song B,Artist X,ax2,Al,al,1\n")
    cfg = job_settings(tmp_path)
    with pytest.raises(ValueError, match="duplicate artists"):
        job.run(cfg)


def test_duplicates_pickle_only_when_present(tmp_path):
    ds = tmp_path / "datasets"
    ds.mkdir()
    (ds / "2023_spotify_ds1.csv").write_text(
        "pid,track_uri,track_name,artist_name,artist_uri,album_name,album_uri,duration_ms\n"
        "0,u1,Song A,X,x,Al,al,1\n0,u2,Song B,X,x,Al,al,1\n1,u1,Song A,X,x,Al,al,1\n"
        "1,u2,Song B,X,x,Al,al,1\n")
    cfg = job_settings(tmp_path, pct=1.0, min_support=0.5)
    job.run(cfg)
    assert not (cfg.pickles_folder / "trackNameToRepeatedUris.pickle").exists()
    rec = load(cfg.pickles_folder / "recommendations.pickle")
    assert rec == {"Song A": {"Song B": 1.0}, "Song B": {"Song A": 1.0}}
    # a name with two URIs (the encoder collapses them inside a playlist)
    (ds / "2023_spotify_ds1.csv").write_text(
        "pid,track_uri,track_name,artist_name,artist_uri,album_name,album_uri,duration_ms\n"
        "0,u1,Song A,X,x,Al,al,1\n0,u3,Song A,X,x,Al,al,1\n0,u2,Song B,X,x,Al,al,1\n")
    cfg2 = job_settings(tmp_path, pct=1.0, min_support=0.5)
    cfg2.base_dir = tmp_path / "api2"
    cfg2.pickles_folder = cfg2.base_dir / "pickles"
    job.run(cfg2)
    dups = load(cfg2.pickles_folder / "trackNameToRepeatedUris.pickle")
    assert dups == {"Song A": ["u1", "u3"]}


def test_marker_written_last_under_fault(pvc, monkeypatch):
    cfg = job_settings(pvc)
    job.run(cfg)
    marker = (cfg.base_dir / "last_execution.txt").read_text()
    rec_before = (cfg.pickles_folder / "recommendations.pickle").read_bytes()
    monkeypatch.setenv("KMLS_FAULT", "before_recommendations")
    with pytest.raises(RuntimeError):
        job.run(cfg)
    # no marker change, old artifacts intact (atomic writes)
    assert (cfg.base_dir / "last_execution.txt").read_text() == marker
    assert (cfg.pickles_folder / "recommendations.pickle").read_bytes() == rec_before
    monkeypatch.setenv("KMLS_FAULT", "before_marker")
    with pytest.raises(RuntimeError):
        job.run(cfg)
    assert (cfg.base_dir / "last_execution.txt").read_text() == marker


def test_support_sweep(pvc, tmp_path):
    cfg = job_settings(pvc)
    t = pp.clean_df(pp.read_tracks(str(pvc / "datasets" / "2023_spotify_ds1.csv"), verbose=False))
    tx = pp.group_tracks_by_playlist(t)
    out = tmp_path / "sweep.csv"
    rows = job.run_support_sweep(cfg, tx, t.n_unique("track_uri"), [0.2, 0.1, 0.05], str(out))
    missing = [r["songs_without_recommendations"] for r in rows]
    assert missing == sorted(missing, reverse=True)  # lower support → more keys
    import pandas as pd
    df = pd.read_csv(out)
    assert list(df.columns[:3]) == ["min_support", "songs_without_recommendations", "duration"]


def test_csv_reader_quotes(tmp_path):
    p = tmp_path / "q.csv"
    p.write_text('pid,track_uri,track_name,artist_name,artist_uri,album_name,album_uri,duration_ms\r\n'
                 '7,"u,1","City Of Stars - From ""La La Land""","A, B",a,"Al",x,3\r\n'
                 '7,u2,Plain,"A, B",a,Al,x,4\r\n')
    t = pp.read_tracks(str(p), verbose=False)
    assert t.n_rows == 2 and t.width == 8
    assert t.uniques["track_name"] == ['City Of Stars - From "La La Land"', "Plain"]
    assert t.uniques["track_uri"] == ["u,1", "u2"]
    assert t.uniques["artist_name"] == ["A, B"]


def test_checkpoint_resume_after_crash(pvc, tmp_path, monkeypatch):
    """A crash after mining leaves a phase checkpoint; the restarted job (same dataset — the
    rotation cursor did not advance) resumes from it and produces the same artifacts."""
    ckdir = tmp_path / "ckpt"
    cfg = job_settings(pvc, checkpoint_dir=ckdir)
    monkeypatch.setenv("KMLS_FAULT", "before_recommendations")
    with pytest.raises(RuntimeError, match="injected fault"):
        job.run(cfg)
    assert any(ckdir.rglob("trie.npz"))
    monkeypatch.delenv("KMLS_FAULT")
    s = job.run(cfg)
    assert s["resumed"] is True and s["dataset_index"] == 1
    assert not any(ckdir.rglob("trie.npz"))  # cleared after success
    rec_resumed = load(cfg.pickles_folder / "recommendations.pickle")
    clean = job_settings(tmp_path / "clean")
    make_datasets(tmp_path / "clean")
    s2 = job.run(clean)
    assert s2["resumed"] is False
    assert load(clean.pickles_folder / "recommendations.pickle") == rec_resumed


def test_unused_reference_helpers(pvc):
    """J16 parity: the reference's never-called helpers behave as written there."""
    t = pp.clean_df(pp.read_tracks(str(pvc / "datasets" / "2023_spotify_ds1.csv"), verbose=False))
    top = pp.get_most_frequent_tracks(t)
    names = pp.save_most_frequent_tracks_dict(top)
    assert names == [x["track_name"] for x in top[:int(len(top) * 0.1)]]
    homo = pp.group_tracks_by_playlist_and_generate_homogeneous_data(t)
    tx = pp.group_tracks_by_playlist(t, backend="cpu")
    assert len(homo) == tx.n_tx
    for pid, row in zip(tx.pids[:20], tx.as_lists()[:20]):
        assert sorted(set(homo[pid])) == sorted(set(row))
    het = pp.group_tracks_by_playlist_and_generate_heterogeneous_data(t)
    first = next(iter(het.values()))
    assert "track_name" in first.columns and "track_uri" not in first.columns
    assert sum(len(v) for v in het.values()) == t.n_rows


def rec_dict(root):
    with open(root / "api-data" / "pickles" / "recommendations.pickle", "rb") as f:
        return pickle.load(f)


def _dist_job_worker(rank, world, port, root, fault, out_q, extra=None):
    import os as _os
    _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                       WORLD_SIZE=str(world), LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    if fault:
        _os.environ["KMLS_FAULT"] = fault
    else:
        _os.environ.pop("KMLS_FAULT", None)
    import pathlib as _pl
    _os.chdir(root)  # the J14 sweep writes its CSV to the working directory (as the reference)
    from kubernetes_machine_learning_server_amd.job import main as _job
    from tests.helpers import job_settings as _js
    cfg = _js(_pl.Path(root), num_gpus=world, checkpoint_dir=_pl.Path(root) / "ck",
              dist_timeout_s=120.0, **(extra or {}))
    try:
        out_q.put((rank, _job.run(cfg), None))
    except Exception as e:  # noqa: BLE001 — the injected fault
        out_q.put((rank, None, repr(e)))


def _run_dist_job(root, world, fault="", extra=None):
    import socket
    import torch.multiprocessing as tmp_mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = tmp_mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_job_worker, args=(r, world, port, str(root), fault, q, extra))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("mode", ["auto", "tx", "shard"])
def test_distributed_job_phase_checkpoints(tmp_path, mode):
    """torchrun-style job at world size 2 (gloo + the CPU protocol): the per-rank sub-trie
    phase is checkpointed; after a crash between mining and publishing, the restarted job
    resumes from every rank's sub-trie (tx mode: rank 0's global trie) without re-mining and
    publishes the same artifacts as a single-process run."""
    make_datasets(tmp_path, shapes=("ds2_weak", "tiny"), seeds=(3, 4))
    extra = {"dist_mode": mode}
    res = _run_dist_job(tmp_path, 2, fault="after_mining_phase", extra=extra)
    assert all("injected fault" in (r[2] or "") for r in res)
    ck_files = list((tmp_path / "ck").rglob("subtrie_r*of2_*.npz"))
    assert len(ck_files) == (1 if mode == "tx" else 2), ck_files
    res = _run_dist_job(tmp_path, 2, extra=extra)
    summary = res[0][1]
    assert summary and summary["dataset_index"] == 1
    assert summary["backend"] == "checkpoint"  # merged from the sub-tries, not re-mined
    single = tmp_path / "single"
    make_datasets(single, shapes=("ds2_weak", "tiny"), seeds=(3, 4))
    ref = job.run(job_settings(single))
    assert summary["n_itemsets"] == ref["n_itemsets"] and summary["n_keys"] == ref["n_keys"]
    assert rec_dict(tmp_path) == rec_dict(single)
    # the deployed index comes from the distributed rule map, byte-equal to one process's
    idx_name = job.RULES_INDEX_FILE
    assert (tmp_path / "api-data" / "pickles" / idx_name).read_bytes() == \
        (single / "api-data" / "pickles" / idx_name).read_bytes()
    assert summary["rule_map"].startswith("distributed-x2")
    assert not list((tmp_path / "ck").rglob("*.npz"))  # cleared after success


@pytest.mark.parametrize("strategy", ["reduce_scatter", "ring", "alltoall"])
def test_distributed_pairs_job_strategies(tmp_path, strategy):
    """RULES_MODE=pairs at world size 2: the job forms the pair matrix with a parallel.pairs
    strategy (item blocks per rank; ring = context-parallel, alltoall = Ulysses analog) and
    publishes the same recommendations as a single-process pairs run."""
    make_datasets(tmp_path, shapes=("ds2_weak", "tiny"), seeds=(3, 4))
    res = _run_dist_job(tmp_path, 2, extra={"rules_mode": "pairs", "pairs_strategy": strategy})
    assert all(r[2] is None for r in res), res
    summary = res[0][1]
    assert summary["backend"] == f"pairs-{strategy}-x2"
    single = tmp_path / "single"
    make_datasets(single, shapes=("ds2_weak", "tiny"), seeds=(3, 4))
    ref = job.run(job_settings(single, rules_mode="pairs"))
    assert summary["n_itemsets"] == ref["n_itemsets"] and summary["n_keys"] == ref["n_keys"]
    assert rec_dict(tmp_path) == rec_dict(single)



def test_distributed_support_sweep(tmp_path):
    """EXPERIMENT_SUPPORTS at world size 2: the sweep points are split over the ranks, each
    mined locally; rank 0 writes every point in grid order, equal to a single-process sweep."""
    import pandas as pd
    make_datasets(tmp_path, shapes=("ds2_weak", "tiny"), seeds=(3, 4))
    res = _run_dist_job(tmp_path, 2, extra={"experiment_supports": True})
    assert all(r[2] is None for r in res), res
    df = pd.read_csv(tmp_path / job.EXPERIMENT_CSV)
    grid = [round(x, 3) for x in np.arange(0.03, 0.2, 0.0025).tolist()]
    assert df["min_support"].tolist() == grid
    single = tmp_path / "single"
    make_datasets(single, shapes=("ds2_weak", "tiny"), seeds=(3, 4))
    cfg = job_settings(single)
    t = pp.clean_df(pp.read_tracks(str(single / "datasets" / "2023_spotify_ds1.csv"), verbose=False))
    tx = pp.group_tracks_by_playlist(t)
    rows = job.run_support_sweep(cfg, tx, t.n_unique("track_uri"), grid[::7],
                                 str(tmp_path / "one.csv"))
    got = df.set_index("min_support")
    for r in rows:
        assert got.loc[r["min_support"], "songs_without_recommendations"] == \
            r["songs_without_recommendations"]
        assert got.loc[r["min_support"], "n_itemsets"] == r["n_itemsets"]
