"""The headline engine as the product's miner: ``fpgrowth()`` / ``mine_csr`` / the job mine short
transaction sets with the deep DFS miner in emit mode (kernels/deep.hip), whose HBM node arena
is compacted into a parent-first trie on the device (kernels/deep_trie.hip).  Every check is by
content against the CPU miner's trie (``trie_digest``: every (itemset, support) pair), plus the
trie invariant the consumers rely on (parents before children)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from kubernetes_machine_learning_server_amd.data.synthetic import generate

pytestmark = pytest.mark.gpu


def _cpu_digest(N, tx, ms, max_len=0):
    ref = N.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms, max_len)
    return N.trie_digest(ref["parent"], ref["item"], ref["count"], ref["depth"])


def _check_trie(par, dep):
    par = np.asarray(par, np.int64)
    idx = np.arange(len(par))
    assert (par < idx).all(), "a parent after its child"
    has = par >= 0
    assert (np.asarray(dep)[has] == np.asarray(dep)[par[has]] + 1).all()
    assert (np.asarray(dep)[~has] == 1).all()


def _onehot_df(tx):
    import pandas as pd
    X = np.zeros((tx.n_tx, tx.n_items), dtype=bool)
    rows = np.repeat(np.arange(tx.n_tx), np.diff(tx.tx_ptr))
    X[rows, tx.items] = True
    return pd.DataFrame(X, columns=[f"t{i:05d}" for i in range(tx.n_items)])


def test_fpgrowth_deep_path_equals_cpu_trie(gpu_mod, monkeypatch):
    """fpgrowth(df, 0.03, use_colnames=True) on ds1-shape data (9.4e6 itemsets up to size 10):
    mined by the deep engine, the trie's content digest equals the CPU miner's."""
    from kubernetes_machine_learning_server_amd.models.fpgrowth import fpgrowth, full_miner
    monkeypatch.setenv("MINER", "gpu")
    tx = generate("ds1", seed=0)
    assert full_miner(tx.n_tx) == "deep"
    trie = fpgrowth(_onehot_df(tx), 0.03, use_colnames=True, as_trie=True)
    assert trie.stats["miner"] == "deep" and trie.stats["backend"] == "gpu"
    want = _cpu_digest(gpu_mod, tx, 0.03)
    got = gpu_mod.trie_digest(trie.parent, trie.item, trie.count, trie.depth)
    assert got["digest"] == want["digest"] and got["per_depth"] == want["per_depth"]
    assert len(trie) == want["n"] == trie.stats["n_itemsets"]
    assert trie.stats["digest"] == want["digest"]  # the count-only digest of the same launch
    _check_trie(trie.parent, trie.depth)
    # narrow widths: 9 B per itemset
    assert trie.parent.dtype == np.int32 and trie.item.dtype == np.uint16
    assert trie.count.dtype == np.uint16 and trie.depth.dtype == np.uint8


@pytest.mark.parametrize("max_len", [0, 3])
def test_fpgrowth_dataframe_deep_equals_levels(gpu_mod, monkeypatch, max_len):
    """The mlxtend-shaped DataFrame (support, frozenset of names) is the same set of rows from
    the deep engine and from the level-wise engine."""
    from kubernetes_machine_learning_server_amd.models.fpgrowth import fpgrowth
    monkeypatch.setenv("MINER", "gpu")
    tx = generate("ds2_weak", seed=3)
    df = _onehot_df(tx)
    out = {}
    for eng in ("deep", "levels"):
        monkeypatch.setenv("KMLS_FULL_MINER", eng)
        r = fpgrowth(df, 0.05, use_colnames=True, max_len=max_len or None)
        out[eng] = set(zip(r["support"].round(12), r["itemsets"]))
    assert out["deep"] == out["levels"] and len(out["deep"]) > 100


def test_mine_csr_deep_builds_the_device_rule_map(gpu_mod, monkeypatch):
    """rule_index on the deep path: the device rule map (pair supports) comes with the trie."""
    from kubernetes_machine_learning_server_amd.models.fpgrowth import mine_csr
    from kubernetes_machine_learning_server_amd.serve.index import (build_index_from_trie,
                                                                    index_from_device_csr)
    tx = generate("ds1", seed=1)
    names = [f"s{i:05d}" for i in range(tx.n_items)]
    trie = mine_csr(tx.tx_ptr, tx.items, tx.n_items, 0.04, backend="gpu", columns=names,
                    rule_index=True)
    assert trie.stats["miner"] == "deep"
    dev = trie.stats.pop("device_rule_map")
    a = index_from_device_csr(dev, tx.n_items, trie.item[trie.depth == 1], tx.n_tx, names)
    b = build_index_from_trie(trie.parent, trie.item, trie.count, trie.depth, tx.n_tx,
                              tx.n_items, names)
    for f in ("row_ptr", "cons", "score", "is_key"):
        assert (getattr(a, f) == getattr(b, f)).all(), f


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _split_worker(rank, world, port, ms, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), KMLS_COMM="host", KMLS_COMM_TIMEOUT_S="120")
    import torch.distributed as dist
    from kubernetes_machine_learning_server_amd.ops import native
    from kubernetes_machine_learning_server_amd.parallel.deep import DeepMiner
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        try:
            tx = generate("ds1", seed=0)
            dm = DeepMiner(tx.tx_ptr, tx.items, tx.n_items, device=0, rank=rank, world=world,
                           comm_backend="host")
            d, arrs = dm.mine_trie(ms)
            got = None
            if rank == 0:
                _check_trie(arrs["parent"], arrs["depth"])
                got = native.load().trie_digest(arrs["parent"], arrs["item"], arrs["count"],
                                                arrs["depth"])["digest"]
            out_q.put((rank, d["digest"], int(d["n_itemsets"]), got))
        except BaseException as e:  # report, so the parent fails fast instead of timing out
            import traceback
            out_q.put((rank, "error", repr(e), traceback.format_exc()))
            raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_deep_split_trie_gathered_on_rank0(gpu_mod, world):
    """The multi-GPU job's deep split (ranks sharing the GPU, host communicator): every rank's
    emitted share compacted on the device and gathered on rank 0 is the whole trie."""
    ms = 0.035
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, ms, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    for _ in range(world):
        res.append(q.get(timeout=150))
        assert res[-1][1] != "error", res[-1]
    res.sort(key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _cpu_digest(gpu_mod, generate("ds1", seed=0), ms)
    for rank, dg, n, got in res:
        assert dg == want["digest"] and n == want["n"]
    assert res[0][3] == want["digest"]


def test_job_full_mining_through_the_deep_engine(tmp_path, gpu_mod):
    """The job (MINER=gpu, RULES_MODE=full) mines with the deep engine: frequent_itemsets.npz
    holds the CPU trie's content, the rule map is still the device pairs_to_csr."""
    from kubernetes_machine_learning_server_amd.job import main as job
    from tests.helpers import job_settings, make_datasets
    make_datasets(tmp_path, shapes=("ds1", "tiny"), seeds=(0, 4))
    cfg = job_settings(tmp_path, miner="gpu", rules_mode="full", min_support=0.04)
    st = job.run(cfg)
    assert st["rule_map"] == "device"
    z = np.load(cfg.pickles_folder / "frequent_itemsets.npz")
    got = gpu_mod.trie_digest(z["parent"], z["item"], z["count"], z["depth"])
    from kubernetes_machine_learning_server_amd.job import preprocess as pp
    t = pp.clean_df(pp.read_tracks(str(tmp_path / "datasets" / "2023_spotify_ds1.csv"), 1.0,
                                   verbose=False))
    tx = pp.group_tracks_by_playlist(t)
    ref = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, len(tx.names), 0.04)
    want = gpu_mod.trie_digest(ref["parent"], ref["item"], ref["count"], ref["depth"])
    assert got["digest"] == want["digest"] and st["n_itemsets"] == want["n"]
    _check_trie(z["parent"], z["depth"])


def _deep_job_worker(rank, world, port, root, fault, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", KMLS_COMM="host",
                      KMLS_COMM_TIMEOUT_S="120", KMLS_DIST_BACKEND="gloo")
    if fault:
        os.environ["KMLS_FAULT"] = fault
    else:
        os.environ.pop("KMLS_FAULT", None)
    import pathlib
    os.chdir(root)
    from kubernetes_machine_learning_server_amd.job import main as job
    from tests.helpers import job_settings
    cfg = job_settings(pathlib.Path(root), miner="gpu", rules_mode="full", min_support=0.04,
                       num_gpus=world, checkpoint_dir=pathlib.Path(root) / "ck",
                       dist_timeout_s=120.0, dist_mode="deep")
    try:
        out_q.put((rank, job.run(cfg), None))
    except Exception as e:  # noqa: BLE001 — the injected fault
        out_q.put((rank, None, repr(e)))


def _run_deep_job(root, world, fault=""):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_deep_job_worker, args=(r, world, port, str(root), fault, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=200) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    return res


def test_deep_split_job_resumes_from_the_trie_checkpoint(tmp_path, gpu_mod):
    """The multi-GPU job's deep split (world 2, ranks sharing the GPU): rank 0 checkpoints the
    gathered trie; after a crash between mining and publishing the restarted job resumes from
    it on every rank (no re-mining) and publishes the CPU trie's content."""
    from tests.helpers import make_datasets
    make_datasets(tmp_path, shapes=("ds1", "tiny"), seeds=(0, 4))
    res = _run_deep_job(tmp_path, 2, fault="after_mining_phase")
    assert all("injected fault" in (r[2] or "") for r in res), res
    assert len(list((tmp_path / "ck").rglob("deeptrie_x2.npz"))) == 1
    res = _run_deep_job(tmp_path, 2)
    assert all(r[2] is None for r in res), res
    summary = res[0][1]
    assert summary["backend"] == "checkpoint" and summary["dataset_index"] == 1
    z = np.load(tmp_path / "api-data" / "pickles" / "frequent_itemsets.npz")
    got = gpu_mod.trie_digest(z["parent"], z["item"], z["count"], z["depth"])
    from kubernetes_machine_learning_server_amd.job import preprocess as pp
    t = pp.clean_df(pp.read_tracks(str(tmp_path / "datasets" / "2023_spotify_ds1.csv"), 1.0,
                                   verbose=False))
    tx = pp.group_tracks_by_playlist(t)
    ref = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, len(tx.names), 0.04)
    want = gpu_mod.trie_digest(ref["parent"], ref["item"], ref["count"], ref["depth"])
    assert got["digest"] == want["digest"] and summary["n_itemsets"] == want["n"]
    assert not list((tmp_path / "ck").rglob("*.npz"))  # cleared after success
