"""Multi-process tests of the distributed mining protocol on CPU (gloo), SURVEY §7.6.

Same code path as the RCCL run (``parallel/dist_miner.py``) with the CPU device-ops backend:
tx-sharded supports + all_reduce, bitmap all_gather re-shard, LPT item-sharded DFS, sub-trie
gather.  The merged result must equal the single-process miner exactly.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, shape, ms, max_len, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), OMP_NUM_THREADS="1")
    import torch.distributed as dist
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import DistMiner, gather_trie
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tx = generate(shape, seed=3)
        dm = DistMiner(tx.tx_ptr, tx.items, tx.n_items, ms, max_len=max_len, backend="cpu")
        r = dm.step()
        merged = gather_trie(r["trie"], rank, world, int(r["stats"]["n_frequent_items"]))
        if rank == 0:
            out_q.put({"merged": merged, "global": r["stats"]["global_itemsets"],
                       "lo_hi": (dm.lo, dm.hi)})
    finally:
        dist.destroy_process_group()


def _sets(par, it, cnt):
    memo, out = [], {}
    for n in range(len(it)):
        s = (memo[par[n]] if par[n] >= 0 else frozenset()) | {int(it[n])}
        memo.append(s)
        out[s] = int(cnt[n])
    return out


@pytest.mark.parametrize("world,shape,ms,max_len", [(2, "ds2_weak", 0.03, 0), (4, "tiny", 0.02, 0),
                                                     (3, "ds2_weak", 0.05, 2)])
def test_dist_protocol_equals_single_process(world, shape, ms, max_len):
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shape, ms, max_len, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    tx = generate(shape, seed=3)
    ref = native.load().mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms, max_len=max_len)
    m = res["merged"]
    assert res["global"] == ref["stats"]["n_itemsets"] == len(m["item"])
    assert _sets(m["parent"], m["item"], m["count"]) == _sets(ref["parent"], ref["item"], ref["count"])


def test_shard_bounds_and_lpt():
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import lpt_partition, shard_bounds
    T = 2246
    for world in (1, 2, 4, 8):
        spans = [shard_bounds(T, world, r) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == T
        assert all(s[2] % 256 == 0 for s in spans)
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    cost = np.array([10, 1, 1, 1, 9, 2, 2, 5], dtype=float)
    own = lpt_partition(cost, 3)
    loads = [cost[own == r].sum() for r in range(3)]
    assert max(loads) - min(loads) <= cost.max()  # greedy dealing bound
    assert (lpt_partition(cost, 3) == own).all()  # deterministic across ranks


def _pairs_worker(rank, world, port, mode, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), OMP_NUM_THREADS="1")
    import torch.distributed as dist
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import DistMiner
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tx = generate("ds2_weak", seed=4)
        dm = DistMiner(tx.tx_ptr, tx.items, tx.n_items, 0.03, backend="cpu", mode="item")
        ids, r0, r1, rows = dm.pair_rows(mode)
        out_q.put((rank, np.asarray(ids), r0, r1, rows))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["allreduce", "reduce_scatter", "alltoall", "ring"])
@pytest.mark.parametrize("world", [2, 3])
def test_pair_strategies_equal_full_gram(world, mode):
    """DP all-reduce, reduce-scatter (item ownership), all-to-all (Ulysses analog)
    and the ring pass (context-parallel analog) all produce the owned row blocks of XᵀX."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pairs_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    tx = generate("ds2_weak", seed=4)
    ids = parts[0][1]
    X = np.zeros((tx.n_tx, tx.n_items), np.float64)
    for t in range(tx.n_tx):
        X[t, tx.items[tx.tx_ptr[t]:tx.tx_ptr[t + 1]]] = 1.0
    G = (X[:, ids].T @ X[:, ids]).astype(np.int64)
    covered = 0
    for rank, pids, r0, r1, rows in sorted(parts, key=lambda p: p[0]):
        np.testing.assert_array_equal(pids, ids)
        np.testing.assert_array_equal(rows.astype(np.int64), G[r0:r1])
        covered += r1 - r0
    assert covered == len(ids)


# ---------------------------------------------------------------------------------------------
# native shared-memory communicator (KMLS_COMM=host backend) and the tx-DP level loop
def _shm_worker(rank, world, uid, die_rank, out_q):
    os.environ["KMLS_COMM_TIMEOUT_S"] = "4"
    from kubernetes_machine_learning_server_amd.ops import native
    N = native.load()
    c = N.ShmComm(rank, world, uid)
    a = np.arange(10_000_000 // 7, dtype=np.uint32) + rank  # > one 8 MB slot: chunked
    c.all_reduce(a, False)
    b = np.full(5, float(rank), np.float64)
    c.all_reduce(b, True)
    res = {"rank": rank, "sum_ok": bool((a == np.arange(a.size, dtype=np.uint32) * world +
                                          sum(range(world))).all()),
           "max": b.tolist()}
    if rank == die_rank:
        out_q.put(res)
        return  # leaves without entering the next collective
    try:
        c.barrier()
        res["after"] = "ok"
    except RuntimeError as e:
        res["after"] = str(e)
    out_q.put(res)


@pytest.mark.parametrize("world", [2, 3])
def test_shm_comm_collectives_and_abort(world):
    """Host communicator: chunked all-reduce (sum, max) over processes, then a rank that leaves
    makes every other rank's next wait raise (bounded by KMLS_COMM_TIMEOUT_S), not hang."""
    from kubernetes_machine_learning_server_amd.ops import native
    uid = native.load().host_comm_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shm_worker, args=(r, world, uid, world - 1, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert r["sum_ok"] and r["max"] == [float(world - 1)] * 5
    for r in res[:-1]:
        assert "timed out" in r["after"] or "aborted" in r["after"], r


def _shm_p2p_worker(rank, world, uid, out_q):
    os.environ["KMLS_COMM_TIMEOUT_S"] = "20"
    from kubernetes_machine_learning_server_amd.ops import native
    c = native.load().ShmComm(rank, world, uid)
    n = 3_000_001  # blocks of 12 MB (u32): past one 8 MB slot, chunked
    send = (np.arange(world * n, dtype=np.uint64) * (rank + 1)).astype(np.uint32)
    rs = c.reduce_scatter(send)
    a2a_send = np.arange(world * 1000, dtype=np.int64) + 10_000 * rank
    a2a = c.all_to_all(a2a_send)
    ring = c.sendrecv(np.full(2_500_000, rank, np.int64), (rank + 1) % world, (rank - 1) % world)
    out_q.put((rank, rs[:5].tolist(), int(rs[-1]), a2a.tolist(), int(ring[0]), int(ring[-1])))


@pytest.mark.parametrize("world", [2, 4])
def test_shm_comm_reduce_scatter_alltoall_sendrecv(world):
    """Host communicator's new collectives against numpy: reduce-scatter of row blocks (the
    config-5 gram), all-to-all (the item re-shard) and a ring shift (the context-parallel pass),
    all past one shared-memory slot."""
    from kubernetes_machine_learning_server_amd.ops import native
    uid = native.load().host_comm_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shm_p2p_worker, args=(r, world, uid, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 3_000_001
    tot = sum(r + 1 for r in range(world))
    for rank, head, last, a2a, r0, r1 in res:
        full = (np.arange(world * n, dtype=np.uint64) * tot).astype(np.uint32)
        blk = full[rank * n:(rank + 1) * n]
        assert head == blk[:5].tolist() and last == int(blk[-1])
        want = np.concatenate([np.arange(rank * 1000, (rank + 1) * 1000) + 10_000 * src
                               for src in range(world)])
        assert a2a == want.tolist()
        assert r0 == r1 == (rank - 1) % world


def _txdp_worker(rank, world, port, shape, ms, max_len, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), OMP_NUM_THREADS="1")
    import torch.distributed as dist
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import DistMiner
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tx = generate(shape, seed=5)
        dm = DistMiner(tx.tx_ptr, tx.items, tx.n_items, ms, max_len=max_len, backend="cpu",
                       mode="tx")
        r = dm.step()["trie"]
        d = native.load().trie_digest(r["parent"], r["item"], r["count"], r["depth"])
        out_q.put((rank, d["digest"], d["n"], (dm.lo, dm.hi)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,shape,ms,max_len", [(2, "ds2_weak", 0.03, 0), (4, "tiny", 0.02, 0),
                                                     (3, "ds1", 0.05, 4)])
def test_txdp_level_loop_multi_process(world, shape, ms, max_len):
    """Transaction-DP protocol with the native level loop (supports + every level's candidate
    counts all-reduced through the host communicator): every rank builds the identical global
    trie, whose (itemset, support) digest equals the single-process CPU miner's."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_txdp_worker, args=(r, world, port, shape, ms, max_len, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    tx = generate(shape, seed=5)
    N = native.load()
    ref = N.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms, max_len)
    rd = N.trie_digest(ref["parent"], ref["item"], ref["count"], ref["depth"])
    assert {r[1] for r in res} == {rd["digest"]}
    assert all(r[2] == rd["n"] for r in res)
    spans = sorted(r[3] for r in res)
    assert spans[0][0] == 0 and spans[-1][1] == tx.n_tx  # the shards cover every transaction


def test_relabel_keeps_itemsets():
    """The weak-scaled bench's per-rank dataset: permuted ids + shuffled rows, same itemsets."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate, relabel
    from kubernetes_machine_learning_server_amd.ops import native
    N = native.load()
    tx = generate("ds2_weak", seed=1)
    r0 = N.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.03, 0)
    for key in (1, 5):
        t2 = relabel(tx, key)
        assert not np.array_equal(t2.items, tx.items)
        assert sorted(t2.names) == sorted(tx.names)
        r = N.mine_cpu(t2.tx_ptr, t2.items, t2.n_items, 0.03, 0)
        assert r["stats"]["n_itemsets"] == r0["stats"]["n_itemsets"]
        assert np.array_equal(np.bincount(r["depth"]), np.bincount(r0["depth"]))


def test_bench_strong_scaling_two_ranks_cpu():
    """bench.py's N-rank contract on the CPU tier: torchrun, one JSON line from rank 0, ONE
    dataset split over the ranks (level-3 tasks t = r mod N), per-size counts + digest combined
    through torch.distributed (gloo here, RCCL on the GPU node) equal to the unsplit count."""
    import json
    import subprocess
    import sys
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=root)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench.py"), "--gpus", "2", "--cpu", "--steps", "2",
           "--warmup", "1", "--min-support", "0.04"]
    p = subprocess.run(cmd, env=env, cwd="/tmp", capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    tx = generate("ds1", seed=0)
    ref = native.load().mine_cpu_count(tx.tx_ptr, tx.items, tx.n_items, 0.04)
    assert out["scaling"] == "strong" and out["n_gpus"] == 0
    assert out["digest"] == ref["digest"]
    assert out["config"]["n_itemsets"] == ref["n_itemsets"] == 573225
    assert out["per_level"] == list(ref["per_level"])[1:]
    assert out["config"]["parallelism"].startswith("dp2-level3-task-split")
    assert abs(out["value"] - ref["n_itemsets"] / (out["ms_per_step"] / 1e3)) / out["value"] < 1e-2
