"""Multi-process GPU tests of the transaction-DP protocol (run on a real MI355X via gpurun).

The GPU boxes have ONE MI355X, so the ranks share it: every rank runs the native tx-DP level
loop (GpuMiner.mine_txdp: tiled supports, shard-local bitmaps, each level's candidate counts
all-reduced in C++) through the host-staged communicator (KMLS_COMM=host: D2H, shared-memory
reduction, H2D).  RCCL itself needs one GPU per rank; its code path is the same Comm interface.
The merged result is checked by content against the single-process CPU miner.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(shape):
    from kubernetes_machine_learning_server_amd.data.synthetic import generate, generate_large
    if shape == "large":
        return generate_large("10Mx1M", seed=7, n_tx=400_000, n_items=200_000), 0.002
    return generate(shape, seed=5), 0.05


def _worker(rank, world, port, shape, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), KMLS_COMM="host", KMLS_COMM_TIMEOUT_S="120")
    import torch.distributed as dist
    from kubernetes_machine_learning_server_amd.ops import native
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import DistMiner
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tx, ms = _data(shape)
        dm = DistMiner(tx.tx_ptr, tx.items, tx.n_items, ms, device=0, mode="tx")
        assert dm.ops.comm.backend == "host"
        out = []
        for _ in range(2):  # the second call reuses the comm stream/events and the arena
            r = dm.step(download=True)
            st = r["stats"]
            d = None
            if rank == 0:
                t = r["trie"]
                d = native.load().trie_digest(t["parent"], t["item"], t["count"], t["depth"])["digest"]
            out.append((int(st["n_itemsets"]), d, st.get("levels_path"), st.get("level2_comm")))
        out_q.put((rank, out, (dm.lo, dm.hi)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,shape", [(2, "ds1"), (4, "ds1"), (2, "large"), (4, "large")])
def test_txdp_multi_rank_on_one_gpu(world, shape):
    from kubernetes_machine_learning_server_amd.ops import native
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shape, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tx, ms = _data(shape)
    N = native.load()
    ref = N.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms)
    rd = N.trie_digest(ref["parent"], ref["item"], ref["count"], ref["depth"])
    for rank, out, _ in res:
        for n, d, path, l2comm in out:
            # the shard grams are combined by a row-block reduce-scatter, not an F^2 all-reduce
            assert l2comm == "reduce_scatter+frequent_allgather", l2comm
            assert n == rd["n"], (rank, n, rd["n"], path)
            if rank == 0:
                assert d == rd["digest"], path
    spans = sorted(r[2] for r in res)
    assert spans[0][0] == 0 and spans[-1][1] == tx.n_tx


def _rccl_worker(shape, out_q):
    os.environ.update(KMLS_COMM="rccl", KMLS_COMM_FORCE="1", KMLS_COMM_TIMEOUT_S="60")
    from kubernetes_machine_learning_server_amd.ops import native
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import DistMiner
    tx, ms = _data(shape)
    dm = DistMiner(tx.tx_ptr, tx.items, tx.n_items, ms, device=0, mode="tx")
    assert dm.ops.comm.backend == "rccl"
    t = dm.step(download=True)["trie"]
    out_q.put(native.load().trie_digest(t["parent"], t["item"], t["count"], t["depth"])["digest"])


@pytest.mark.parametrize("shape", ["ds1", "large"])
def test_txdp_through_a_one_rank_rccl_communicator(shape):
    """The native RCCL communicator (dlopen of the RCCL library, non-blocking init polled against
    the deadline, all-reduces of supports, gram and per-level counts, teardown) forced on for one
    rank: the multi-GPU transport itself needs one GPU per rank, but everything around it runs
    here.  In a child process, so a failure of the library cannot take the test session down."""
    from kubernetes_machine_learning_server_amd.ops import native
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(shape, q))
    p.start()
    d = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    tx, ms = _data(shape)
    N = native.load()
    ref = N.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms)
    assert d == N.trie_digest(ref["parent"], ref["item"], ref["count"], ref["depth"])["digest"]


def _pair_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), KMLS_COMM="host", KMLS_COMM_TIMEOUT_S="120")
    import torch.distributed as dist
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import DistMiner
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tx, ms = _data("ds1")
        dm = DistMiner(tx.tx_ptr, tx.items, tx.n_items, ms, device=0, mode="item")
        got = {}
        for mode in ("reduce_scatter", "ring", "ring"):  # the second ring reuses stream/events
            ids, r0, r1, rows = dm.pair_rows(mode)
            got.setdefault(mode, []).append((r0, r1, np.asarray(rows, np.int64)))
        out_q.put((rank, got, dm._ncomm.backend if getattr(dm, "_ncomm", None) else None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_native_ring_pair_rows_on_one_gpu(world):
    """The context-parallel pair ring in C++ (GpuMiner.ring_pair_rows: shards rotating through
    the native communicator's sendrecv on a side stream) equals the reduce-scatter strategy row
    block for row block, on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pair_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got, backend in res:
        assert backend == "host"
        r0, r1, ref = got["reduce_scatter"][0]
        assert ref.sum() > 0
        for a0, a1, rows in got["ring"]:
            assert (a0, a1) == (r0, r1)
            np.testing.assert_array_equal(rows, ref)


def _shard_worker(rank, world, port, out_q, hooks="cooc=2"):
    # cooc=2: the horizontal plan even where the cost model prefers the GEMM (small F here)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), KMLS_COMM="host", KMLS_COMM_TIMEOUT_S="120",
                      KMLS_TEST_HOOKS=hooks)
    import torch.distributed as dist
    from kubernetes_machine_learning_server_amd.ops import native
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import DistMiner, gather_trie
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        try:
            tx, ms = _data("large")
            dm = DistMiner(tx.tx_ptr, tx.items, tx.n_items, ms, device=0, mode="shard")
            out = []
            for _ in range(2):
                r = dm.step(download=True)
                st = r["stats"]
                t = gather_trie(r["trie"], rank, world, int(st["n_frequent_items"]))
                d = None
                if rank == 0:
                    d = native.load().trie_digest(t["parent"], t["item"], t["count"], t["depth"])
                    d = (d["digest"], d["n"])
                out.append((st.get("levels_path"), int(st["global_itemsets"]), d))
            out_q.put((rank, out))
        except BaseException as e:
            import traceback
            out_q.put((rank, "error", repr(e), traceback.format_exc()))
            raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,hooks", [(1, "cooc=2"), (2, "cooc=2"), (3, "cooc=2"),
                                         (2, "cooc=2,pair_rows=0")])
def test_native_item_shard_on_one_gpu(world, hooks):
    """Item-sharded mining without bitmaps (GpuMiner.mine_shard): each rank all-gathers the
    frequent-rank CSRs, counts the pair rows and horizontal levels of its own items; the
    gathered sub-tries are the whole trie (content digest of the CPU miner).  With the row
    count disabled (pair_rows=0) every rank must decline the native plan together (the
    scattered-atomic fallback would count only the rank's own CSR) and the bitmap shard
    protocol mines instead: the same digest."""
    from kubernetes_machine_learning_server_amd.ops import native
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q, hooks))
             for r in range(world)]
    for p in procs:
        p.start()
    res = []
    for _ in range(world):
        res.append(q.get(timeout=240))
        assert res[-1][1] != "error", res[-1]
    res.sort(key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tx, ms = _data("large")
    N = native.load()
    ref = N.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms)
    rd = N.trie_digest(ref["parent"], ref["item"], ref["count"], ref["depth"])
    for rank, out in res:
        for path, glob, d in out:
            if "pair_rows=0" in hooks:
                assert path != "horizontal-item-shard", path
            else:
                assert path == "horizontal-item-shard", path
            assert glob == rd["n"]
            if rank == 0:
                assert d == (rd["digest"], rd["n"])
