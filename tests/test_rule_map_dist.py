"""Config 5 across ranks (``parallel/rule_map.py``): transaction shards -> supports all-reduce ->
shard gram -> reduce-scatter of full-row blocks -> per-rank rule-map rows -> gather by item id.

CPU tier: the identical protocol with host kernels and the host shared-memory communicator
(gloo for the rendezvous), world 2 and 3; the assembled CSR must equal the world-1 result AND the
rule index built by ``serve.index.build_index_from_trie`` from the CPU miner's pairs (the
reference's rule-map loop, ``machine-learning/main.py:282-304``), and the ``rules.idx`` bytes
must not depend on the world size.  GPU tier: ranks sharing one MI355X over the native host
communicator, byte-equal to the single-GPU ``rule_map_from_gram`` artifact.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

SHAPE, MS = "ds2_weak", 0.01


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _idx_bytes(csr, tx, ids):
    from kubernetes_machine_learning_server_amd.serve.index import index_from_device_csr
    ix = index_from_device_csr(csr, tx.n_items, ids, tx.n_tx)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "rules.idx")
        ix.save(p)
        with open(p, "rb") as f:
            return f.read()


def _worker(rank, world, port, backend, comm, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), OMP_NUM_THREADS="1")
    import torch.distributed as dist
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import shard_bounds
    from kubernetes_machine_learning_server_amd.parallel.rule_map import DistRuleMap
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tx = generate(SHAPE, seed=5)
        lo, hi, _ = shard_bounds(tx.n_tx, world, rank)
        ptr = tx.tx_ptr[lo:hi + 1] - tx.tx_ptr[lo]
        items = tx.items[tx.tx_ptr[lo]:tx.tx_ptr[hi]]
        rm = DistRuleMap(ptr, items, tx.n_items, tx.n_tx, MS, device=0, backend=backend,
                         comm_backend=comm)
        r = None
        for _ in range(2):  # a second call reuses the held buffers
            r = rm.step()
        if rank == 0:
            out_q.put({k: r[k] for k in ("row_ptr", "cons", "count", "ids", "nnz", "status",
                                         "n_frequent_items")})
    except Exception as e:  # noqa: BLE001
        out_q.put({"error": repr(e), "rank": rank})
        raise
    finally:
        if world > 1:
            dist.destroy_process_group()


def _run(world, backend, comm="host"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, backend, comm, q))
          for r in range(world)]
    for p in ps:
        p.start()
    out = q.get(timeout=600)
    for p in ps:
        p.join(timeout=120)
    assert "error" not in out, out
    return out


def _same(a, b):
    for k in ("row_ptr", "cons", "count"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k


def test_assemble_by_id_roundtrip():
    from kubernetes_machine_learning_server_amd.parallel.rule_map import assemble_by_id
    ids = np.array([5, 1, 3], np.int64)            # rank order -> item ids
    lens = np.array([2, 1, 0], np.int64)           # rows of ids 5, 1, 3
    cons = np.array([1, 3, 5], np.int32)
    cnt = np.array([9, 8, 7], np.uint32)
    out = assemble_by_id(ids, lens, cons, cnt, 6)
    assert out["row_ptr"].tolist() == [0, 0, 1, 1, 1, 1, 3]
    assert out["cons"].tolist() == [5, 1, 3] and out["count"].tolist() == [7, 9, 8]


@pytest.mark.parametrize("world", [2, 3])
def test_dist_rule_map_cpu_equals_single_and_cpu_index(world):
    from kubernetes_machine_learning_server_amd.bench.bench_mine import cpu_index, index_equal
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    one = _run(1, "cpu")
    many = _run(world, "cpu")
    assert one["n_frequent_items"] > 50 and one["nnz"] > 1000
    _same(one, many)
    N = native.load()
    tx = generate(SHAPE, seed=5)
    ref = cpu_index(N, tx, MS, None)
    assert index_equal(many, ref)
    assert _idx_bytes(many, tx, many["ids"]) == _idx_bytes(one, tx, one["ids"])


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_dist_rule_map_gpu_host_comm_equals_single_gpu(world):
    """Ranks sharing one GPU (native host communicator): rules.idx byte-equal to the 1-GPU
    rule_map_from_gram artifact."""
    import torch
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    N = native.require_gpu()
    tx = generate(SHAPE, seed=5)
    g = N.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    cnt = torch.zeros(tx.n_items, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # torch's fill ran on its stream, the miner has its own
    g.item_support(cnt.data_ptr())
    torch.cuda.synchronize()
    F = g.select(cnt.cpu().numpy().view(np.uint32), tx.n_tx, MS)
    ids, _, minsup = g.frequent()
    Wp = g.words_local()
    bm = torch.zeros((F, Wp), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    g.encode_bitmaps(bm.data_ptr(), Wp, 0)
    gram = torch.empty((F, F), dtype=torch.int32, device="cuda")
    g.pair_counts(bm.data_ptr(), Wp, gram.data_ptr(), True)
    ref = g.rule_map_from_gram(gram.data_ptr(), F, int(minsup))
    torch.cuda.synchronize()
    assert ref["status"] == 0
    one = _run(1, "gpu")
    _same(one, ref)
    many = _run(world, "gpu", "host")
    _same(many, ref)
    assert _idx_bytes(many, tx, many["ids"]) == _idx_bytes(ref, tx, ids)


def _ck_worker(rank, world, port, root, fault, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), OMP_NUM_THREADS="1")
    if fault:
        os.environ["KMLS_FAULT"] = fault
    import torch.distributed as dist
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import shard_bounds
    from kubernetes_machine_learning_server_amd.parallel.rule_map import DistRuleMap
    from kubernetes_machine_learning_server_amd.utils.checkpoint import PhaseCheckpoint
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tx = generate(SHAPE, seed=5)
        lo, hi, _ = shard_bounds(tx.n_tx, world, rank)
        ck = PhaseCheckpoint(root, {"run": "rule-map-test"})
        rm = DistRuleMap(tx.tx_ptr[lo:hi + 1] - tx.tx_ptr[lo], tx.items[tx.tx_ptr[lo]:tx.tx_ptr[hi]],
                         tx.n_items, tx.n_tx, MS, backend="cpu", ck=ck)
        r = rm.step()
        if rank == 0:
            out_q.put({k: r[k] for k in ("row_ptr", "cons", "count", "resumed_from_phase")})
    except Exception as e:  # noqa: BLE001 — the injected fault
        if rank == 0:
            out_q.put({"error": repr(e)})
    finally:
        dist.destroy_process_group()


def test_dist_rule_map_phase_checkpoints(tmp_path):
    """SURVEY §5.4 at config-5 scale: supports, every rank's reduce-scattered gram rows and CSR
    rows are checkpointed; a run that dies after the CSR phase resumes from it on restart (no
    gram recomputed) and assembles the same map."""
    def run(fault=""):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        ps = [ctx.Process(target=_ck_worker, args=(r, 2, port, str(tmp_path), fault, q))
              for r in range(2)]
        for p in ps:
            p.start()
        out = q.get(timeout=600)
        for p in ps:
            p.join(timeout=120)
        return out
    crashed = run("rulemap_after_csr")
    assert "injected fault" in crashed.get("error", ""), crashed
    names = sorted(p.name for p in tmp_path.rglob("*.npz"))
    assert "rulemap_supports.npz" in names and "rulemap_rows_r1of2.npz" in names, names
    resumed = run()
    assert resumed.get("resumed_from_phase") == 3, resumed
    ref = _run(1, "cpu")
    _same(resumed, ref)
