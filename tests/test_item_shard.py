"""Item-sharded bitmaps (``parallel/item_shard.py``, ``DistMiner(mode="shard")``).

CPU tier: world 1/2/3/4 over gloo with the host backend — the gathered trie must equal the
single-process ``mine_cpu`` result itemset for itemset (sets and supports), and each rank may
hold only its item shard's rows (ceil(F/N) of F) plus batch bitmaps <= 1/N of the transactions.
GPU tier: the compress kernel against its numpy reference, and shard mining on one MI355X
(world 1, and ranks sharing the GPU over gloo) equal to ``mine_cpu``.
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


def _sets(par, it, cnt):
    memo, out = [], {}
    for n in range(len(it)):
        s = (memo[par[n]] if par[n] >= 0 else frozenset()) | {int(it[n])}
        memo.append(s)
        out[s] = int(cnt[n])
    return out


def _worker(rank, world, port, shape, ms, max_len, backend, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), OMP_NUM_THREADS="1")
    import torch.distributed as dist
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import (DistMiner, gather_trie,
                                                                            shard_bounds)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tx = generate(shape, seed=3)
        lo, hi, _ = shard_bounds(tx.n_tx, world, rank)
        ptr = tx.tx_ptr[lo:hi + 1]
        dm = DistMiner(ptr, tx.items, tx.n_items, ms, max_len=max_len, backend=backend,
                       mode="shard", global_n_tx=tx.n_tx, device=0, arena_bytes=1 << 30)
        r = None
        for _ in range(2):  # the second call reuses the miner's buffers
            r = dm.step()
        st = r["stats"]
        merged = gather_trie(r["trie"], rank, world, int(st["n_frequent_items"]))
        stats = {k: st[k] for k in ("own_rows", "own_bitmap_bytes", "replicated_bitmap_bytes",
                                    "peak_batch_bitmap_bytes", "rounds", "n_frequent_items",
                                    "batch_cap_bits", "max_root_support")}
        if world > 1:
            allst = [None] * world
            dist.all_gather_object(allst, stats)
        else:
            allst = [stats]
        if rank == 0:
            out_q.put({"merged": merged, "global": st["global_itemsets"], "stats": allst})
    except Exception as e:  # noqa: BLE001
        out_q.put({"error": repr(e), "rank": rank})
        raise
    finally:
        if world > 1:
            dist.destroy_process_group()


def _run(world, shape, ms, max_len=0, backend="cpu"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, shape, ms, max_len, backend, q))
          for r in range(world)]
    for p in ps:
        p.start()
    out = q.get(timeout=600)
    for p in ps:
        p.join(timeout=120)
    assert "error" not in out, out
    return out


def _check(res, world, shape, ms, max_len=0):
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    tx = generate(shape, seed=3)
    ref = native.load().mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms, max_len=max_len)
    m = res["merged"]
    assert res["global"] == ref["stats"]["n_itemsets"] == len(m["item"])
    assert _sets(m["parent"], m["item"], m["count"]) == _sets(ref["parent"], ref["item"],
                                                              ref["count"])
    F = res["stats"][0]["n_frequent_items"]
    for st in res["stats"]:
        # 1/N of the replicated bitmap: only the rows of this rank's items
        assert st["own_rows"] == -(-F // world) or st["own_rows"] == F // world
        assert st["own_bitmap_bytes"] * world <= st["replicated_bitmap_bytes"] + world * 8 * \
            (st["replicated_bitmap_bytes"] // (8 * F))
        # a round's compressed bitmap: F rows of max(T/N, the largest lone root) bits (+ padding)
        bits = max(st["batch_cap_bits"], st["max_root_support"])
        assert st["peak_batch_bitmap_bytes"] <= F * 8 * ((-(-bits // 64) + 7) // 8 * 8)
        assert st["batch_cap_bits"] <= max(64, st["replicated_bitmap_bytes"] // (8 * F) * 64 // world)


def test_compress_np_and_batches():
    from kubernetes_machine_learning_server_amd.parallel.item_shard import compress_np, plan_batches
    rng = np.random.default_rng(0)
    rows = rng.integers(0, 2**63, size=(5, 7), dtype=np.int64).view(np.uint64)
    mask = rng.integers(0, 2**63, size=7, dtype=np.int64).view(np.uint64) & \
        rng.integers(0, 2**63, size=7, dtype=np.int64).view(np.uint64)
    out = compress_np(rows, mask, 8)
    mb = [(int(mask[w]) >> b) & 1 for w in range(7) for b in range(64)]
    for r in range(5):
        rb = [(int(rows[r, w]) >> b) & 1 for w in range(7) for b in range(64)]
        want = [x for x, m in zip(rb, mb) if m]
        got = [(int(out[r, q]) >> b) & 1 for q in range(8) for b in range(64)]
        assert got[:len(want)] == want and not any(got[len(want):])
    b = plan_batches(np.array([0, 2, 4, 6, 8]), np.array([5, 0, 5, 0, 5, 0, 20, 0, 1]), 10)
    assert [x.tolist() for x in b] == [[0, 2], [4], [6], [8]]


@pytest.mark.parametrize("world,shape,ms,max_len", [(1, "ds2_weak", 0.03, 0),
                                                     (2, "ds2_weak", 0.03, 0),
                                                     (3, "tiny", 0.02, 0),
                                                     (4, "ds2_weak", 0.03, 0),
                                                     (2, "ds2_weak", 0.05, 2)])
def test_shard_mode_equals_single_process(world, shape, ms, max_len):
    _check(_run(world, shape, ms, max_len), world, shape, ms, max_len)


@pytest.mark.gpu
@pytest.mark.parametrize("density", ["dense", "sparse", "empty"])
def test_gpu_compact_rows_kernel(density):
    """Masks of ~16 bits per word, of a few bits per many words (one output word gathers many
    input words), and empty."""
    import torch
    from kubernetes_machine_learning_server_amd.ops import native
    from kubernetes_machine_learning_server_amd.parallel.item_shard import compress_np
    N = native.require_gpu()
    g = N.GpuMiner(0)
    rng = np.random.default_rng(1)
    R, W = 37, 1000
    rows = rng.integers(-2**63, 2**63 - 1, size=(R, W), dtype=np.int64)
    mask = rng.integers(-2**63, 2**63 - 1, size=W, dtype=np.int64)
    mask &= rng.integers(-2**63, 2**63 - 1, size=W, dtype=np.int64)
    mask[::7] = 0
    if density == "sparse":
        mask = np.where(rng.random(W) < 0.3, np.int64(1) << rng.integers(0, 63, size=W), 0)
        mask = mask.astype(np.int64)
    elif density == "empty":
        mask[:] = 0
    d_rows = torch.from_numpy(rows).cuda()
    d_mask = torch.from_numpy(mask).cuda()
    cnt = torch.empty(W, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    g.word_popc(d_mask.data_ptr(), W, cnt.data_ptr())
    g.synchronize()
    c64 = cnt.to(torch.int64)
    nz = torch.nonzero(c64).flatten()
    off = (torch.cumsum(c64, 0) - c64)[nz].contiguous()
    bits = int(c64.sum())
    wc = max(8, (-(-bits // 64) + 7) // 8 * 8)
    out = torch.zeros((R, wc), dtype=torch.int64, device="cuda")
    idx = torch.tensor([3, 5, 30], dtype=torch.int32, device="cuda")
    um = torch.empty(W, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    g.compact_rows(d_rows.data_ptr(), R, W, d_mask.data_ptr(), nz.data_ptr(), off.data_ptr(),
                   nz.numel(), out.data_ptr(), wc)
    g.rows_union(d_rows.data_ptr(), W, idx.data_ptr(), 3, W, um.data_ptr())
    g.synchronize()
    want = compress_np(rows.view(np.uint64), mask.view(np.uint64), wc)
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want)
    assert np.array_equal(um.cpu().numpy(), rows[3] | rows[5] | rows[30])


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2])
def test_gpu_shard_mode_equals_single_process(world):
    """world 2: two ranks share the one GPU (gloo; collectives staged through the host)."""
    _check(_run(world, "ds2_weak", 0.03, 0, backend="gpu"), world, "ds2_weak", 0.03)
