"""Large-shape pipeline benchmark — BASELINE configs 3 ("10M-transaction x 1M-item synthetic,
item-sharded FP-Growth across 8 GPUs") and 5 ("100M-transaction bitmap + rule-gen + hot-reload
serve").  The reference has no such configuration (its job is one mlxtend process over a 240k-row
CSV); this measures the MI355X design at that scale.

Each rank generates ONLY its transaction shard (``synth_transactions(tx_begin, tx_end)`` is
bit-identical to the same rows of the full dataset), so host memory is T/N per process.  Timed
step = the whole mining call: tiled supports (+ overlapped all-reduce), frequent-item selection,
shard bitmap encode, level-2 gram, all levels (candidate counts all-reduced per level in
``mode=tx``), trie download on rank 0.  With ``--rules`` rank 0 then times association rules
(native), the serving index build, the ``rules.idx`` write and a hot reload of it (C++ matcher
+ HBM index).

Run: ``python -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M``
(N GPUs: ``torchrun --nproc-per-node N --master-addr 127.0.0.1 -m ...bench_large``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="10Mx1M")
    ap.add_argument("--n-tx", type=int, default=0, help="override the shape's transaction count")
    ap.add_argument("--min-support", type=float, default=0.001)
    ap.add_argument("--max-len", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", default="tx", choices=["tx", "item", "auto"])
    ap.add_argument("--tiles", type=int, default=4, help="support tiles (all-reduce overlap)")
    ap.add_argument("--arena-gb", type=float, default=48.0,
                    help="device arena of the level loop (>10k frequent items need >8 GB)")
    ap.add_argument("--mfma", action="store_true")
    ap.add_argument("--rules", action="store_true", help="also time rules + index + hot reload")
    ap.add_argument("--min-confidence", type=float, default=0.3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--pairs", default="", choices=["", "allreduce", "reduce_scatter", "alltoall", "ring"],
                    help="pairs-only pipeline (RULES_MODE=pairs) with this distributed strategy")
    ap.add_argument("--rule-map", action="store_true",
                    help="config 5: the deployed artifact (pair rule map) at HBM scale, every "
                         "rank of the job (transaction shards, gram row reduce-scatter)")
    ap.add_argument("--verify-rows", type=int, default=64,
                    help="--rule-map: gram rows re-counted by the independent popcount kernel")
    args = ap.parse_args(argv)
    if args.rule_map:
        return rule_map_main(args)

    import numpy as np
    import torch
    import torch.distributed as dist

    from ..data.synthetic import SHAPES
    from ..ops import native
    from ..parallel.dist_miner import DistMiner, shard_bounds

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    N = native.require_gpu()
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    shape = SHAPES[args.shape]
    T = args.n_tx or shape.n_tx
    t0 = time.perf_counter()
    if args.pairs:
        args.mode = "item"  # transaction-sharded protocol; the shard is generated per rank
    if args.mode == "item" and not args.pairs:
        ptr, items = N.synth_transactions(T, shape.n_items, shape.mean_len, shape.n_genres,
                                          shape.genre_affinity, 0.85, args.seed)
        kw = {}
    else:
        lo, hi, _ = shard_bounds(T, world, rank)
        ptr, items = N.synth_transactions(T, shape.n_items, shape.mean_len, shape.n_genres,
                                          shape.genre_affinity, 0.85, args.seed, 0, lo, hi)
        kw = {"global_n_tx": T}
    gen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    dm = DistMiner(ptr, items, shape.n_items, args.min_support, device=local_rank,
                   max_len=args.max_len, mfma=args.mfma, mode=args.mode,
                   support_tiles=args.tiles, arena_bytes=int(args.arena_gb * (1 << 30)), **kw)
    load_s = time.perf_counter() - t0

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize()

    if args.pairs:
        for _ in range(args.warmup):
            dm.pair_rows(args.pairs)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ids, r0, r1, rows = dm.pair_rows(args.pairs)
        dm.synchronize()
        barrier()
        ms = (time.perf_counter() - t0) * 1000.0 / max(1, args.steps)
        if world > 1:
            t = torch.tensor([ms], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ms = float(t.item())
        if rank == 0:
            print(json.dumps({"bench": "large-pairs", "shape": args.shape, "n_tx": T,
                              "n_gpus": world, "pairs_mode": args.pairs,
                              "n_frequent_items": int(len(ids)), "rows_owned": int(r1 - r0),
                              "ms_per_step": round(ms, 3),
                              "tx_per_s": round(T / (ms / 1000.0), 1)}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return 0
    r = None
    for _ in range(args.warmup):
        r = dm.step(download=True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = dm.step(download=True)
    dm.synchronize()
    barrier()
    ms = (time.perf_counter() - t0) * 1000.0 / max(1, args.steps)
    if world > 1:
        t = torch.tensor([ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
    st = r["stats"]
    out = {
        "bench": "large", "shape": args.shape, "n_tx": T, "n_items": shape.n_items,
        "nnz_local": int(len(items)), "n_gpus": world, "mode": dm.mode,
        "min_support": args.min_support, "ms_per_step": round(ms, 3),
        "tx_per_s": round(T / (ms / 1000.0), 1),
        "itemsets": int(st.get("global_itemsets", st.get("n_itemsets", 0))),
        "itemsets_per_s": round(int(st.get("global_itemsets", 0)) / (ms / 1000.0), 1),
        "n_frequent_items": int(st.get("n_frequent_items", 0)),
        "max_depth": int(st.get("max_depth", 0)),
        "levels_path": st.get("levels_path"), "phases_ms": st.get("phases_ms"),
        "gen_s_local_shard": round(gen_s, 2), "load_s": round(load_s, 2),
    }
    if args.rules and rank == 0:
        from ..models.fpgrowth import ItemsetTrie
        from ..models.rules import rules_from_trie
        from ..serve.index import RuleIndexData, build_index_from_trie
        tr = r["trie"]
        trie = ItemsetTrie(tr["parent"], tr["item"], tr["count"], tr["depth"], T,
                           args.min_support, dict(st), None)
        t1 = time.perf_counter()
        rules = rules_from_trie(trie, "confidence", args.min_confidence)
        out["rules"] = len(rules)
        out["rules_ms"] = round((time.perf_counter() - t1) * 1000, 2)
        t1 = time.perf_counter()
        idx = build_index_from_trie(tr["parent"], tr["item"], tr["count"], tr["depth"], T,
                                    shape.n_items)
        out["index_build_ms"] = round((time.perf_counter() - t1) * 1000, 2)
        out["index_keys"], out["index_nnz"] = idx.n_keys, idx.nnz
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "rules.idx")
            t1 = time.perf_counter()
            idx.save(path)
            out["index_write_ms"] = round((time.perf_counter() - t1) * 1000, 2)
            t1 = time.perf_counter()
            back = RuleIndexData.load(path)
            back.native()
            out["reload_cpu_ms"] = round((time.perf_counter() - t1) * 1000, 2)
            t1 = time.perf_counter()
            g = N.GpuRuleIndex(local_rank, back.native())
            out["reload_hbm_ms"] = round((time.perf_counter() - t1) * 1000, 2)
            del g
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def rule_map_main(args) -> int:
    """BASELINE config 5: the reference's deployed artifact (the rule map = the pair-support
    matrix, machine-learning/main.py:282-296) at a min_support that leaves >10k frequent items of
    a 1M vocabulary, over 100M transactions — the bitmap alone is ~185 GB of HBM at one GPU.

    One process per GPU (``torchrun --nproc-per-node N``; N = 1 without torchrun): every rank
    generates ONLY its transaction shard and runs ``parallel.rule_map.DistRuleMap``: shard
    supports + all-reduce, selection, banded LDS-slab encode, MFMA gram of the shard, mirror,
    reduce-scatter of full-row blocks over the native communicator (RCCL), the CSR of its rows,
    gather to rank 0 by item id.  Timed step = that whole call, max over ranks.  Then on rank 0:
    the rules.idx write, a hot reload into the C++ matcher and the HBM index, batched queries.
    Verification: ``--verify-rows`` rows of every rank's shard gram re-counted by the popcount
    bit-GEMM (a different kernel), and sampled rule-map rows checked against co-occurrence counts
    computed on the host from every shard's CSR (all-reduced)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from ..data.synthetic import SHAPES
    from ..ops import native
    from ..parallel.dist_miner import shard_bounds
    from ..parallel.rule_map import DistRuleMap
    from ..serve.index import RuleIndexData, index_from_device_csr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    N = native.require_gpu()
    dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    own_group = False
    if world > 1 and not dist.is_initialized():  # (bench.py calls in with its group up)
        import datetime
        own_group = True
        backend = os.environ.get("KMLS_BENCH_DIST", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev),
                                    timeout=datetime.timedelta(seconds=600))
        else:  # ranks sharing a GPU (rehearsal): gloo rendezvous + the host communicator
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=600))
    shape = SHAPES[args.shape]
    T, I = args.n_tx or shape.n_tx, shape.n_items
    lo, hi, _ = shard_bounds(T, world, rank)
    t0 = time.perf_counter()
    ptr, items = N.synth_transactions(T, I, shape.mean_len, shape.n_genres, shape.genre_affinity,
                                      0.85, args.seed, 0, lo, hi)
    gen_s = time.perf_counter() - t0
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(dev)[0]  # every allocation (native hipMalloc included)
    t0 = time.perf_counter()
    rm = DistRuleMap(ptr, items, I, T, args.min_support, device=dev)
    load_s = time.perf_counter() - t0
    out = {"bench": "large-rule-map", "shape": args.shape, "n_tx": T, "n_items": I,
           "nnz_local": int(len(items)), "n_gpus": world,
           "parallelism": f"tx-shard{world}+gram-row-reduce-scatter({rm.comm_backend})"
           if world > 1 else "single", "min_support": args.min_support,
           "gen_s_local_shard": round(gen_s, 2), "load_s": round(load_s, 2)}

    def bar():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    r = None
    for _ in range(args.warmup):
        r = rm.step()
    bar()
    t0 = time.perf_counter()
    for _ in range(max(1, args.steps)):
        r = rm.step()
    bar()
    ms = (time.perf_counter() - t0) * 1000.0 / max(1, args.steps)
    if world > 1:
        t = torch.tensor([ms], dtype=torch.float64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
    g = rm.ops.g
    ids, fcounts, minsup = g.frequent()
    ids = np.asarray(ids)
    F = len(ids)
    Ws = rm.ops.Ws
    out.update({"ms_per_step": round(ms, 1), "n_frequent_items": int(F),
                "bitmap_gb_per_rank": (round(F * Ws * 8 / 1e9, 1)
                                       if "bm" in rm.ops.held else 0.0),
                "bitmap_gb_replicated_equiv": round(F * Ws * 8 * world / 1e9, 1),
                "gram_gb": round(F * F * 4 / 1e9, 2),
                # device memory the rule map holds after its steps (its buffers are grow-only and
                # kept across calls, so this is the high-water mark): hipMemGetInfo before the
                # miner existed minus now — native hipMalloc buffers included, unlike torch's
                # allocator statistics
                "hbm_gb_used_rank0": round((free0 - torch.cuda.mem_get_info(dev)[0]) / 1e9, 2),
                "hbm_gb_torch_allocator_rank0": round(torch.cuda.max_memory_allocated() / 1e9, 2)})
    if rank == 0:
        out.update({"rule_map_entries": int(r["nnz"]), "rule_map_status": int(r["status"]),
                    "frequent_pairs": int(r["nnz"]) // 2,
                    "phase_wall_ms_rank0": r["phases_ms"]})
    # 1. each rank's shard gram rows re-counted independently: by the popcount bit-GEMM over the
    # shard's bitmaps when the gram came from them, by the host from the shard's CSR when the
    # gram was counted horizontally (cooc.hip: no bitmaps exist)
    out["level2_method"] = getattr(rm.ops, "method", "gram")
    gram = rm.ops.held["gram"]
    bm = rm.ops.held.get("bm")
    k = min(args.verify_rows, F)
    gm = gram[:k, :F].cpu().numpy()
    if bm is not None:
        chk = torch.zeros((k, F), dtype=torch.int32, device="cuda")
        g.bitgemm_rect(bm.data_ptr(), k, bm.data_ptr(), F, Ws, chk.data_ptr(), F)
        torch.cuda.synchronize()
        ck = chk.cpu().numpy()
        del chk
    else:
        rank_of = np.full(I, -1, np.int64)
        rank_of[ids] = np.arange(F)
        sel = np.zeros(I, bool)
        sel[ids[:k]] = True
        pos_ = np.flatnonzero(sel[items])           # occurrences of the k checked items
        rows_r = rank_of[items[pos_]]
        txs = np.searchsorted(ptr, pos_, side="right") - 1
        lens = (ptr[txs + 1] - ptr[txs]).astype(np.int64)
        first = np.repeat(ptr[txs] - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)
        seg = items[first + np.arange(int(lens.sum()))]   # every item of those transactions
        rk = rank_of[seg]
        rr = np.repeat(rows_r, lens)
        keep = rk >= 0
        ck = np.bincount(rr[keep] * F + rk[keep], minlength=k * F).reshape(k, F)
    # (the gram holds the mirrored shard counts before the reduce-scatter: full rows, so every
    # off-diagonal entry of the k rows is compared — upper entries and their mirror images)
    off = np.ones(gm.shape, bool)
    off[np.arange(k), np.arange(k)] = False
    ok_rows = bool(np.array_equal(gm[off].astype(np.int64), ck[off].astype(np.int64)))
    # 2. sampled rule-map rows vs host co-occurrence counts, summed over the shards
    rng = np.random.default_rng(1)
    sample = np.sort(rng.choice(ids, size=min(6, F), replace=False)).astype(np.int32)
    pos = np.flatnonzero(np.isin(items, sample))
    tx_of = np.searchsorted(ptr, pos, side="right") - 1
    tids = {int(x): np.unique(tx_of[items[pos] == x]) for x in sample}
    co = np.zeros((len(sample), len(sample)), np.int64)
    for a_, x in enumerate(sample):
        for b_, y in enumerate(sample):
            co[a_, b_] = np.intersect1d(tids[int(x)], tids[int(y)], assume_unique=True).size
    flags = np.array([int(ok_rows)], np.int64)
    if world > 1:
        tco = torch.from_numpy(co)
        tfl = torch.from_numpy(flags)
        if dist.get_backend() == "nccl":
            tco, tfl = tco.cuda(), tfl.cuda()
        dist.all_reduce(tco)
        dist.all_reduce(tfl, op=dist.ReduceOp.MIN)
        co, flags = tco.cpu().numpy(), tfl.cpu().numpy()
    out["verified_gram_rows_all_ranks"] = bool(flags[0])
    if rank == 0:
        row_ptr, cons, rcount = r["row_ptr"], r["cons"], r["count"]
        ok = True
        for a_, x in enumerate(sample):
            row = slice(int(row_ptr[x]), int(row_ptr[x + 1]))
            c_row, n_row = cons[row], rcount[row]
            ok &= bool(np.all(np.diff(n_row.astype(np.int64)) <= 0))  # count desc
            got = dict(zip(c_row.tolist(), n_row.tolist()))
            for b_, y in enumerate(sample):
                if y == x:
                    continue
                want = int(co[a_, b_])
                ok &= (got.get(int(y), 0) == want) if want >= minsup else (int(y) not in got)
        out["verified_rule_map_sample"] = bool(ok)
    rm.release()
    del bm, gram
    if rank == 0:
        # 3. artifact: rules.idx write, hot reload into the C++ matcher + HBM index, queries
        ix = index_from_device_csr({"row_ptr": r["row_ptr"], "cons": r["cons"],
                                    "count": r["count"]}, I, ids, T)
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "rules.idx")
            t1 = time.perf_counter()
            ix.save(path)
            out["index_write_ms"] = round((time.perf_counter() - t1) * 1000, 1)
            out["index_bytes"] = os.path.getsize(path)
            t1 = time.perf_counter()
            back = RuleIndexData.load(path)
            host = back.native()
            out["reload_cpu_ms"] = round((time.perf_counter() - t1) * 1000, 1)
            t1 = time.perf_counter()
            gidx = N.GpuRuleIndex(dev, host)
            out["reload_hbm_ms"] = round((time.perf_counter() - t1) * 1000, 1)
            # rows here hold thousands of entries: past the HIP kernel's per-wave LDS table, so
            # its queries take the host path inside query_batch (measured, not hidden)
            for B in (1, 64, 1024):
                lens = rng.integers(1, 6, size=B)
                q_ptr = np.zeros(B + 1, np.int64)
                np.cumsum(lens, out=q_ptr[1:])
                seeds = ids[rng.integers(0, F, int(q_ptr[-1]))].astype(np.int32)
                res = {}
                for nm, fn in (("cpp", host.query_batch), ("hip", gidx.query_batch)):
                    fn(q_ptr, seeds, 10)
                    t1 = time.perf_counter()
                    reps = 3
                    for _ in range(reps):
                        got = fn(q_ptr, seeds, 10)
                    res[nm] = ((time.perf_counter() - t1) / reps * 1e6, got)
                same = bool(np.array_equal(res["cpp"][1][0], res["hip"][1][0]) and
                            np.array_equal(res["cpp"][1][1], res["hip"][1][1]))
                out[f"query_batch{B}_us"] = {"cpp": round(res["cpp"][0], 1),
                                             "hip": round(res["hip"][0], 1), "same": same}
            del gidx
            pvc = getattr(args, "pvc_dir", None)
            if pvc:
                out["pvc"] = write_config5_pvc(pvc, r, I, ids, fcounts, T, minsup)
        if not getattr(args, "quiet", False):
            print(json.dumps(out), flush=True)
    if world > 1 and own_group:
        dist.destroy_process_group()
    args.result = out
    return 0


def write_config5_pvc(pvc_dir: str, r: dict, I: int, ids, fcounts, T: int, minsup: int,
                      alt_factor: float = 1.5, top: float = 0.03) -> dict:
    """A serving PVC of the config-5 artifact (``<pvc>/api-data/{pickles/rules.idx,
    pickles/best_tracks.pickle, last_execution.txt}``) plus ``<pvc>/rules_alt.idx``, the rule
    map of the same data at alt_factor x the support (the pair rows filtered to counts >= the
    higher threshold, keys = items frequent at it): what the next job run would publish, for the
    reload-under-load run (``bench_serve --reload-index``)."""
    import pathlib
    import pickle
    import numpy as np
    from ..serve.index import index_from_device_csr
    base = pathlib.Path(pvc_dir) / "api-data"
    pk = base / "pickles"
    pk.mkdir(parents=True, exist_ok=True)
    names = [f"track_{i}" for i in range(I)]  # random-init vocabulary (make_large_pvc.py)
    ix = index_from_device_csr({k: r[k] for k in ("row_ptr", "cons", "count")}, I, ids, T, names)
    ix.save(pk / "rules.idx")
    ix.save(pathlib.Path(pvc_dir) / "rules_main.idx")  # to restore between reload runs
    fc = np.asarray(fcounts, np.int64)
    order = np.argsort(-fc, kind="stable")[:max(10, int(len(ids) * top))]
    best = [{"track_name": f"track_{int(ids[o])}", "count": int(fc[o])} for o in order]
    with open(pk / "best_tracks.pickle", "wb") as f:
        pickle.dump(best, f)
    (base / "last_execution.txt").write_text("initial")
    ms2 = int(np.ceil(minsup * alt_factor))
    row_ptr = np.asarray(r["row_ptr"], np.int64)
    cons, cnt = np.asarray(r["cons"]), np.asarray(r["count"])
    keep = cnt >= ms2
    csum = np.zeros(len(cnt) + 1, np.int64)
    np.cumsum(keep, out=csum[1:])
    per_row = csum[row_ptr[1:]] - csum[row_ptr[:-1]]
    rp2 = np.zeros(I + 1, np.int64)
    np.cumsum(per_row, out=rp2[1:])
    ids2 = np.asarray(ids)[fc >= ms2]
    alt = index_from_device_csr({"row_ptr": rp2, "cons": cons[keep], "count": cnt[keep]}, I,
                                ids2, T, names)
    alt_path = pathlib.Path(pvc_dir) / "rules_alt.idx"
    alt.save(alt_path)
    return {"dir": str(pvc_dir), "keys": int(ix.n_keys), "alt_keys": int(alt.n_keys),
            "alt_min_count": ms2, "alt_entries": int(keep.sum())}


def run_rule_map(shape: str = "100Mx1M", min_support: float = 2e-4, steps: int = 3,
                 warmup: int = 1, n_tx: int = 0, seed: int = 0, verify_rows: int = 64,
                 pvc_dir: str = "") -> dict:
    """``rule_map_main`` as a function (bench.py's config-5 section): every rank of the caller's
    process group (or one process) generates its shard and times ``DistRuleMap.step``; the
    result dict (complete on rank 0) is returned instead of printed.  ``pvc_dir``: rank 0 also
    writes the serving PVC of the artifact (``write_config5_pvc``)."""
    ns = argparse.Namespace(shape=shape, n_tx=n_tx, min_support=min_support, steps=steps,
                            warmup=warmup, seed=seed, verify_rows=verify_rows, quiet=True,
                            pvc_dir=pvc_dir)
    rule_map_main(ns)
    return ns.result


if __name__ == "__main__":
    sys.exit(main())
