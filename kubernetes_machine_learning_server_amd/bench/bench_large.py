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
    ap.add_argument("--mfma", action="store_true")
    ap.add_argument("--rules", action="store_true", help="also time rules + index + hot reload")
    ap.add_argument("--min-confidence", type=float, default=0.3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--pairs", default="", choices=["", "allreduce", "reduce_scatter", "alltoall", "ring"],
                    help="pairs-only pipeline (RULES_MODE=pairs) with this distributed strategy")
    args = ap.parse_args(argv)

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
                   support_tiles=args.tiles, **kw)
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


if __name__ == "__main__":
    sys.exit(main())
