#!/usr/bin/env python3
"""Rank-by-rank probe of the config-5 rule map split over N transaction shards, on ONE GPU: the
work each of N ranks does in parallel, run one rank after the other and timed alone.

BASELINE config 5 (100M transactions x 1M items @ 2e-4, 8 x MI355X) shards the transactions
(``parallel/rule_map.py`` DistRuleMap.step): every rank counts its shard's item supports
(all-reduced), selects the frequent items from the GLOBAL supports, counts its shard's pair gram
from its CSR and mirrors it; the grams are reduce-scattered into row blocks and each rank builds the
CSR of its rows.  Here each rank's shard is generated exactly as the N-rank run generates it
(``synth_transactions(..., lo, hi)``); the global supports are the host sum of the shards' counts
(the all-reduce's result) and the global gram is the device sum of the shard grams (the
reduce-scatter's result), so every rank's local phases run on the inputs the real run gives them:

  supports  zero + item_support of the shard
  select    selection from the global supports (on the device: ``select_device``)
  gram      pair_counts_csr_direct of the shard + gram_mirror
  csr       rule_map_rows of the rank's row block of the GLOBAL gram

The collectives are not run (one GPU).  Their payloads per rank are reported, with a time at an
assumed ring bus bandwidth (``--bus-gbps``).  Checks: the summed shard grams equal the 1-rank gram
(all F x F entries) and the rule-map entry count over the row blocks equals the 1-rank count.

    python scripts/shard_probe.py --worlds 1,2,4,8
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="100Mx1M")
    ap.add_argument("--min-support", type=float, default=2e-4)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--bus-gbps", type=float, default=300.0,
                    help="assumed ring all-reduce / reduce-scatter bus bandwidth per rank (GB/s)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from kubernetes_machine_learning_server_amd.data.synthetic import SHAPES
    from kubernetes_machine_learning_server_amd.ops import native
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import shard_bounds
    from kubernetes_machine_learning_server_amd.parallel.rule_map import row_block
    N = native.require_gpu()
    torch.cuda.set_device(0)
    s = SHAPES[a.shape]
    T, I = s.n_tx, s.n_items
    ref_gram, ref_nnz = None, None

    def sync(g=None):
        if g is not None:
            g.synchronize()
        torch.cuda.synchronize()

    for world in [int(x) for x in a.worlds.split(",")]:
        t_gen = time.perf_counter()
        shards = []
        counts = np.zeros(I, np.uint64)
        for r in range(world):
            lo, hi, _ = shard_bounds(T, world, r)
            ptr, items = N.synth_transactions(T, I, s.mean_len, s.n_genres, s.genre_affinity, 0.85,
                                              a.seed, 0, lo, hi)
            shards.append((ptr, items))
            counts += np.bincount(np.asarray(items), minlength=I).astype(np.uint64)
        counts = counts.astype(np.uint32)  # = the all-reduced supports
        gen_s = time.perf_counter() - t_gen
        ranks, glob, F = [], None, None
        for r, (ptr, items) in enumerate(shards):
            g = N.GpuMiner(0, 1 << 30)
            g.load_csr(ptr, items, I)
            cnt = torch.empty(I, dtype=torch.int32, device="cuda")
            gcnt = torch.from_numpy(counts.view(np.int32)).cuda()  # the all-reduce's result
            best = None
            for _ in range(a.reps):
                sync(g)
                t0 = time.perf_counter()
                cnt.zero_()
                g.item_support(cnt.data_ptr())
                sync(g)
                t1 = time.perf_counter()
                F = g.select_device(gcnt.data_ptr(), T, a.min_support)
                sync(g)
                t2 = time.perf_counter()
                gram = torch.empty((F, F), dtype=torch.int32, device="cuda")
                ok = g.cooc_likely() and g.pair_counts_csr_direct(gram.data_ptr(), F)
                g.gram_mirror(gram.data_ptr(), F, F)
                sync(g)
                t3 = time.perf_counter()
                ph = {"supports": (t1 - t0) * 1e3, "select": (t2 - t1) * 1e3,
                      "gram": (t3 - t2) * 1e3}
                if best is None or sum(ph.values()) < sum(best.values()):
                    best = ph
                if _ + 1 < a.reps:
                    del gram
            if not ok:
                raise SystemExit(f"rank {r}: the horizontal pair count declined")
            local_sup = cnt.cpu().numpy().view(np.uint32)
            glob = gram.clone() if glob is None else glob.add_(gram)
            ranks.append({"rank": r, "n_tx": int(len(ptr) - 1), "nnz": int(len(items)),
                          "supports_local_ok": bool(np.array_equal(
                              local_sup, np.bincount(np.asarray(items), minlength=I))),
                          "phases_ms": {k: round(v, 3) for k, v in best.items()}})
            del gram, g, cnt, gcnt
            torch.cuda.empty_cache()
        # the rule-map rows of every rank's block of the reduced gram (one miner, any shard: the
        # kernel reads only the rows and the selection)
        ptr0, items0 = shards[0]
        g = N.GpuMiner(0, 1 << 30)
        g.load_csr(ptr0, items0, I)
        gcnt = torch.from_numpy(counts.view(np.int32)).cuda()
        g.select_device(gcnt.data_ptr(), T, a.min_support)  # (the same order as the grams')
        minsup = int(g.frequent()[2])
        nnz = 0
        for r in range(world):
            per, r0, nrows = row_block(F, world, r)
            best = None
            for _ in range(a.reps):
                sync(g)
                t0 = time.perf_counter()
                m = g.rule_map_rows(glob[r0].data_ptr() if nrows else glob.data_ptr(), F, r0,
                                    nrows, minsup)
                sync(g)
                dt = (time.perf_counter() - t0) * 1e3
                best = dt if best is None else min(best, dt)
            ranks[r]["phases_ms"]["csr"] = round(best, 3)
            ranks[r]["rows"] = int(nrows)
            ranks[r]["rule_map_nnz"] = int(m["nnz"])
            nnz += int(m["nnz"])
        del g, gcnt
        if world == 1:
            ref_gram, ref_nnz = glob, nnz
        gram_ok = bool(torch.equal(glob, ref_gram)) if ref_gram is not None else None
        if world != 1:
            del glob
        torch.cuda.empty_cache()
        for x in ranks:
            x["local_ms"] = round(sum(x["phases_ms"].values()), 3)
        per, _, _ = row_block(F, world, 0)
        sup_b, gram_b = 4 * I, 4 * per * world * F
        frac = (world - 1) / world
        coll = {"supports_allreduce_bytes": sup_b, "gram_reduce_scatter_bytes": gram_b,
                "ms_at_bus_gbps": round((2 * frac * sup_b + frac * gram_b)
                                        / (a.bus_gbps * 1e9) * 1e3, 3)}
        slow = max(x["local_ms"] for x in ranks)
        print(json.dumps({
            "probe": "config5_tx_split", "shape": a.shape, "min_support": a.min_support,
            "world": world, "F": int(F), "gen_s": round(gen_s, 1), "ranks": ranks,
            "slowest_rank_local_ms": slow, "collectives": coll, "bus_gbps_assumed": a.bus_gbps,
            "projected_step_ms": round(slow + coll["ms_at_bus_gbps"], 3),
            "rule_map_nnz": nnz, "rule_map_nnz_equal_1rank": nnz == ref_nnz,
            "gram_equal_1rank": gram_ok}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
