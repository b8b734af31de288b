"""Probe of the product path of the deep miner (emit -> device trie compaction -> host trie):
phase times at one support, digest against the count-only run.  GPU box only.

    python scripts/deep_trie_probe.py --support 0.02 [--reps 2]
"""
import argparse
import json
import sys
import time

sys.path.insert(0, ".")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--support", type=float, default=0.02)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--digest", action="store_true", help="host trie_digest of the download")
    a = ap.parse_args()
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    N = native.require_gpu()
    tx = generate("ds1", seed=0)
    g = N.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    cnt = g.mine_deep(a.support)
    for rep in range(a.reps):
        t0 = time.perf_counter()
        d = g.mine_deep(a.support, emit=True)
        t1 = time.perf_counter()
        t = g.deep_arena_trie(1, 0)
        t2 = time.perf_counter()
        out = {"rep": rep, "support": a.support, "n_itemsets": d["n_itemsets"], "trie_n": t["n"],
               "emit_ms": round((t1 - t0) * 1e3, 1), "trie_and_download_ms": round((t2 - t1) * 1e3, 1),
               "bytes": int(sum(t[k].nbytes for k in ("parent", "item", "count", "depth"))),
               "digest_equals_count_only": d["digest"] == cnt["digest"]}
        if a.digest and rep == a.reps - 1:
            t3 = time.perf_counter()
            hd = N.trie_digest(t["parent"], t["item"], t["count"], t["depth"])
            out["host_digest_ms"] = round((time.perf_counter() - t3) * 1e3, 1)
            out["host_digest_ok"] = hd["digest"] == cnt["digest"]
        print(json.dumps(out), flush=True)
        del t


if __name__ == "__main__":
    main()
