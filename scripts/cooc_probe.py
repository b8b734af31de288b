#!/usr/bin/env python3
"""Level-2 method probe at the large BASELINE shapes: the horizontal co-occurrence count
(cooc.hip) against the MFMA bit-GEMM on the same shard, and the config-3 mining step with each.

  python scripts/cooc_probe.py --shape 10Mx1M --min-support 2e-4 --reps 3 [--step]

One JSON line per measurement on stdout.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="10Mx1M")
    ap.add_argument("--min-support", type=float, default=2e-4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--step", action="store_true", help="also time mine_txdp with each method")
    ap.add_argument("--no-gemm", action="store_true", help="skip the bit-GEMM side")
    a = ap.parse_args()
    import numpy as np
    import torch
    from kubernetes_machine_learning_server_amd.data.synthetic import SHAPES
    from kubernetes_machine_learning_server_amd.ops import native
    N = native.require_gpu()
    s = SHAPES[a.shape]
    t = time.time()
    ptr, items = N.synth_transactions(s.n_tx, s.n_items, s.mean_len, s.n_genres, s.genre_affinity,
                                      0.85, 0, 0, 0, s.n_tx)
    print(f"[cooc_probe] generated {s.n_tx} tx in {time.time() - t:.1f} s", file=sys.stderr,
          flush=True)
    ts = torch.cuda.Stream()
    torch.cuda.set_stream(ts)  # torch fills and the miner share one stream
    g = N.GpuMiner(0, 48 << 30, ts.cuda_stream)
    g.load_csr(ptr, items, s.n_items)
    cnt = torch.zeros(s.n_items, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    g.item_support(cnt.data_ptr())
    g.synchronize()
    counts = cnt.cpu().numpy().view(np.uint32).copy()
    F = g.select(counts, s.n_tx, a.min_support)
    st = g.cooc_stats()
    gram = torch.empty((F, F), dtype=torch.int32, device="cuda")

    def timed(fn):
        best = 1e30
        for _ in range(a.reps):
            g.synchronize()
            t = time.perf_counter()
            fn()
            g.synchronize()
            best = min(best, (time.perf_counter() - t) * 1e3)
        return best

    ok = [True]
    ms_cooc = timed(lambda: ok.__setitem__(0, g.pair_counts_csr(gram.data_ptr(), F)))
    iu = None
    got = gram.cpu().numpy()
    out = {"probe": "cooc", "shape": a.shape, "min_support": a.min_support, "F": F,
           "pairs": st["pairs"], "max_k": st["max_k"], "ok": ok[0], "cooc_ms": round(ms_cooc, 3),
           "pairs_per_s": round(st["pairs"] / (ms_cooc / 1e3), 1),
           "frequent_pairs": int((np.triu(got, 1) >= g.frequent()[2]).sum())}
    if not a.no_gemm:
        Wp = g.words_local()
        bm = torch.empty((F, Wp), dtype=torch.int64, device="cuda")
        if Wp * 64 > s.n_tx:
            bm[:, (s.n_tx + 63) // 64:] = 0
        torch.cuda.synchronize()
        ms_enc = timed(lambda: g.encode_bitmaps(bm.data_ptr(), Wp, 0))
        ref = torch.empty((F, F), dtype=torch.int32, device="cuda")
        ms_gemm = timed(lambda: g.pair_counts(bm.data_ptr(), Wp, ref.data_ptr(), True))
        iu = np.triu_indices(F, 1)
        out.update(encode_ms=round(ms_enc, 3), gemm_ms=round(ms_gemm, 3),
                   equal_to_gemm=bool((ref.cpu().numpy()[iu] == got[iu]).all()))
        del bm, ref
    print(json.dumps(out), flush=True)
    del gram
    if a.step:
        for hook in ("cooc=2", "cooc=0"):
            os.environ["KMLS_TEST_HOOKS"] = hook
            best, r = 1e30, None
            for _ in range(a.reps + 1):
                t = time.perf_counter()
                r = g.mine_txdp(None, s.n_tx, a.min_support)
                best = min(best, (time.perf_counter() - t) * 1e3)
            d = N.trie_digest(r["parent"], r["item"], r["count"], r["depth"])
            print(json.dumps({"probe": "txdp_step", "hook": hook, "ms": round(best, 3),
                              "level2_method": r["stats"]["level2_method"],
                              "n_itemsets": r["stats"]["n_itemsets"], "digest": d["digest"],
                              "phases_ms": r["stats"].get("phases_ms")}), flush=True)
        os.environ.pop("KMLS_TEST_HOOKS", None)
    return 0


if __name__ == "__main__":
    sys.exit(main())
