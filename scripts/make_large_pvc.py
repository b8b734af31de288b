#!/usr/bin/env python3
"""A serving PVC holding the BASELINE config-5 artifact: the rule map of 100M synthetic
transactions x 1M items at min_support 2e-4 (14.8k keys, rows of up to thousands of entries),
built on the GPU by ``parallel.rule_map.DistRuleMap`` (world 1), plus a second index of the same
data at another support for hot-reload tests (``<out>/rules_alt.idx``).

  python scripts/make_large_pvc.py --out /tmp/pvc_c5 [--shape 100Mx1M --min-support 2e-4
                                                     --alt-support 3e-4]

Layout: <out>/api-data/{pickles/rules.idx, pickles/best_tracks.pickle, last_execution.txt}
(the files the server reads; recommendations.pickle is not needed when rules.idx exists).
Item names are "track_<id>" (random-init vocabulary).
"""
import argparse
import json
import os
import pathlib
import pickle
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--shape", default="100Mx1M")
    ap.add_argument("--min-support", type=float, default=2e-4)
    ap.add_argument("--alt-support", type=float, default=3e-4)
    ap.add_argument("--top", type=float, default=0.03, help="best-tracks fraction of the keys")
    ap.add_argument("--n-tx", type=int, default=0, help="override the shape's transactions")
    ap.add_argument("--backend", default="gpu", choices=("gpu", "cpu"))
    a = ap.parse_args()
    import numpy as np
    from kubernetes_machine_learning_server_amd.data.synthetic import SHAPES
    from kubernetes_machine_learning_server_amd.ops import native
    from kubernetes_machine_learning_server_amd.parallel.rule_map import DistRuleMap
    from kubernetes_machine_learning_server_amd.serve.index import (index_from_device_csr,
                                                                     name_tie_rank)
    N = native.require_gpu() if a.backend == "gpu" else native.load()
    s = SHAPES[a.shape]
    T, I = a.n_tx or s.n_tx, s.n_items
    t0 = time.time()
    ptr, items = N.synth_transactions(T, I, s.mean_len, s.n_genres, s.genre_affinity, 0.85, 0, 0,
                                      0, T)
    gen_s = time.time() - t0
    names = [f"track_{i}" for i in range(I)]
    tie = name_tie_rank(names)
    base = pathlib.Path(a.out) / "api-data"
    pk = base / "pickles"
    pk.mkdir(parents=True, exist_ok=True)
    info = {"shape": a.shape, "n_tx": T, "n_items": I, "gen_s": round(gen_s, 1)}
    for tag, ms, path in (("main", a.min_support, pk / "rules.idx"),
                          ("alt", a.alt_support, pathlib.Path(a.out) / "rules_alt.idx")):
        rm = DistRuleMap(ptr, items, I, T, ms, device=0, backend=a.backend)
        rm.set_tie_rank(tie)
        t1 = time.time()
        r = rm.step()
        step_s = time.time() - t1
        ids = np.asarray(r["ids"])
        ix = index_from_device_csr(r, I, ids, T, names)
        ix.save(path)
        info[tag] = {"min_support": ms, "keys": int(ix.n_keys), "entries": int(r["nnz"]),
                     "max_row": int(np.diff(np.asarray(r["row_ptr"])).max()),
                     "index_bytes": path.stat().st_size, "rule_map_s": round(step_s, 3),
                     "level2_method": r.get("level2_method")}
        if tag == "main":
            fc = np.asarray(r["fcounts"])
            order = np.argsort(-fc, kind="stable")[:max(10, int(len(ids) * a.top))]
            best = [{"track_name": names[int(ids[o])], "count": int(fc[o])} for o in order]
            with open(pk / "best_tracks.pickle", "wb") as f:
                pickle.dump(best, f)
        rm.release()
        del rm
    (base / "last_execution.txt").write_text("initial")
    print(json.dumps({"pvc": str(base), **info}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
