"""The ML job: one run = pick the next dataset, mine it, publish artifacts.

Reference driver: ``machine-learning/main.py:421-484``.  Same sequence, same artifacts, same
print lines, same exit code; the mining itself runs on the HIP miner (``MINER=gpu``), the
native CPU miner (``cpu``) or the mlxtend-faithful oracle (``oracle``):

  get_dataset_list → get_next_run_index → read_tracks/clean → total_songs →
  artistsMapping.pickle (validate) → trackNameToRepeatedUris.pickle (if any) →
  trackIdsToInfo.pickle → best_tracks.pickle → transactions → [experiment sweep] →
  FP-Growth + rule map → recommendations.pickle (+ rules.idx, frequent_itemsets.npz) →
  dataset_history.csv + last_execution.txt (marker LAST) → exit 0

Multi-GPU: ``torchrun --nproc-per-node N -m kubernetes_machine_learning_server_amd.job`` with
``NUM_GPUS=N`` mines with ``parallel.dist_miner`` (RCCL); rank 0 writes every artifact.
Run: ``python -m kubernetes_machine_learning_server_amd.job``.
"""
from __future__ import annotations

import os
import sys
import time
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..config import JobSettings
from ..models.fpgrowth import ItemsetTrie, default_backend, mine_csr
from ..serve.index import RuleIndexData, build_index_from_trie, index_from_device_csr
from ..utils.atomic_io import atomic_pickle, atomic_write_with
from ..utils.checkpoint import PhaseCheckpoint
from ..utils.timeutil import current_time_str, format_timedelta
from . import preprocess as pp
from . import rotation as rot

PICKLE_ARTISTS_FILE = "artistsMapping.pickle"
PICKLE_TRACK_ID_TO_TRACK_INFO = "trackIdsToInfo.pickle"
PICKLE_DUPLICATED_TRACKS = "trackNameToRepeatedUris.pickle"
RULES_INDEX_FILE = "rules.idx"
ITEMSETS_FILE = "frequent_itemsets.npz"
EXPERIMENT_CSV = "fp_growth_experiment_results.csv"


def save_pickle(cfg: JobSettings, name: str, data) -> None:
    full = cfg.pickles_folder / name
    print("\tSaving pickle to", full)
    atomic_pickle(full, data)


def _fault(point: str) -> None:
    """Fault injection for tests: KMLS_FAULT=<point> raises at that point."""
    if os.environ.get("KMLS_FAULT") == point:
        raise RuntimeError(f"injected fault at {point}")


def mine_rules(cfg: JobSettings, tx: pp.PlaylistTransactions, min_support: float,
               total_songs: int, backend: Optional[str] = None, verbose: bool = True
               ) -> Tuple[RuleIndexData, ItemsetTrie, str, Tuple[int, float]]:
    """``calculate_and_save_fp_growth_fast`` (main.py:262-313): mine + rule map + timing.

    On the GPU the rule map (the ``songs_to_song_sets`` loop, main.py:282-304, = the pair-support
    rows) is built by the device kernel inside the mining call (``pairs_to_csr``) and becomes
    ``rules.idx`` / ``recommendations.pickle`` directly; the CPU and oracle miners build it on the
    host from the trie (same rows, same order)."""
    t0 = time.perf_counter()
    backend = backend or (default_backend() if cfg.miner == "auto" else cfg.miner)
    trie = mine_csr(tx.tx_ptr, tx.items, len(tx.names), min_support, backend=backend,
                    pairs_only=(cfg.rules_mode == "pairs"), columns=tx.names,
                    rule_index=(backend == "gpu"))
    dev_map = trie.stats.pop("device_rule_map", None) if isinstance(trie.stats, dict) else None
    if dev_map is not None:
        idx = index_from_device_csr(dev_map, len(tx.names), trie.item[trie.depth == 1], tx.n_tx,
                                    tx.names)
        trie.stats["rule_map"] = "device"
    else:
        idx = build_index_from_trie(trie.parent, trie.item, trie.count, trie.depth, tx.n_tx,
                                    len(tx.names), tx.names)
    missing = total_songs - idx.n_keys
    dur = time.perf_counter() - t0
    if verbose:
        print("Songs without recommendations:", missing)
        print(f"Time elapsed in rule generation: {format_timedelta(dur)}")
    info = f"min_support: {min_support} \tmissing songs: {missing} \ttime: {format_timedelta(dur)}"
    return idx, trie, info, (missing, dur)


def mine_pairs_distributed(cfg: JobSettings, tx: pp.PlaylistTransactions, min_support: float,
                           total_songs: int
                           ) -> Optional[Tuple[RuleIndexData, ItemsetTrie, str, Tuple[int, float]]]:
    """RULES_MODE=pairs on several GPUs: the rule map is the pair-support matrix, so
    the job forms it with one of the ``parallel.pairs`` strategies over transaction shards
    (reduce-scatter by default; ring = the context-parallel analog, alltoall = Ulysses) — each
    rank ends with the complete rows of its item block — and gathers only the frequent pairs of
    its rows to rank 0, which builds the same index and 2-itemset trie as a single process."""
    import torch.distributed as dist
    from ..parallel.dist_miner import DistMiner, gather_arrays
    from ..serve.index import build_index_from_pairs
    t0 = time.perf_counter()
    rank, world = dist.get_rank(), dist.get_world_size()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dm = DistMiner(tx.tx_ptr, tx.items, len(tx.names), min_support, device=local, max_len=2,
                   backend="cpu" if cfg.miner == "cpu" else "gpu", mode="item")
    ids, r0, r1, rows = dm.pair_rows(cfg.pairs_strategy)
    fcounts, minsup = np.asarray(dm.ops.sel[1]), int(dm.ops.sel[2])
    rows = np.asarray(rows, np.int64)[: r1 - r0]
    upper = np.arange(rows.shape[1])[None, :] > np.arange(r0, r1)[:, None]  # each pair once
    ii, jj = np.nonzero((rows >= minsup) & upper)
    pa, pb = (ii + r0).astype(np.int64), jj.astype(np.int64)  # ranks, a < b
    pc = rows[ii, jj].astype(np.int64)
    got = gather_arrays({"a": pa, "b": pb, "c": pc}, rank, world)
    if rank != 0:
        return None
    ids = np.asarray(ids, np.int64)
    F = len(ids)
    pa, pb, pc = got["a"], got["b"], got["c"]
    order = np.lexsort((pb, pa))  # trie: level-2 nodes grouped by parent rank
    pa, pb, pc = pa[order], pb[order], pc[order]
    trie = ItemsetTrie(np.concatenate([np.full(F, -1, np.int64), pa]),
                       np.concatenate([ids, ids[pb]]).astype(np.int32),
                       np.concatenate([fcounts.astype(np.int64), pc]).astype(np.uint32),
                       np.concatenate([np.ones(F, np.uint8), np.full(len(pa), 2, np.uint8)]),
                       tx.n_tx, min_support,
                       {"n_frequent_items": F, "backend": f"pairs-{cfg.pairs_strategy}-x{world}"},
                       tx.names)
    idx = build_index_from_pairs(len(tx.names), ids, ids[pa], ids[pb], pc, tx.n_tx, tx.names)
    missing = total_songs - idx.n_keys
    dur = time.perf_counter() - t0
    print("Songs without recommendations:", missing)
    print(f"Time elapsed in rule generation: {format_timedelta(dur)}")
    info = f"min_support: {min_support} \tmissing songs: {missing} \ttime: {format_timedelta(dur)}"
    return idx, trie, info, (missing, dur)


def mine_rules_distributed(cfg: JobSettings, tx: pp.PlaylistTransactions, min_support: float,
                           total_songs: int, ck: Optional[PhaseCheckpoint] = None
                           ) -> Optional[Tuple[RuleIndexData, ItemsetTrie, str, Tuple[int, float]]]:
    """Multi-GPU mining (torchrun); returns the result on rank 0, None elsewhere.

    Phase checkpoints: after mining, every rank saves its own sub-trie (tx mode:
    rank 0 saves the global trie, which every rank holds) under the run's checkpoint key (dataset,
    min_support, rules mode, sample ratio: the frequent order is a pure function of these).  A
    restarted job whose ranks ALL find their phase output (tx mode: rank 0's) skips mining and
    goes straight to the merge; a partial set is ignored (every rank re-mines)."""
    import torch
    import torch.distributed as dist
    from ..parallel.dist_miner import DistMiner, gather_trie
    t0 = time.perf_counter()
    rank, world = dist.get_rank(), dist.get_world_size()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if use_deep_split(cfg, tx.n_tx):
        return mine_rules_deep_split(cfg, tx, min_support, total_songs, rank, world, local, t0,
                                     ck)
    dm = DistMiner(tx.tx_ptr, tx.items, len(tx.names), min_support, device=local,
                   max_len=2 if cfg.rules_mode == "pairs" else 0,
                   backend="cpu" if cfg.miner == "cpu" else "gpu", mode=cfg.dist_mode)
    phase = f"subtrie_r{rank}of{world}_{dm.mode}"
    tx_follower = dm.mode == "tx" and rank != 0  # needs nothing: rank 0 holds the global trie
    have = 1 if (tx_follower or (ck is not None and ck.has(phase))) else 0
    flag = torch.tensor([have], dtype=torch.int64,
                        device=torch.device("cuda", local) if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 1:  # every rank has its phase output: no re-mining
        sub, st = None, {"backend": "checkpoint"}
        if not tx_follower:
            z = ck.load(phase)
            sub = {k: z[k] for k in ("parent", "item", "count", "depth")}
            st["n_frequent_items"] = int(z["n_frequent"])
        if rank == 0:
            print("Resumed per-rank sub-tries from checkpoint", ck.dir)
    else:
        r = dm.step(download=True)
        sub = {k: np.asarray(v) for k, v in r["trie"].items() if k in ("parent", "item", "count", "depth")}
        st = dict(r["stats"])
        if ck is not None and ck.enabled and (dm.mode != "tx" or rank == 0):
            ck.save(phase, n_frequent=np.int64(st.get("n_frequent_items", 0)), **sub)
        _fault("after_mining_phase")
    F = int(st.get("n_frequent_items", 0))
    if dm.mode == "tx":  # every rank holds the identical global trie; rank 0 downloaded it
        merged = sub if rank == 0 else None
    else:
        merged = gather_trie(sub, rank, world, F)
    del dm  # its device buffers go before the rule map's
    # the deployed artifact (rules.idx / recommendations.pickle = the pair-support rows,
    # main.py:282-304) through the distributed rule map: every rank counts its transaction
    # shard's pairs, row blocks are reduce-scattered, each rank builds the CSR of its rows
    rmap = rule_map_distributed(cfg, tx, min_support, rank, world, local)
    if rank != 0:
        return None
    trie = ItemsetTrie(merged["parent"], merged["item"], merged["count"], merged["depth"],
                       tx.n_tx, min_support, st, tx.names)
    idx = index_from_device_csr(rmap, len(tx.names), rmap["ids"], tx.n_tx, tx.names)
    trie.stats["rule_map"] = f"distributed-x{world}({rmap.get('level2_method', 'gram')})"
    missing = total_songs - idx.n_keys
    dur = time.perf_counter() - t0
    print("Songs without recommendations:", missing)
    print(f"Time elapsed in rule generation: {format_timedelta(dur)}")
    info = f"min_support: {min_support} \tmissing songs: {missing} \ttime: {format_timedelta(dur)}"
    return idx, trie, info, (missing, dur)


def use_deep_split(cfg: JobSettings, n_tx: int) -> bool:
    """The multi-GPU job mines with the headline's deep DFS split (``DeepMiner.mine_trie``) when
    it mines every itemset on GPUs and the dataset fits the deep miner's tid rows."""
    from ..models.fpgrowth import full_miner
    if cfg.miner == "cpu" or cfg.rules_mode != "full" or cfg.dist_mode not in ("auto", "deep"):
        return False
    ok = full_miner(n_tx) == "deep"
    if cfg.dist_mode == "deep" and not ok:
        raise ValueError(f"KMLS_DIST_MODE=deep needs <= 4096 transactions (got {n_tx})")
    return ok


def mine_rules_deep_split(cfg: JobSettings, tx: pp.PlaylistTransactions, min_support: float,
                          total_songs: int, rank: int, world: int, local: int, t0: float,
                          ck: Optional[PhaseCheckpoint] = None):
    """Full mining split over the ranks (the headline engine, ``parallel/deep.py``): level-3
    tasks dealt by measured cost, every rank's itemsets emitted into its HBM arena, compacted on
    its GPU and gathered on rank 0 as one trie; the rule map through ``DistRuleMap``.

    Phase checkpoint: rank 0 (the only holder of the gathered trie) saves it; a restarted job
    whose rank 0 finds it skips the mining on every rank (the vote is all-reduced, so all ranks
    take the same branch and the rule map's collectives still line up)."""
    import torch
    import torch.distributed as dist
    from ..parallel.deep import DeepMiner
    phase = f"deeptrie_x{world}"
    have = 1 if (rank != 0 or (ck is not None and ck.has(phase))) else 0
    flag = torch.tensor([have], dtype=torch.int64,
                        device=torch.device("cuda", local) if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    keys = ("parent", "item", "count", "depth")
    if int(flag.item()) == 1:
        arrs, st = None, {"backend": "checkpoint", "miner": "deep", "dist_mode": f"deep-x{world}"}
        if rank == 0:
            z = ck.load(phase)
            arrs = {k: z[k] for k in keys}
            st.update(n_frequent_items=int(z["n_frequent"]), n_itemsets=int(z["n_itemsets"]),
                      digest=str(z["digest"]))
            print("Resumed the gathered deep trie from checkpoint", ck.dir)
    else:
        dm = DeepMiner(tx.tx_ptr, tx.items, len(tx.names), device=local, rank=rank, world=world)
        d, arrs = dm.mine_trie(min_support)
        st = {"n_frequent_items": int(d["n_frequent_items"]), "n_itemsets": int(d["n_itemsets"]),
              "digest": d["digest"], "miner": "deep", "dist_mode": f"deep-x{world}",
              "backend": "gpu"}
        del dm  # its device buffers go before the rule map's
        if rank == 0 and ck is not None and ck.enabled:
            ck.save(phase, n_frequent=np.int64(st["n_frequent_items"]),
                    n_itemsets=np.int64(st["n_itemsets"]), digest=np.array(st["digest"]),
                    **{k: np.asarray(arrs[k]) for k in keys})
    _fault("after_mining_phase")
    rmap = rule_map_distributed(cfg, tx, min_support, rank, world, local)
    if rank != 0:
        return None
    trie = ItemsetTrie(arrs["parent"], arrs["item"], arrs["count"], arrs["depth"], tx.n_tx,
                       min_support, st, tx.names)
    idx = index_from_device_csr(rmap, len(tx.names), rmap["ids"], tx.n_tx, tx.names)
    trie.stats["rule_map"] = f"distributed-x{world}({rmap.get('level2_method', 'gram')})"
    missing = total_songs - idx.n_keys
    dur = time.perf_counter() - t0
    print("Songs without recommendations:", missing)
    print(f"Time elapsed in rule generation: {format_timedelta(dur)}")
    info = f"min_support: {min_support} \tmissing songs: {missing} \ttime: {format_timedelta(dur)}"
    return idx, trie, info, (missing, dur)


def rule_map_distributed(cfg: JobSettings, tx: pp.PlaylistTransactions, min_support: float,
                         rank: int, world: int, local: int) -> Optional[Dict]:
    """``parallel.rule_map.DistRuleMap`` over this rank's transaction shard (every rank holds
    the whole dataset; the shards are the same contiguous ranges the tx-DP miner uses).  The
    item-id CSR comes back on rank 0 (None elsewhere), rows ordered count desc, name asc: the
    same bytes as the single-process index."""
    from ..parallel.dist_miner import shard_bounds
    from ..parallel.rule_map import DistRuleMap
    from ..serve.index import name_tie_rank
    lo, hi, _ = shard_bounds(tx.n_tx, world, rank)
    ptr = np.asarray(tx.tx_ptr[lo:hi + 1], np.int64)
    its = np.ascontiguousarray(tx.items[int(ptr[0]):int(ptr[-1])], np.int32)
    rm = DistRuleMap(ptr - ptr[0], its, len(tx.names), tx.n_tx, min_support, device=local,
                     backend="cpu" if cfg.miner == "cpu" else "gpu")
    try:
        rm.set_tie_rank(name_tie_rank([str(n) for n in tx.names]))
        return rm.step()
    finally:
        rm.release()


def resume_from_checkpoint(ck: PhaseCheckpoint, tx: pp.PlaylistTransactions, min_support: float,
                           total_songs: int) -> Tuple[RuleIndexData, ItemsetTrie, str, Tuple[int, float]]:
    z = ck.load("trie")
    trie = ItemsetTrie(z["parent"], z["item"], z["count"], z["depth"], int(z["n_tx"]), min_support,
                       {"backend": "checkpoint"}, tx.names)
    idx = build_index_from_trie(trie.parent, trie.item, trie.count, trie.depth, tx.n_tx,
                                len(tx.names), tx.names)
    missing = total_songs - idx.n_keys
    dur = float(z["seconds"])
    print("Songs without recommendations:", missing)
    print(f"Time elapsed in rule generation: {format_timedelta(dur)}")
    info = f"min_support: {min_support} \tmissing songs: {missing} \ttime: {format_timedelta(dur)}"
    return idx, trie, info, (missing, dur)


def run_support_sweep(cfg: JobSettings, tx: pp.PlaylistTransactions, total_songs: int,
                      supports: Optional[List[float]] = None, out_csv: str = EXPERIMENT_CSV,
                      group=None):
    """J14: the min_support sweep (main.py:450-473), written to ``fp_growth_experiment_results.csv``.

    Multi-GPU (``group`` = the job's gloo side group): the sweep points are dealt over the ranks
    in snake order (low supports cost the most) and every rank mines its points on its own GPU
    with no collective (dataset-parallel, like ``DistMiner(mode="local")``); one gather over the
    side group brings the rows to rank 0, which writes them in grid order."""
    import pandas as pd
    supports = supports if supports is not None else np.arange(0.03, 0.2, 0.0025).tolist()
    world, rank = 1, 0
    if group is not None:
        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)
    mine_idx = [i for i in range(len(supports))
                if ((i // world) % 2 == 0 and i % world == rank) or
                   ((i // world) % 2 == 1 and world - 1 - i % world == rank)]
    rows = []
    for i in mine_idx:
        ms = round(supports[i], 3)
        if rank == 0:
            print(f"Calculating for min_support: {ms}")
        _, trie, _, (missing, dur) = mine_rules(cfg, tx, ms, total_songs, verbose=rank == 0)
        rows.append((i, {"min_support": ms, "songs_without_recommendations": missing,
                         "duration": dur, "n_itemsets": len(trie)}))
        if world == 1:
            pd.DataFrame([r for _, r in rows]).to_csv(out_csv, index=False)
    if world > 1:
        import torch.distributed as dist
        parts = [None] * world
        dist.all_gather_object(parts, rows, group=group)
        rows = sorted((r for part in parts for r in part), key=lambda x: x[0])
        if rank == 0:
            pd.DataFrame([r for _, r in rows]).to_csv(out_csv, index=False)
    return [r for _, r in rows]


def save_itemsets(cfg: JobSettings, trie: ItemsetTrie) -> None:
    """``frequent_itemsets.npz``: the trie arrays as mined (narrow widths kept: 9 B per itemset
    from the GPU miners), streamed into the temp file of the atomic write — at ds1 @0.02 that
    is 1.4e9 itemsets, so no in-memory copy of the archive is made."""
    def write(f):
        np.savez(f, parent=trie.parent, item=trie.item, count=trie.count, depth=trie.depth,
                 n_tx=np.int64(trie.n_tx), min_support=np.float64(trie.min_support))
    atomic_write_with(cfg.pickles_folder / ITEMSETS_FILE, write)


def run(cfg: Optional[JobSettings] = None) -> Dict:
    cfg = cfg or JobSettings.from_env()
    distributed = cfg.num_gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) > 1
    rank = 0
    side = None  # gloo group for long host-side waits (the sweep), off the RCCL watchdog
    if distributed:
        import datetime
        import torch
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # bounded rendezvous and collectives: a rank that never joins or dies
        # fails the job within KMLS_DIST_TIMEOUT_S instead of hanging it; K8s then re-runs it.
        # MINER=cpu runs the same protocol over gloo (the CPU test tier)
        timeout = datetime.timedelta(seconds=cfg.dist_timeout_s)
        # KMLS_DIST_BACKEND=gloo: GPU miners under a gloo group (tests: ranks sharing one GPU,
        # with KMLS_COMM=host for the native collectives; RCCL refuses two ranks on one device)
        if cfg.miner == "cpu" or os.environ.get("KMLS_DIST_BACKEND") == "gloo":
            dist.init_process_group("gloo", timeout=timeout)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
        rank = dist.get_rank()
        if cfg.experiment_supports:
            side = dist.new_group(backend="gloo",
                                  timeout=datetime.timedelta(seconds=cfg.sweep_timeout_s))
    say = print if rank == 0 else (lambda *a, **k: None)
    say("=== Starting execution on ", current_time_str(), " ===")
    datasets = rot.get_dataset_list(cfg) if rank == 0 else None
    if distributed:
        import torch.distributed as dist
        box = [datasets]
        dist.broadcast_object_list(box, src=0)
        datasets = box[0]
    new_index = rot.get_next_run_index(cfg, datasets)
    selected = datasets[new_index - 1]
    say(f"Selected dataset: {selected}")
    t = pp.clean_df(pp.read_tracks(selected, cfg.sample_ratio, verbose=rank == 0))
    total_songs = t.n_unique("track_uri")
    if rank == 0:
        save_pickle(cfg, PICKLE_ARTISTS_FILE, pp.validate_and_map_artists_names_to_ids(t))
        dups = pp.extract_repeated_track_names(t)
        if dups:
            print(f"\tFound {len(dups)} duplicate songs, saving to {PICKLE_DUPLICATED_TRACKS}")
            save_pickle(cfg, PICKLE_DUPLICATED_TRACKS, dups)
        save_pickle(cfg, PICKLE_TRACK_ID_TO_TRACK_INFO, pp.map_song_ids_to_song_info(t))
        best = pp.filter_best_tracks(pp.get_most_frequent_tracks(t), cfg.top_tracks_save_percentile)
        save_pickle(cfg, cfg.best_tracks_file, best)
    else:
        pp.validate_and_map_artists_names_to_ids(t)  # every rank fails the same way
    _fault("after_best_tracks")
    tx = pp.group_tracks_by_playlist(t)
    if cfg.experiment_supports:  # every rank mines its share; the gather runs on gloo
        if distributed and cfg.miner != "cpu":
            os.environ.setdefault("KMLS_DEVICE", os.environ.get("LOCAL_RANK", "0"))
        run_support_sweep(cfg, tx, total_songs, group=side)
    ck = PhaseCheckpoint.for_dataset(cfg.checkpoint_dir, selected, min_support=cfg.min_support,
                                     rules_mode=cfg.rules_mode, sample_ratio=cfg.sample_ratio)
    resumed = ck.has("trie") if rank == 0 else False
    if distributed:
        import torch.distributed as dist
        box = [resumed]
        dist.broadcast_object_list(box, src=0)
        resumed = box[0]
    if resumed:  # a previous attempt on this dataset crashed after mining
        res = resume_from_checkpoint(ck, tx, cfg.min_support, total_songs) if rank == 0 else None
        say("Resumed mining results from checkpoint", ck.dir)
    elif distributed and cfg.rules_mode == "pairs" and cfg.pairs_strategy != "trie":
        res = mine_pairs_distributed(cfg, tx, cfg.min_support, total_songs)
    elif distributed:
        res = mine_rules_distributed(cfg, tx, cfg.min_support, total_songs, ck)
    else:
        res = mine_rules(cfg, tx, cfg.min_support, total_songs)
    if rank == 0 and not resumed and ck.enabled:
        trie = res[1]
        ck.save("trie", parent=trie.parent, item=trie.item, count=trie.count, depth=trie.depth,
                n_tx=np.int64(trie.n_tx), seconds=np.float64(res[3][1]))
    summary: Dict = {}
    if rank == 0:
        idx, trie, info, (missing, dur) = res
        _fault("before_recommendations")
        save_pickle(cfg, cfg.recommendations_file, idx.to_rec_dict())
        idx.save(cfg.pickles_folder / RULES_INDEX_FILE)
        if cfg.rules_mode == "full":
            save_itemsets(cfg, trie)
        _fault("before_marker")
        ts = rot.append_dataset_history(cfg, new_index, selected)
        ck.clear()  # the run is complete: nothing to resume
        summary = {"dataset_index": new_index, "dataset": selected, "marker": ts,
                   "n_keys": idx.n_keys, "songs_without_recommendations": missing,
                   "n_itemsets": len(trie), "rule_seconds": dur, "backend": trie.stats.get("backend"),
                   "rule_map": trie.stats.get("rule_map", "host"), "resumed": resumed}
        print("=== Run complete. Exiting, current time is ", current_time_str(), " ===")
    if distributed:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    return summary


def main() -> int:
    run()
    return 0


if __name__ == "__main__":
    sys.exit(main())
