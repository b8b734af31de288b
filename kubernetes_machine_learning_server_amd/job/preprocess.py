"""Job pre-processing: CSV ingest and the artifacts derived from it.

Reference (polars): ``read_tracks``/``clean_df`` (``machine-learning/main.py:148-166``),
``validate_and_map_artists_names_to_ids`` (51-83), ``extract_repeated_track_names`` (86-109),
``map_song_ids_to_song_info`` (112-133), ``get_most_frequent_tracks``/``filter_best_tracks``
(168-184), ``group_tracks_by_playlist_and_generate_homogeneous_data`` (195-207).

Here the CSV is scanned once by the native reader (``csrc/host/csv_encode.cpp``) which
dictionary-encodes every needed column to int32 codes (first-appearance order); every group-by
below is integer numpy work on those codes, and the playlist transactions are built as a CSR
over track-name codes by the native group-by (rows deduplicated — ``TransactionEncoder``
collapses duplicates, main.py:267-268).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..ops import native

COLUMNS = ["pid", "track_uri", "track_name", "artist_name", "artist_uri", "album_name"]
DROP_COLUMNS = ["duration_ms"]


@dataclasses.dataclass
class TracksTable:
    n_rows: int
    width: int
    codes: Dict[str, np.ndarray]
    uniques: Dict[str, List[str]]

    def n_unique(self, col: str) -> int:
        return len(self.uniques[col])

    def head(self, n: int) -> "TracksTable":
        codes = {k: v[:n] for k, v in self.codes.items()}
        uniq = {}
        for k, v in codes.items():  # re-encode so uniques only cover the kept rows
            u, first, inv = np.unique(v, return_index=True, return_inverse=True)
            order = np.argsort(first, kind="stable")
            remap = np.empty(len(u), np.int32)
            remap[order] = np.arange(len(u), dtype=np.int32)
            codes[k] = remap[inv].astype(np.int32)
            uniq[k] = [self.uniques[k][int(u[i])] for i in order]
        return TracksTable(n, self.width, codes, uniq)


def read_tracks(path: str, sample_ratio: float = 1.0, verbose: bool = True) -> TracksTable:
    out = native.load().read_csv_encoded(str(path), COLUMNS)
    cols = out["columns"]
    t = TracksTable(int(out["n_rows"]), len(out["header"]),
                    {k: np.asarray(cols[k][0]) for k in COLUMNS},
                    {k: list(cols[k][1]) for k in COLUMNS})
    if 0 < sample_ratio < 1:
        if verbose:
            print(f"Sample ratio: {sample_ratio}")
        t = t.head(max(1, int(t.n_rows * sample_ratio)))
    if verbose:
        print(f"Rows: {t.n_rows}, Columns: {t.width}")
        print(f"Unique pids: {t.n_unique('pid')}")
        print(f"Unique songs: {t.n_unique('track_uri')}")
    return t


def clean_df(t: TracksTable) -> TracksTable:
    """``df.drop(DROP_COLUMNS)``: the dropped column is never decoded; only the width changes."""
    return dataclasses.replace(t, width=t.width - len(DROP_COLUMNS))


def _unique_pairs(a: np.ndarray, b: np.ndarray, nb: int) -> Tuple[np.ndarray, np.ndarray]:
    """Distinct (a, b) pairs in first-appearance order."""
    key = a.astype(np.int64) * max(nb, 1) + b.astype(np.int64)
    _, first = np.unique(key, return_index=True)
    first.sort()
    return a[first], b[first]


def validate_and_map_artists_names_to_ids(t: TracksTable) -> Dict[str, str]:
    """Raise ``ValueError`` if an artist name maps to >1 artist URI; else {name: uri}."""
    an, au = t.codes["artist_name"], t.codes["artist_uri"]
    pa, pu = _unique_pairs(an, au, t.n_unique("artist_uri"))
    per_name = np.bincount(pa, minlength=t.n_unique("artist_name"))
    dup = np.nonzero(per_name > 1)[0]
    if len(dup) > 0:
        msg = f"Found {len(dup)} duplicate artists"
        print(msg)
        for d in dup[:20]:
            uris = [t.uniques["artist_uri"][u] for u in pu[pa == d]]
            print(f"\t{t.uniques['artist_name'][d]}: {uris}")
        raise ValueError(msg)
    names, uris = t.uniques["artist_name"], t.uniques["artist_uri"]
    return {names[a]: uris[u] for a, u in zip(pa, pu)}


def extract_repeated_track_names(t: TracksTable) -> Dict[str, List[str]]:
    """{track_name: [uris]} for names shared by more than one URI (may be empty)."""
    tn, tu = t.codes["track_name"], t.codes["track_uri"]
    pn, pu = _unique_pairs(tn, tu, t.n_unique("track_uri"))
    per_name = np.bincount(pn, minlength=t.n_unique("track_name"))
    names, uris = t.uniques["track_name"], t.uniques["track_uri"]
    out: Dict[str, List[str]] = {}
    for n, u in zip(pn, pu):
        if per_name[n] > 1:
            out.setdefault(names[n], []).append(uris[u])
    return out


def map_song_ids_to_song_info(t: TracksTable) -> Dict[str, Dict[str, str]]:
    """{track_uri: {track_name, artist_name, album_name}} from each URI's first row (pl.first)."""
    tu = t.codes["track_uri"]
    _, first = np.unique(tu, return_index=True)
    first.sort()
    U, TN, AN, AL = (t.uniques[c] for c in ("track_uri", "track_name", "artist_name", "album_name"))
    ctn, can, cal = t.codes["track_name"], t.codes["artist_name"], t.codes["album_name"]
    return {U[tu[r]]: {"track_name": TN[ctn[r]], "artist_name": AN[can[r]],
                       "album_name": AL[cal[r]]} for r in first}


def get_most_frequent_tracks(t: TracksTable) -> List[Dict]:
    """Rows per track_name, descending (``.sort("count").reverse()``; ties: reverse of first
    appearance, i.e. a stable ascending sort reversed)."""
    cnt = np.bincount(t.codes["track_name"], minlength=t.n_unique("track_name"))
    order = np.argsort(cnt, kind="stable")[::-1]
    names = t.uniques["track_name"]
    return [{"track_name": names[i], "count": int(cnt[i])} for i in order]


def filter_best_tracks(track_infos: List[Dict], percentile: float, verbose: bool = True) -> List[Dict]:
    keep = track_infos[:int(len(track_infos) * percentile)]
    if verbose:
        print("Most frequent songs >")
        print(f"\tKeeping {len(keep)} most frequent tracks out of {len(track_infos)}")
        print("\t3 most frequent tracks are: ", keep[:3])
    return keep


@dataclasses.dataclass
class PlaylistTransactions:
    tx_ptr: np.ndarray     # int64[P+1]
    items: np.ndarray      # int32 track-name codes, rows deduplicated + sorted
    names: List[str]       # code -> track name
    pids: List[str]        # row -> pid

    @property
    def n_tx(self) -> int:
        return len(self.tx_ptr) - 1

    def as_lists(self) -> List[List[str]]:
        return [[self.names[i] for i in self.items[self.tx_ptr[r]:self.tx_ptr[r + 1]]]
                for r in range(self.n_tx)]


GPU_GROUPBY_MIN_ROWS = 4_000_000  # below this the PCIe round trip costs more than the host sort


def group_tracks_by_playlist(t: TracksTable, backend: str = "auto") -> PlaylistTransactions:
    """{pid: [track_name, ...]} as CSR over name codes (the miners' input).

    ``backend``: "cpu" (C++ group-by), "gpu" (HIP radix-sort group-by, kernels/groupby.hip) or
    "auto" (GPU for >= 4M rows when a device is visible; env ``GROUPBY`` overrides)."""
    import os
    backend = os.environ.get("GROUPBY", backend).lower()
    keys, vals = t.codes["pid"], t.codes["track_name"]
    if backend == "auto":
        backend = "gpu" if (len(keys) >= GPU_GROUPBY_MIN_ROWS and native.gpu_available()) else "cpu"
    if backend == "gpu":
        ptr, items = native.require_gpu().group_to_csr_gpu(keys, vals, t.n_unique("pid"), True)
    else:
        ptr, items = native.load().group_to_csr(keys, vals, t.n_unique("pid"), True, True)
    return PlaylistTransactions(np.asarray(ptr), np.asarray(items), t.uniques["track_name"],
                                t.uniques["pid"])


# ---- J16: helpers the reference defines but never calls (kept for API parity) -------------------
def save_most_frequent_tracks_dict(sorted_most_frequent: List[Dict],
                                   best_percentage: float = 0.1) -> List[str]:
    """Names of the first ``int(len * 0.1)`` tracks of a popularity-sorted list
    (``save_most_frequent_tracks_dict``, machine-learning/main.py:186-193; unused there)."""
    k = int(len(sorted_most_frequent) * best_percentage)
    return [t["track_name"] for t in sorted_most_frequent[:k]]


def group_tracks_by_playlist_and_generate_homogeneous_data(t: TracksTable) -> Dict[str, List[str]]:
    """``{pid: [track_name, ...]}`` with duplicates and row order kept, as polars'
    ``group_by(pid).agg(list)`` (main.py:195-207).  The miners use the CSR form instead."""
    pid, name = t.codes["pid"], t.codes["track_name"]
    order = np.argsort(pid, kind="stable")
    bounds = np.flatnonzero(np.diff(pid[order])) + 1
    out: Dict[str, List[str]] = {}
    for grp in np.split(order, bounds):
        if len(grp):
            out[t.uniques["pid"][int(pid[grp[0]])]] = [t.uniques["track_name"][int(c)] for c in name[grp]]
    return out


def group_tracks_by_playlist_and_generate_heterogeneous_data(t: TracksTable):
    """Per-pid tables of the remaining columns (main.py:209-222, unused there; the reference's
    version filters the whole frame once per pid, O(P*N)).  One stable sort here; returns
    ``{pid: pandas.DataFrame}`` without the columns the reference drops
    (track_uri, album_name, artist_uri)."""
    import pandas as pd
    keep = [c for c in t.codes if c not in ("pid", "track_uri", "album_name", "artist_uri")]
    pid = t.codes["pid"]
    order = np.argsort(pid, kind="stable")
    bounds = np.flatnonzero(np.diff(pid[order])) + 1
    out = {}
    for grp in np.split(order, bounds):
        if len(grp):
            out[t.uniques["pid"][int(pid[grp[0]])]] = pd.DataFrame(
                {c: [t.uniques[c][int(x)] for x in t.codes[c][grp]] for c in keep})
    return out
