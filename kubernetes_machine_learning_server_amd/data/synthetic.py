"""Synthetic playlist data of the reference's named shapes (ds1/ds2 are missing blobs).

The reference reads ``2023_spotify_ds*.csv`` (8 columns, ``machine-learning/main.py:38,153``);
those files are not in the mounted repo (``.MISSING_LARGE_BLOBS``), so every benchmark and test
here runs on synthetic data of the published ds2 shape (``relatorio.pdf`` p.5-6):

* 2,246 playlists, 2,171 unique track URIs, 48 track names shared by >1 URI, 240,249 rows;
* item popularity calibrated to the published "songs without recommendations vs min_support"
  curve (keys = items with support >= ms: ~1571 @0.03, 755 @0.05, 121 @0.10, 11 @0.198);
* co-occurrence structure: playlists draw most tracks from one or two "genre" clusters, which
  is what makes deep frequent itemsets appear (real playlists are strongly clustered).

Two output forms: CSR transactions (``tx_ptr``, ``items``) for the miners/bench, and a
reference-schema CSV for the job pipeline.  Everything is seeded and deterministic.
"""
from __future__ import annotations

import csv
import dataclasses
import io
import pathlib
from typing import Dict, List, Optional, Tuple

import numpy as np

# published ds2 survival curve of per-item playlist counts, as (support, #items >= support)
# read off relatorio.pdf p.5 (songs w/o recommendations = 2171 - keys)
_DS2_CURVE = [
    (0.0085, 2171), (0.0150, 2050), (0.0200, 1900), (0.03, 1571), (0.04, 1071), (0.05, 755),
    (0.06, 541), (0.07, 371), (0.08, 261), (0.10, 121), (0.13, 51), (0.16, 26), (0.198, 11),
    (0.26, 3), (0.32, 1),
]


@dataclasses.dataclass(frozen=True)
class Shape:
    name: str
    n_tx: int
    n_items: int
    mean_len: float
    n_genres: int
    genre_affinity: float  # probability that a track is drawn from the playlist's genres
    dup_names: int = 48     # names shared by 2 URIs (ds2: 48)
    dup_rows: float = 0.01  # fraction of extra duplicate rows inside a playlist (collapsed by encoder)
    p_two_genres: float = 0.35  # probability that a playlist mixes two genres
    len_sigma: float = 0.6      # log-normal sigma of playlist lengths
    calib_v2: bool = False  # deterministic curve quantiles + tail-only length rescale


SHAPES: Dict[str, Shape] = {
    # published ds2 shape (relatorio.pdf p.6); ds1 is assumed to be the same size (753 vs 755
    # keys).  Calibrated by bench/calibrate.py (profiles/r2_calibration.md) against all three
    # constraints the reference documents: the p.5 key curve, the sweep being minable from
    # min_support 0.03 (9.4M itemsets there; <= 1e7) and the published 20.31 s at 0.05, which
    # the replayed reference timed region approaches as closely as constraint 2 allows
    # (78k itemsets, depth 10 at 0.05).
    "ds2": Shape("ds2", 2246, 2171, 240249 / 2246 / 1.01, 6, 0.97, calib_v2=True),
    "ds1": Shape("ds1", 2246, 2171, 240249 / 2246 / 1.01, 6, 0.97, calib_v2=True),
    # round-1 headline shape, kept as a dense stress test: 12 genres at affinity 0.97 give
    # 1.16M itemsets (depth 14) at 0.05 but 40M at 0.04 -- too clustered for the reference's
    # own 0.03 sweep to have been minable, so it is not a fair stand-in for ds1/ds2
    "ds_dense": Shape("ds_dense", 2246, 2171, 240249 / 2246 / 1.01, 12, 0.97),
    # weakly clustered variant (same support curve, 2k itemsets @0.05)
    "ds2_weak": Shape("ds2_weak", 2246, 2171, 240249 / 2246 / 1.01, 24, 0.80),
    # SURVEY §6.3 sanity shape (milder clustering)
    "ds2_mild": Shape("ds2_mild", 2246, 2171, 107.0, 12, 0.55),
    # plumbing config 1 of BASELINE.json: 1k transactions x 100 items
    "tiny": Shape("tiny", 1000, 100, 12.0, 6, 0.7, dup_names=2),
    # config 3 / 5 shapes (generated directly as CSR, never as CSV)
    "10Mx1M": Shape("10Mx1M", 10_000_000, 1_000_000, 40.0, 2000, 0.85, dup_names=0, dup_rows=0.0),
    # BASELINE config 5: 100M transactions sized for one GPU's 288 GB HBM
    "100Mx1M": Shape("100Mx1M", 100_000_000, 1_000_000, 40.0, 2000, 0.85, dup_names=0, dup_rows=0.0),
}


def _target_counts(shape: Shape, rng: np.random.Generator) -> np.ndarray:
    """Per-item target playlist counts, sampled from the published survival curve."""
    sup = np.array([s for s, _ in _DS2_CURVE])
    frac = np.array([n for _, n in _DS2_CURVE], dtype=np.float64) / 2171.0
    if shape.calib_v2:  # evenly spaced survival quantiles: no sampling noise on the key curve
        u = (np.arange(shape.n_items, 0, -1) - 0.5) / shape.n_items
    else:
        u = np.sort(rng.random(shape.n_items))[::-1]  # survival quantiles
    # interpolate log(support) against log(survival)
    ls = np.interp(np.log(u), np.log(frac[::-1]), np.log(sup[::-1]))
    counts = np.exp(ls) * shape.n_tx
    # match the mean playlist length; calib_v2 puts the whole correction on the
    # items below the lowest published key threshold (0.03), so the key curve itself is kept
    total = shape.mean_len * shape.n_tx
    if shape.calib_v2:
        lo = counts < 0.028 * shape.n_tx
        hi_sum = counts[~lo].sum()
        scale = max(total - hi_sum, 0.0) / max(counts[lo].sum(), 1e-9)
        counts[lo] = np.minimum(counts[lo] * scale, 0.028 * shape.n_tx)
    else:
        counts *= total / counts.sum()
    return np.maximum(counts, 1.0)


@dataclasses.dataclass
class Transactions:
    """CSR transactions over integer item ids (rows deduplicated, ascending)."""
    tx_ptr: np.ndarray  # int64[T+1]
    items: np.ndarray   # int32[nnz]
    n_items: int
    names: Optional[List[str]] = None  # item id -> track name (may repeat for duplicate names)

    @property
    def n_tx(self) -> int:
        return len(self.tx_ptr) - 1

    def rows(self):
        for t in range(self.n_tx):
            yield self.items[self.tx_ptr[t]:self.tx_ptr[t + 1]]

    def to_lists(self, use_names: bool = False) -> List[List]:
        out = []
        for r in self.rows():
            out.append([self.names[i] for i in r] if use_names and self.names else r.tolist())
        return out

    def onehot(self) -> np.ndarray:
        X = np.zeros((self.n_tx, self.n_items), dtype=bool)
        for t, r in enumerate(self.rows()):
            X[t, r] = True
        return X


def relabel(tx: Transactions, key: int) -> Transactions:
    """A distinct copy of ``tx`` of identical mining difficulty: item ids permuted and
    transactions shuffled by a ``key``-seeded permutation (``key == 0`` returns ``tx``).  The
    frequent itemsets are the images of the original ones under the item permutation, so the
    itemset count and depth are unchanged while every bitmap word differs — the per-GPU dataset
    of the weak-scaled bench (one dataset per rank, none shared)."""
    if key == 0:
        return tx
    rng = np.random.default_rng(0x5EED0000 + int(key))
    perm = rng.permutation(tx.n_items).astype(np.int32)      # old id -> new id
    order = rng.permutation(tx.n_tx)                          # new row -> old row
    lens = np.diff(tx.tx_ptr)[order]
    ptr = np.zeros(tx.n_tx + 1, np.int64)
    np.cumsum(lens, out=ptr[1:])
    row = np.repeat(np.arange(tx.n_tx, dtype=np.int64), lens)
    src = np.concatenate([np.arange(tx.tx_ptr[o], tx.tx_ptr[o + 1]) for o in order]) \
        if tx.n_tx else np.zeros(0, np.int64)
    new = perm[tx.items[src]]
    srt = np.lexsort((new, row))                               # rows ascending again
    names = None
    if tx.names is not None:
        names = [""] * tx.n_items
        for old, nid in enumerate(perm.tolist()):
            names[nid] = tx.names[old]
    return Transactions(ptr, np.ascontiguousarray(new[srt], np.int32), tx.n_items, names)


def generate(shape: "Shape | str", seed: int = 0, n_tx: Optional[int] = None,
             n_items: Optional[int] = None, calib_iters: int = 4) -> Transactions:
    """Generate clustered playlists of a named shape as CSR.

    Each playlist t has a length L_t and one or two genres; it takes the top-L_t items of
    ``log w_i + log(boost if genre(i) in genres(t)) + Gumbel`` (weighted sampling without
    replacement).  The item weights ``w`` are then re-fitted a few times so that the realised
    per-item playlist counts follow the published survival curve.
    """
    if isinstance(shape, str):
        shape = SHAPES[shape]
    if n_tx is not None or n_items is not None:
        shape = dataclasses.replace(shape, n_tx=n_tx or shape.n_tx, n_items=n_items or shape.n_items)
    rng = np.random.default_rng(seed)
    I, T = shape.n_items, shape.n_tx
    target = np.sort(_target_counts(shape, rng))[::-1]
    item_genre = rng.integers(0, shape.n_genres, size=I)
    rank_of = rng.permutation(I)  # item i gets the rank_of[i]-th largest target
    tgt = target[rank_of]
    sig = shape.len_sigma
    lens = np.clip(rng.lognormal(np.log(shape.mean_len) - sig * sig / 2, sig, size=T), 2,
                   I).astype(np.int64)
    n_g = 1 + (rng.random(T) < shape.p_two_genres)
    g1 = rng.integers(0, shape.n_genres, size=T)
    g2 = np.where(n_g > 1, rng.integers(0, shape.n_genres, size=T), g1)
    # boost so that ~genre_affinity of a playlist's tracks come from its genres
    frac_g = 1.5 / shape.n_genres
    a = shape.genre_affinity
    boost = max(1.0, a * (1 - frac_g) / max((1 - a) * frac_g, 1e-9))
    in_g = (item_genre[None, :] == g1[:, None]) | (item_genre[None, :] == g2[:, None])
    logb = np.where(in_g, np.float32(np.log(boost)), np.float32(0.0))
    gumbel = -np.log(-np.log(rng.random((T, I), dtype=np.float32) + np.float32(1e-12)) + np.float32(1e-12))
    w = np.log(tgt).astype(np.float32)
    X = None
    for it in range(calib_iters + 1):
        score = logb + gumbel + w[None, :]
        order = np.argsort(-score, axis=1, kind="stable")
        X = np.zeros((T, I), dtype=bool)
        mask = np.arange(I)[None, :] < lens[:, None]
        rows = np.repeat(np.arange(T), lens)
        X[rows, order[mask]] = True
        if it == calib_iters:
            break
        got = X.sum(axis=0).astype(np.float64) + 0.5
        w += (0.8 * np.log(tgt / got)).astype(np.float32)
    rows = [np.nonzero(X[t])[0].astype(np.int32) for t in range(T)]
    ptr = np.zeros(T + 1, dtype=np.int64)
    ptr[1:] = np.cumsum([len(r) for r in rows])
    items = np.concatenate(rows) if rows else np.zeros(0, np.int32)
    names = _track_names(I, shape.dup_names, rng)
    return Transactions(ptr, items, I, names)


def generate_large(shape: "Shape | str", seed: int = 0, n_tx: Optional[int] = None,
                   n_items: Optional[int] = None, chunk: int = 1 << 20,
                   backend: str = "auto") -> Transactions:
    """Generator for 10M+ transaction shapes (no names, no CSV).

    ``backend="native"`` (default when the extension is built): the multi-threaded C++
    generator (csrc/host/synth.cpp, ~2 s per 10M transactions, identical output for any thread
    count); ``"numpy"``: the vectorised reference implementation below (same model, different
    random stream)."""
    if isinstance(shape, str):
        shape = SHAPES[shape]
    if n_tx is not None or n_items is not None:
        shape = dataclasses.replace(shape, n_tx=n_tx or shape.n_tx, n_items=n_items or shape.n_items)
    if backend in ("auto", "native"):
        try:
            from ..ops import native
            N = native.load()
        except Exception:
            if backend == "native":
                raise
            N = None
        if N is not None:
            ptr, items = N.synth_transactions(shape.n_tx, shape.n_items, shape.mean_len,
                                              shape.n_genres, shape.genre_affinity, 0.85, seed)
            return Transactions(ptr, items, shape.n_items, None)
    rng = np.random.default_rng(seed)
    I, T = shape.n_items, shape.n_tx
    # heavy-tailed (Zipf-like) popularity for million-item vocabularies
    pop = 1.0 / np.power(np.arange(1, I + 1, dtype=np.float64), 0.85)
    pop = pop[rng.permutation(I)]
    G = shape.n_genres
    item_genre = rng.integers(0, G, size=I)
    order = np.argsort(item_genre, kind="stable")
    g_start = np.searchsorted(item_genre[order], np.arange(G + 1))
    w_sorted = pop[order]
    cdf_sorted = np.cumsum(w_sorted)
    glob_cdf = np.cumsum(pop) / pop.sum()
    genre_mass = np.add.reduceat(w_sorted, g_start[:-1])
    genre_p = genre_mass / genre_mass.sum()
    ptrs = [np.zeros(1, np.int64)]
    out = []
    base = 0
    for c0 in range(0, T, chunk):
        n = min(chunk, T - c0)
        lens = np.clip(rng.poisson(shape.mean_len, size=n), 1, None)
        g = rng.choice(G, size=n, p=genre_p)
        tot = int(lens.sum())
        tx_of = np.repeat(np.arange(n), lens)
        in_genre = rng.random(tot) < shape.genre_affinity
        lo = np.where(g_start[g[tx_of]] > 0, cdf_sorted[np.maximum(g_start[g[tx_of]] - 1, 0)], 0.0)
        hi = cdf_sorted[g_start[g[tx_of] + 1] - 1]
        u = rng.random(tot)
        pick_g = order[np.minimum(np.searchsorted(cdf_sorted, lo + u * (hi - lo)), I - 1)]
        pick_x = np.minimum(np.searchsorted(glob_cdf, rng.random(tot)), I - 1)
        it = np.where(in_genre, pick_g, pick_x).astype(np.int64)
        key = np.unique(tx_of.astype(np.int64) * I + it)
        t_id = key // I
        cnt = np.bincount(t_id, minlength=n)
        out.append((key % I).astype(np.int32))
        ptrs.append(base + np.cumsum(cnt))
        base += int(cnt.sum())
    return Transactions(np.concatenate(ptrs), np.concatenate(out), I, None)


def _track_names(n: int, dup_names: int, rng: np.random.Generator) -> List[str]:
    syll = ["la", "mo", "ri", "ta", "ven", "sol", "kai", "dre", "nu", "bel", "sky", "fire",
            "gold", "moon", "zo", "pa", "lu", "ny", "ex", "or"]
    names = []
    seen = set()
    for i in range(n):
        while True:
            k = int(rng.integers(2, 5))
            w = "".join(rng.choice(syll, size=k)).capitalize()
            nm = f"{w} {i:05d}"
            if nm not in seen:
                break
        seen.add(nm)
        names.append(nm)
    # reproduce ds2's "48 names with >1 URI": item j takes the name of item j - 1
    if dup_names:
        victims = rng.choice(np.arange(1, n), size=min(dup_names, n - 1), replace=False)
        for v in victims:
            names[v] = names[v - 1]
    return names


def to_reference_csv(tx: Transactions, path: "str | pathlib.Path | None" = None,
                     seed: int = 0, dup_rows: Optional[float] = None) -> str:
    """Write the 8-column reference CSV schema (``pid,track_uri,track_name,artist_name,
    artist_uri,album_name,album_uri,duration_ms``); one row per (playlist, track).

    Artists are consistent per track (one URI per artist name), so the job's artist
    validator (``machine-learning/main.py:62-68``) passes.
    """
    rng = np.random.default_rng(seed + 7)
    n = tx.n_items
    names = tx.names or [f"Track {i:05d}" for i in range(n)]
    n_art = max(1, n // 3)
    artist_of = rng.integers(0, n_art, size=n)
    album_of = rng.integers(0, max(1, n // 2), size=n)
    dur = rng.integers(90_000, 420_000, size=n)
    dup = 0.01 if dup_rows is None else dup_rows
    buf = io.StringIO()
    w = csv.writer(buf, lineterminator="\n")
    w.writerow(["pid", "track_uri", "track_name", "artist_name", "artist_uri", "album_name",
                "album_uri", "duration_ms"])
    for pid, row in enumerate(tx.rows()):
        extra = row[rng.random(len(row)) < dup] if dup > 0 else row[:0]
        for i in list(row) + list(extra):
            a = int(artist_of[i])
            w.writerow([pid, f"spotify:track:{i:022d}", names[i], f"Artist, \"{a}\"",
                        f"spotify:artist:{a:022d}", f"Album {int(album_of[i])}",
                        f"spotify:album:{int(album_of[i]):022d}", int(dur[i])])
    text = buf.getvalue()
    if path is not None:
        pathlib.Path(path).write_text(text, encoding="utf-8")
    return text


def item_support_curve(tx: Transactions, supports) -> List[Tuple[float, int]]:
    cnt = np.bincount(tx.items, minlength=tx.n_items)
    return [(s, int((cnt / tx.n_tx >= s).sum())) for s in supports]
