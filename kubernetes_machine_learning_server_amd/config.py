"""Typed settings over the reference's env-var config surface.

Every variable name and default of the reference is kept, including the API's ``PICKLE_DIR``
vs the job's ``PICKLES_FOLDER`` (``machine-learning/main.py:17-47``,
``rest_api/app/main.py:31-47``).  New knobs: ``MINER`` (gpu|cpu|oracle), ``RULES_MODE``
(full|pairs), ``NUM_GPUS``, ``SERVE_BACKEND`` (auto|hip|loop|cpu), ``BATCH_MAX``, ``BATCH_WAIT_US``,
``MIN_CONFIDENCE``, ``KMLS_FAULT`` (fault injection, tests only).
"""
from __future__ import annotations

import dataclasses
import os
import pathlib
from typing import Optional

from .utils.dotenv import load_dotenv


def _env(name: str, default: str) -> str:
    v = os.environ.get(name)
    return default if v is None else v


@dataclasses.dataclass
class JobSettings:
    min_support: float
    base_dir: pathlib.Path
    datasets_dir: pathlib.Path
    pickles_folder: pathlib.Path
    recommendations_file: str
    best_tracks_file: str
    data_invalidation_file: str
    regex_filename: str
    top_tracks_save_percentile: float
    base_index: int = 1
    sample_ratio: float = 1.0
    experiment_supports: bool = False
    miner: str = "auto"          # gpu | cpu | oracle | auto
    rules_mode: str = "full"     # full (all itemsets, as mlxtend) | pairs (SURVEY §0 fast path)
    # RULES_MODE=pairs on several GPUs: how the pair matrix is formed (parallel/pairs.py:
    # allreduce | reduce_scatter | alltoall | ring), or "trie" (mine 2-itemsets, gather sub-tries)
    pairs_strategy: str = "reduce_scatter"
    # KMLS_DIST_MODE: auto | deep | tx | item | shard | replicate (multi-GPU mining); auto = deep
    # (the headline DFS split, parallel/deep.py) for GPU full mining of <= 4096 transactions
    dist_mode: str = "auto"
    num_gpus: int = 1
    min_confidence: float = 0.04  # legacy confidence rules (main.py:227)
    checkpoint_dir: Optional[pathlib.Path] = None  # KMLS_CHECKPOINT_DIR: phase resume
    dist_timeout_s: float = 600.0      # KMLS_DIST_TIMEOUT_S: process-group init + collectives
    sweep_timeout_s: float = 86400.0   # KMLS_SWEEP_TIMEOUT_S: ranks waiting for rank 0's sweep

    DIST_MODES = ("auto", "deep", "tx", "item", "shard", "replicate")

    def __post_init__(self):
        # 'local' (every rank mines the whole dataset) is a DistMiner test mode: in the job it
        # would gather N copies of every itemset into the rule map
        if self.dist_mode not in self.DIST_MODES:
            raise ValueError(f"KMLS_DIST_MODE={self.dist_mode!r}: expected one of "
                             f"{', '.join(self.DIST_MODES)}")

    @property
    def dataset_list_file(self) -> pathlib.Path:
        return self.base_dir / "datasets_list.txt"

    @property
    def dataset_history_file(self) -> pathlib.Path:
        return self.base_dir / "dataset_history.csv"

    @property
    def marker_file(self) -> pathlib.Path:
        return self.base_dir / self.data_invalidation_file

    @classmethod
    def from_env(cls, dotenv: bool = True) -> "JobSettings":
        if dotenv:
            load_dotenv()
        base = pathlib.Path(_env("BASE_DIR", "../datasets/"))
        return cls(
            min_support=float(_env("MIN_SUPPORT", "0.05")),
            base_dir=base,
            datasets_dir=pathlib.Path(_env("DATASETS_DIR", "../datasets/")),
            pickles_folder=base / _env("PICKLES_FOLDER", "pickles/"),
            recommendations_file=_env("RECOMMENDATIONS_FILE", "recommendations.pickle"),
            best_tracks_file=_env("BEST_TRACKS_FILE", "best_tracks.pickle"),
            data_invalidation_file=_env("DATA_INVALIDATION_FILE", "last_execution.txt"),
            regex_filename=_env("REGEX_FILENAME", "2023_spotify_ds*.csv"),
            top_tracks_save_percentile=float(_env("TOP_TRACKS_SAVE_PERCENTILE", "0.03")),
            sample_ratio=float(_env("SAMPLE_RATIO", "1")),
            experiment_supports=_env("EXPERIMENT_SUPPORTS", "false").lower() in ("1", "true", "yes"),
            miner=_env("MINER", "auto").lower(),
            rules_mode=_env("RULES_MODE", "full").lower(),
            pairs_strategy=_env("PAIRS_STRATEGY", "reduce_scatter").lower(),
            dist_mode=_env("KMLS_DIST_MODE", "auto").lower(),
            num_gpus=int(_env("NUM_GPUS", "1")),
            min_confidence=float(_env("MIN_CONFIDENCE", "0.04")),
            checkpoint_dir=(pathlib.Path(os.environ["KMLS_CHECKPOINT_DIR"])
                            if os.environ.get("KMLS_CHECKPOINT_DIR") else None),
            dist_timeout_s=float(_env("KMLS_DIST_TIMEOUT_S", "600")),
            sweep_timeout_s=float(_env("KMLS_SWEEP_TIMEOUT_S", "86400")),
        )


@dataclasses.dataclass
class ApiSettings:
    base_dir: pathlib.Path
    pickles_folder: pathlib.Path
    k_best_tracks: int
    version: str
    polling_wait_in_minutes: float
    recommendations_file: str
    best_tracks_file: str
    data_invalidation_file: str
    app_path_from_root: Optional[pathlib.Path]
    # auto | hip (every batch through the batch kernels) | loop (queries up to the wave matcher's
    # merge size through the persistent serving kernel) | cpu | python
    serve_backend: str = "auto"
    batch_max: int = 256
    batch_wait_us: int = 200
    gpu_min_batch: int = 16       # below this a batch is answered by the C++ CPU matcher

    @property
    def cache_file(self) -> pathlib.Path:
        return self.base_dir / self.data_invalidation_file

    @property
    def templates_dir(self) -> pathlib.Path:
        here = pathlib.Path(__file__).resolve().parent / "serve"
        if self.app_path_from_root is not None:
            cand = self.app_path_from_root / "templates"
            if (cand / "client.html").exists():
                return cand
        return here / "templates"

    @property
    def static_dir(self) -> pathlib.Path:
        if self.app_path_from_root is not None:
            return self.app_path_from_root / "static"
        return pathlib.Path(__file__).resolve().parent / "serve" / "static"

    @classmethod
    def from_env(cls, dotenv: bool = True) -> "ApiSettings":
        if dotenv:
            load_dotenv()
        base = pathlib.Path(_env("BASE_DIR", "machine-learning/api-data/"))
        app_path = os.environ.get("APP_PATH_FROM_ROOT")
        return cls(
            base_dir=base,
            pickles_folder=base / _env("PICKLE_DIR", "pickles/"),
            k_best_tracks=int(_env("K_BEST_TRACKS", "10")),
            version=_env("VERSION", "V0.1"),
            polling_wait_in_minutes=float(_env("POLLING_WAIT_IN_MINUTES", "1")),
            recommendations_file=_env("RECOMMENDATIONS_FILE", "recommendations.pickle"),
            best_tracks_file=_env("BEST_TRACKS_FILE", "best_tracks.pickle"),
            data_invalidation_file=_env("DATA_INVALIDATION_FILE", "last_execution.txt"),
            app_path_from_root=pathlib.Path(app_path) if app_path else None,
            serve_backend=_env("SERVE_BACKEND", "auto").lower(),
            batch_max=int(_env("BATCH_MAX", "256")),
            batch_wait_us=int(_env("BATCH_WAIT_US", "200")),
            gpu_min_batch=int(_env("GPU_MIN_BATCH", "16")),
        )
