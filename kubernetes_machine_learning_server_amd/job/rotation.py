"""Dataset catalog + round-robin run cursor (file formats §2.F).

Reference: ``get_dataset_list``/``read_dataset``/``write_dataset_and_reset_index``
(``machine-learning/main.py:315-346``) and ``read_history_csv``/``get_next_run_index``/
``append_dataset_history`` (``main.py:349-411``).  Same files and formats:

* ``datasets_list.txt``: one path per line, ``sorted(DATASETS_DIR.glob(REGEX_FILENAME))``;
* ``dataset_history.csv``: header ``time,dataset_index,dataset_file``; 1-based index that wraps
  to ``BASE_INDEX``; malformed last line → ``BASE_INDEX``;
* marker ``last_execution.txt``: Sao Paulo time, no newline, written LAST.

Differences (documented fixes): the next-index computation takes the
dataset list as an argument instead of a module global (B.2); the marker is written atomically.
"""
from __future__ import annotations

import os
import pathlib
from typing import List

from ..config import JobSettings
from ..utils.atomic_io import append_line, atomic_write_text
from ..utils.timeutil import current_time_str

HISTORY_HEADER = "time,dataset_index,dataset_file\n"


def write_dataset_and_reset_index(cfg: JobSettings) -> List[str]:
    cfg.datasets_dir.mkdir(parents=True, exist_ok=True)
    cfg.base_dir.mkdir(parents=True, exist_ok=True)
    datasets = [str(p.as_posix()) for p in sorted(cfg.datasets_dir.glob(cfg.regex_filename))]
    if not datasets:
        raise FileNotFoundError("No datasets found with pattern. Please check your environment setup.")
    atomic_write_text(cfg.dataset_list_file, "".join(f"{d}\n" for d in datasets))
    print(f"Datasets written to {cfg.dataset_list_file.as_posix()}")
    return datasets


def read_dataset(cfg: JobSettings) -> List[str]:
    with open(cfg.dataset_list_file, "r") as f:
        datasets = f.read().splitlines()
    print(f"Datasets read from {cfg.dataset_list_file}")
    return datasets


def get_dataset_list(cfg: JobSettings) -> List[str]:
    if not os.path.exists(cfg.dataset_list_file):
        print("Current dataset file not found. Initializing...")
        return write_dataset_and_reset_index(cfg)
    return read_dataset(cfg)


def read_history_csv(cfg: JobSettings) -> List[str]:
    if not os.path.exists(cfg.dataset_history_file):
        print(f"{cfg.dataset_history_file} not found, returning empty history.")
        return []
    with open(cfg.dataset_history_file, "r", encoding="utf-8") as f:
        return f.read().splitlines()


def get_next_run_index(cfg: JobSettings, datasets: List[str]) -> int:
    lines = read_history_csv(cfg)
    if len(lines) <= 1:
        print("No previous run found in history, defaulting to base index.")
        return cfg.base_index
    parts = lines[-1].split(",")
    try:
        new_index = int(parts[1].strip()) + 1
        if new_index > len(datasets):
            new_index = cfg.base_index
        return new_index
    except (ValueError, IndexError):
        print("History file had a malformed line. Defaulting to base index.")
        return cfg.base_index


def append_dataset_history(cfg: JobSettings, dataset_index: int, dataset_file: str) -> str:
    """Append the run row, then write the invalidation marker (LAST, atomically)."""
    ts = current_time_str()
    append_line(cfg.dataset_history_file, f"{ts},{dataset_index},{dataset_file}\n", HISTORY_HEADER)
    atomic_write_text(cfg.marker_file, ts)
    print(f"Appended dataset {dataset_index} ({dataset_file}) to history.")
    print(f"Updated cache file: {cfg.marker_file}")
    return ts
