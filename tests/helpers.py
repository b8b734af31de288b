"""Shared fixtures: a tmp "PVC" populated by the real job on synthetic reference-schema CSVs."""
import os
import pathlib

from kubernetes_machine_learning_server_amd.config import ApiSettings, JobSettings
from kubernetes_machine_learning_server_amd.data.synthetic import generate, to_reference_csv


def make_datasets(root: pathlib.Path, shapes=("tiny", "tiny"), seeds=(1, 2)):
    ds = root / "datasets"
    ds.mkdir(parents=True, exist_ok=True)
    for i, (shape, seed) in enumerate(zip(shapes, seeds), 1):
        tx = generate(shape, seed=seed)
        to_reference_csv(tx, ds / f"2023_spotify_ds{i}.csv", seed=seed)
    return ds


def job_settings(root: pathlib.Path, **kw) -> JobSettings:
    base = root / "api-data"
    cfg = JobSettings(min_support=kw.pop("min_support", 0.05), base_dir=base,
                      datasets_dir=root / "datasets", pickles_folder=base / "pickles",
                      recommendations_file="recommendations.pickle",
                      best_tracks_file="best_tracks.pickle",
                      data_invalidation_file="last_execution.txt",
                      regex_filename="2023_spotify_ds*.csv",
                      top_tracks_save_percentile=kw.pop("pct", 0.3), miner=kw.pop("miner", "cpu"))
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def api_settings(root: pathlib.Path, **kw) -> ApiSettings:
    base = root / "api-data"
    cfg = ApiSettings(base_dir=base, pickles_folder=base / "pickles", k_best_tracks=10,
                      version="V-test", polling_wait_in_minutes=60,
                      recommendations_file="recommendations.pickle",
                      best_tracks_file="best_tracks.pickle",
                      data_invalidation_file="last_execution.txt",
                      app_path_from_root=None, serve_backend=kw.pop("serve_backend", "cpu"))
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg
