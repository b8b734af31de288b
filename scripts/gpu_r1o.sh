#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 600
step bench 240 python -u bench.py
step pairs_rs 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --pairs reduce_scatter --steps 3 --warmup 1
step partition_scaling 300 python -u scripts/partition_scaling.py
