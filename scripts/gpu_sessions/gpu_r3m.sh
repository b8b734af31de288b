#!/usr/bin/env bash
# Round-3 m: config 3 (10M x 1M) at min_support 2e-4 (14.8k frequent items), tx-DP on 1 GPU.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step c3_2e4 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --min-support 0.0002 --mode tx --steps 2 --warmup 1 &&
step c3_5e4 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --min-support 0.0005 --mode tx --steps 2 --warmup 1
