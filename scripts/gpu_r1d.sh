#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DFS_TIMEOUT_MS=10000
step dfs_debug 200 python -u scripts/dfs_debug.py
step bench_persist 240 python -u bench.py --steps 30 --warmup 5
step bench_levelwise 240 python -u bench.py --steps 30 --warmup 5 --level-wise
step pytest_gpu 400 python -u -m pytest tests -m gpu -v -x --timeout 120
step rocprof 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3
