#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_LEVEL_TRACE_FILE=/tmp/level_trace.bin
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "miner or fused or compact or partition or replicated or dfs"
for c in 1 2 4; do
  KMLS_COUNT_CPT=$c step bench_cpt$c 240 python -u bench.py --steps 30 --warmup 5
  KMLS_COUNT_CPT=$c KMLS_LEVEL_TRACE=5 step trace5_cpt$c 200 python -u scripts/probe_level_trace.py
done
