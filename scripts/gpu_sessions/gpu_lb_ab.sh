#!/usr/bin/env bash
# Look-back width A/B (KMLS_LB_WIN=1: one window of 64 per round; default: whole block) with the
# GPU kernel tests first, then per-tile phase traces of a big level for both.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_kern 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread
for w in 0 1 0 1; do
  KMLS_LB_WIN=$w step bench_lb${w}_$RANDOM 240 python -u bench.py --steps 50 --warmup 5
done
export KMLS_LEVEL_TRACE_FILE=/tmp/level_trace.bin
for w in 0 1; do
  KMLS_LB_WIN=$w KMLS_LEVEL_TRACE=6 step trace6_lb$w 200 python -u scripts/probe_level_trace.py
done
