#!/usr/bin/env bash
# Round-2 g: fold fixes (leaf levels), full GPU suite, headline + timeline + level traces.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_all 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
B=(python3 bench.py --no-config2 --serve-qps "" --steps 50 --warmup 5)
step bench_fold 300 "${B[@]}"
export KMLS_LEVEL_TRACE_FILE=/tmp/level_trace.bin
KMLS_LEVEL_TRACE=2 step trace2 200 python -u scripts/probe_level_trace.py
KMLS_LEVEL_TRACE=4 step trace4 200 python -u scripts/probe_level_trace.py
KMLS_LEVEL_TRACE=7 step trace7 200 python -u scripts/probe_level_trace.py
