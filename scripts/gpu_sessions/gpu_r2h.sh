#!/usr/bin/env bash
# Round-2 h: epilogue variant A/B (correctness subset + headline + level traces).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_fold 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -k "miner_matches_cpu or max_len or compact or repeat or rule_index or partition or chunked"
B=(python3 bench.py --no-config2 --serve-qps "" --steps 100 --warmup 5)
step bench_v 300 "${B[@]}"
export KMLS_LEVEL_TRACE_FILE=/tmp/level_trace.bin
KMLS_LEVEL_TRACE=2 step trace2 200 python -u scripts/probe_level_trace.py
KMLS_LEVEL_TRACE=4 step trace4 200 python -u scripts/probe_level_trace.py
KMLS_LEVEL_TRACE=7 step trace7 200 python -u scripts/probe_level_trace.py
