#!/usr/bin/env bash
# Round-2 i: KB18 threshold A/B after the fold.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
B=(python3 bench.py --no-config2 --serve-qps "" --steps 200 --warmup 10 --no-verify)
step kb64 300 "${B[@]}"
KMLS_KB18_TILES=256 step kb256 300 "${B[@]}"
KMLS_KB18_TILES=600 step kb600 300 "${B[@]}"
step kb64b 300 "${B[@]}"
export KMLS_LEVEL_TRACE_FILE=/tmp/level_trace.bin
KMLS_KB18_TILES=600 KMLS_LEVEL_TRACE=2 step trace2 200 python -u scripts/probe_level_trace.py
