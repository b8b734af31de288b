#!/usr/bin/env bash
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_LEVEL_TRACE_FILE=/tmp/level_trace.bin
KMLS_LEVEL_TRACE=5 step trace5 200 python -u scripts/probe_level_trace.py
KMLS_LEVEL_TRACE=10 step trace10 200 python -u scripts/probe_level_trace.py
KMLS_LEVEL_TRACE=1 step trace1 200 python -u scripts/probe_level_trace.py
