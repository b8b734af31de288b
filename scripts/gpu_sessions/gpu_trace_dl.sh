#!/usr/bin/env bash
# Per-tile phase traces of the two biggest levels + with/without download timing.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_LEVEL_TRACE_FILE=/tmp/level_trace.bin
KMLS_LEVEL_TRACE=6 step trace6 200 python -u scripts/probe_level_trace.py
KMLS_LEVEL_TRACE=7 step trace7 200 python -u scripts/probe_level_trace.py
step probe_dl 240 python -u scripts/probe_download.py
