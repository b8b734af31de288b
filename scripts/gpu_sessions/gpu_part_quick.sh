#!/usr/bin/env bash
# Replicated-partition change check: partition tests, the scaling probe, rank timelines.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_part 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "partition or replic or prefetch"
step partition_scaling 300 python -u scripts/partition_scaling.py
WORLD=8 RANKS="0" bash scripts/gpu_partition_trace.sh
