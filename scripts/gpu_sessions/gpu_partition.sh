#!/usr/bin/env bash
# Per-rank steady-state cost of the replicated multi-GPU mode (each rank its own miner).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
for w in 1 2 4 8; do step part_w$w 300 python -u scripts/probe_partition_rank.py $w max; done
