#!/usr/bin/env bash
# Round-3 y: item-shard batch size sweep on config 3 (world 1), plus a short rocprof kernel trace
# of one shard-mode step.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
run c3_shard_sweep 600 python -u scripts/c3_shard.py --mode shard --steps 2 --warmup 1 --batch-div 1,4,16,64
