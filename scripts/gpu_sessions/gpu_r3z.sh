#!/usr/bin/env bash
# Round-3 z (re-run in round 4 as r4t): item-shard rounds without the per-round re-selection:
# GPU shard tests, batch size sweep on config 3 (world 1), kernel trace of one shard step.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
run shard_tests 300 python -u -m pytest tests/test_item_shard.py -x -q -m gpu --timeout 200 --timeout-method thread &&
run c3_shard_sweep2 600 python -u scripts/c3_shard.py --mode shard --steps 2 --warmup 1 --batch-div 2,4,8 &&
step shard_ktrace 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4t_prof_shard -o shard -- python3 scripts/c3_shard.py --mode shard --steps 1 --warmup 1
