#!/usr/bin/env bash
# Round-3 u: batch steps of up to 512 / 1024 candidate pairs (kCap): parity + timing.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=30
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py --no-parity"
run deep_tests 300 python -u -m pytest tests/test_gpu_deep.py -x -q --timeout 120 --timeout-method thread &&
run sweep 300 $P --reps 3 --supports 0.02 --sweep 0:16:8:3:1:1,0:32:8:3:1:1 &&
run w8 120 $P --reps 2 --supports 0.02 --world 8
