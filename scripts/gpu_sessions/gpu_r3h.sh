#!/usr/bin/env bash
# Round-3 h: work stealing without fences (write-through hand-offs, per-slot polling):
# parity, steal vs rounds sweep at ds1 @0.02, 8-rank split simulation.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=30
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py"
run deep_tests 400 python -u -m pytest tests/test_gpu_deep.py -v -x --timeout 120 --timeout-method thread &&
run sweep 400 $P --reps 3 --supports 0.02 --sweep 1024:1024:8:3:0,0:256:8:3:1:1,0:64:8:3:1:1,0:16:8:3:1:1,0:64:16:3:1:1,0:64:4:3:1:1,0:64:8:3:1:8 &&
run world8 200 $P --no-parity --reps 1 --supports 0.02 --world 8 --budget 64 --split-min 8 &&
run world8_rounds 200 $P --no-parity --reps 1 --supports 0.02 --world 8 --rounds --budget 1024 --budget0 1024
