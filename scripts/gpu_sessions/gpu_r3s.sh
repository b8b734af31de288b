#!/usr/bin/env bash
# Round-3 s: direct hand-offs, shorter check intervals.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=30
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py --no-parity"
run sweep 300 $P --reps 3 --supports 0.02 --sweep 0:8:8:3:1:1,0:16:8:3:1:1,0:32:8:3:1:1,0:64:8:3:1:1 &&
run w8_8 120 $P --reps 1 --supports 0.02 --world 8 --budget 8 &&
run w8_16 120 $P --reps 1 --supports 0.02 --world 8 --budget 16 &&
run w8_32 120 $P --reps 1 --supports 0.02 --world 8 --budget 32 &&
run w8_64 120 $P --reps 1 --supports 0.02 --world 8 --budget 64
