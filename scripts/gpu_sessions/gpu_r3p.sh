#!/usr/bin/env bash
# Round-3 p: donation granularity (split_min) x check interval (budget), 1 GPU and the 8-rank split.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=30
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py --no-parity"
run sweep 300 $P --reps 3 --supports 0.02 --sweep 0:256:8:3:1:1,0:256:64:3:1:1,0:256:1000000:3:1:1,0:128:64:3:1:1,0:128:1000000:3:1:1,0:64:1000000:3:1:1 &&
run w8_256_8 120 $P --reps 1 --supports 0.02 --world 8 --budget 256 --split-min 8 &&
run w8_256_64 120 $P --reps 1 --supports 0.02 --world 8 --budget 256 --split-min 64 &&
run w8_256_inf 120 $P --reps 1 --supports 0.02 --world 8 --budget 256 --split-min 1000000 &&
run w8_128_64 120 $P --reps 1 --supports 0.02 --world 8 --budget 128 --split-min 64 &&
run w8_128_inf 120 $P --reps 1 --supports 0.02 --world 8 --budget 128 --split-min 1000000 &&
run w8_64_inf 120 $P --reps 1 --supports 0.02 --world 8 --budget 64 --split-min 1000000
