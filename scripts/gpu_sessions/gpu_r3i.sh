#!/usr/bin/env bash
# Round-3 i: spill-round budgets for the 8-rank split (round floor = budget x step latency) and
# for one rank; steal mode at coarse check intervals.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=30
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py --no-parity --reps 1 --supports 0.02 --world 8 --rounds"
run sweep1 300 python -u scripts/deep_probe.py --no-parity --reps 3 --supports 0.02 --sweep 1024:1024:8:3:0,1024:512:8:3:0,512:512:8:3:0,1024:256:8:3:0,512:256:8:3:0,256:256:8:3:0,0:512:8:3:1:1,0:1024:8:3:1:1 &&
run w8_1024_1024 200 $P --budget0 1024 --budget 1024 &&
run w8_512_256 200 $P --budget0 512 --budget 256 &&
run w8_256_256 200 $P --budget0 256 --budget 256 &&
run w8_256_128 200 $P --budget0 256 --budget 128 &&
run w8_128_128 200 $P --budget0 128 --budget 128 &&
run w8_128_64 200 $P --budget0 128 --budget 64 &&
run w8_64_64 200 $P --budget0 64 --budget 64
