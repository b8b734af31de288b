#!/usr/bin/env bash
# Round-3 r: direct hand-offs (requester identity in the mailbox, per-wave inbox): parity,
# check-interval sweep at 1 GPU and the 8-rank split.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=30
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py --no-parity"
run deep_tests 300 python -u -m pytest tests/test_gpu_deep.py -x -v --timeout 120 --timeout-method thread &&
run sweep 300 $P --reps 3 --supports 0.02 --sweep 0:64:8:3:1:1,0:128:8:3:1:1,0:256:8:3:1:1,0:512:8:3:1:1,0:128:1000000:3:1:1 &&
run w8_64 120 $P --reps 1 --supports 0.02 --world 8 --budget 64 &&
run w8_128 120 $P --reps 1 --supports 0.02 --world 8 --budget 128 &&
run w8_256 120 $P --reps 1 --supports 0.02 --world 8 --budget 256 &&
run w8_128_inf 120 $P --reps 1 --supports 0.02 --world 8 --budget 128 --split-min 1000000
