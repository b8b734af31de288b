#!/usr/bin/env bash
# Round-3 j: work stealing with per-wave mailboxes and done flags (no hot-address polling).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=30
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py --no-parity --reps 1 --supports 0.02 --world 8"
run deep_tests 400 python -u -m pytest tests/test_gpu_deep.py -v -x --timeout 120 --timeout-method thread &&
run sweep1 300 python -u scripts/deep_probe.py --no-parity --reps 3 --supports 0.02 --sweep 1024:1024:8:3:0,0:64:8:3:1:1,0:128:8:3:1:1,0:256:8:3:1:1,0:512:8:3:1:1,0:128:16:3:1:1,0:128:4:3:1:1 &&
run w8_rounds 200 $P --rounds --budget0 1024 --budget 1024 &&
run w8_s64 200 $P --budget 64 &&
run w8_s128 200 $P --budget 128 &&
run w8_s256 200 $P --budget 256 &&
run w8_s512 200 $P --budget 512
