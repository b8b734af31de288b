#!/usr/bin/env bash
# Round-3 w: waiting waves ask the busiest of 4 candidates (published open-class counts);
# parity, timing at 1 GPU and the 8-rank split; then the full GPU suite.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=30
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py --no-parity"
run deep_tests 300 python -u -m pytest tests/test_gpu_deep.py -x -q --timeout 120 --timeout-method thread &&
run sweep 300 $P --reps 3 --supports 0.02 --sweep 0:16:8:3:1:1,0:32:8:3:1:1 &&
run w8 120 $P --reps 2 --supports 0.02 --world 8 &&
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
