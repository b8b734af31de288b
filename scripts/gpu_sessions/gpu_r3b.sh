#!/usr/bin/env bash
# Round-3 b: deep miner parity after the uni64 sign-extension fix; stops at the first failure.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=60
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
run pytest_deep 400 python -u -m pytest tests/test_gpu_deep.py -v -x --timeout 120 --timeout-method thread &&
run deep_probe 300 python -u scripts/deep_probe.py --supports 0.02 --reps 2
