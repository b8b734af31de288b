#!/usr/bin/env bash
# Round-3 a: first GPU run of the count-only deep miner: parity tests, then a 0.02 probe.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=60
step pytest_deep 400 python -u -m pytest tests/test_gpu_deep.py -v -x --timeout 120 --timeout-method thread
step deep_probe 300 python -u scripts/deep_probe.py --supports 0.02 --reps 2
