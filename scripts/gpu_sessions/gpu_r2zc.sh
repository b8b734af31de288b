#!/usr/bin/env bash
# Round-2 zc: one-rank RCCL communicator test + tx-DP multi-rank tests, then scripts/gpu_r2zb.sh.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_dist 600 python -u -m pytest tests/test_gpu_dist.py -v -x --timeout 300 --timeout-method thread
bash "$(dirname "$0")/gpu_r2zb.sh"
