#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_e2e 600 python -u -m pytest tests/test_gpu_e2e.py -m gpu -v -x --timeout 300 --timeout-method thread
