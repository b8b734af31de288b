#!/usr/bin/env bash
# Round-3 v: the full GPU suite once more (the rule-map test's stream fix).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
