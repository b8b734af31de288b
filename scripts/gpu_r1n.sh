#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 600
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 240 python -u bench.py
