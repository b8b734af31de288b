#!/usr/bin/env bash
# Round-2 re-entry check of HEAD: full GPU suite, smoke(), the driver's default bench line.
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py --gpus 1 --steps 20 --warmup 5
