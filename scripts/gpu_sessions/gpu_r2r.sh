#!/usr/bin/env bash
# Round-2 r: checkpoint — full GPU suite, smoke, full bench.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_all 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_full 600 python3 bench.py
