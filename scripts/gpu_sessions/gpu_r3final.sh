#!/usr/bin/env bash
# Round-3 end: the committed tree — full GPU suite and smoke.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
run pytest_gpu_final 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread &&
run smoke_final 300 python -u -c "import __graft_entry__ as g; g.smoke()"
