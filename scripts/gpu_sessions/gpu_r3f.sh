#!/usr/bin/env bash
# Round-3 f (re-entry): full GPU suite, then the shipped bench.py at N=1, then kernel stats of
# the headline deep miner.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python -u bench.py --steps 10 --warmup 2
cp gpurun_out/bench.log gpurun_out/bench.json.log
step ktrace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace_deep -o run -- python3 scripts/deep_probe.py --no-parity --reps 3 --supports 0.02
