#!/usr/bin/env bash
# Round-3 k: full GPU suite after the hygiene pass, smoke, the shipped bench.py, and a kernel
# trace of the headline (work-stealing deep miner).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread &&
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" &&
step bench 600 python -u bench.py --steps 10 --warmup 2 &&
step ktrace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace_deep -o run -- python3 scripts/deep_probe.py --no-parity --reps 3 --supports 0.02
