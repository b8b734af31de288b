#!/usr/bin/env bash
# Session-3 GPU check of HEAD: GPU suite, smoke, headline bench, replicated-partition scaling
# probe, and a rocprofv3 kernel-stats pass of the headline bench.
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 240 python -u bench.py --steps 30 --warmup 5
step partition_scaling 300 python -u scripts/partition_scaling.py
step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s3a -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify
