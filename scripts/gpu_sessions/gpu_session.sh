#!/usr/bin/env bash
# Canonical GPU session (what the driver runs at round end, plus evidence): the GPU test suite,
# smoke(), the headline bench, the replicated-partition scaling probe and a per-step kernel
# timeline.  Every step has its own time limit; a fault/abort/timeout stops the session.
#   gpurun --timeout 1200 -- bash scripts/gpu_session.sh
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 240 python -u bench.py --steps 50 --warmup 5
step partition_scaling 300 python -u scripts/partition_scaling.py
step ktrace 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline.md 2>&1
rm -rf /tmp/prof_k
