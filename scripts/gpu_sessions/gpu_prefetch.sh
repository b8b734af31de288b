#!/usr/bin/env bash
# Launch-ahead (prefetch) pipeline: full GPU tests, then same-box benches with / without it,
# the partition scaling probe and a kernel timeline.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
for i in 1 2 3; do
  step pre_$i 240 python -u bench.py --steps 50 --warmup 5
  step nopre_$i 240 python -u bench.py --steps 50 --warmup 5 --no-prefetch
done
step partition_scaling 300 python -u scripts/partition_scaling.py
step ktrace 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline.md 2>&1
rm -rf /tmp/prof_k
