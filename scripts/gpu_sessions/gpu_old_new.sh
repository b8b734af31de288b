#!/usr/bin/env bash
# Same-box A/B: the previous build (ab_old/, not tracked) vs the working tree, after the GPU
# kernel tests of the working tree.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_kern 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread
for i in 1 2 3; do
  step old_$i 240 python -u ab_old/bench.py --steps 50 --warmup 5 --no-verify
  step new_$i 240 python -u bench.py --steps 50 --warmup 5 --no-verify
done
step ktrace 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline.md 2>&1
rm -rf /tmp/prof_k
