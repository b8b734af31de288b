#!/usr/bin/env bash
# Quick check after a kernel change: GPU kernel tests, headline bench x2, kernel timeline.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_kern 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread
step bench_a 240 python -u bench.py --steps 50 --warmup 5
step bench_b 240 python -u bench.py --steps 50 --warmup 5
step partition_scaling 300 python -u scripts/partition_scaling.py
step ktrace 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline.md 2>&1
rm -rf /tmp/prof_k
