#!/usr/bin/env bash
# Deferred-download variants: kernel tests, copy-block A/B, download cost, kernel timeline.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_kern 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread
for cb in 8 16 32 64 8 16 32 64; do
  KMLS_COPY_BLOCKS=$cb step bench_cb${cb}_$RANDOM 240 python -u bench.py --steps 50 --warmup 5
done
step probe_dl 240 python -u scripts/probe_download.py
step ktrace 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline.md 2>&1
rm -rf /tmp/prof_k
