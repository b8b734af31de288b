#!/usr/bin/env bash
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step bench_deferred 240 python -u bench.py --steps 30 --warmup 5
KMLS_DL_MODE=inline step bench_inline 240 python -u bench.py --steps 30 --warmup 5
step probe_dl 240 python -u scripts/probe_download.py
step ktrace 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline.md 2>&1
rm -rf /tmp/prof_k
