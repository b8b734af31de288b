#!/usr/bin/env bash
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step bench_spin 240 python -u bench.py --steps 50 --warmup 5
KMLS_SPIN_SYNC=0 step bench_block 240 python -u bench.py --steps 50 --warmup 5
step bench_spin2 240 python -u bench.py --steps 50 --warmup 5
step hiptrace 300 rocprofv3 --kernel-trace --hip-trace -d /tmp/prof_s3b -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify
python3 scripts/rocpd_timeline.py /tmp/prof_s3b/run_results.db --api > gpurun_out/hiptrace_timeline.md 2>&1
rm -rf /tmp/prof_s3b
