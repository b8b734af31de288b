#!/usr/bin/env bash
# Round-2 s12: headline steady-state timeline (kernel trace of the bench loop, rocpd database).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step trace_bench 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 30 --warmup 3 --no-verify --no-config2 --no-config3 --serve-qps ""
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline_s12.md 2>&1
cp /tmp/prof_k/run_results.db gpurun_out/tb_results.db 2>/dev/null
rm -rf /tmp/prof_k
