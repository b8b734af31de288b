#!/usr/bin/env bash
# Round-2 j: final fold state — GPU suite, headline, timeline, traces, partition predictor.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_all 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step bench_full 600 python3 bench.py
step ktrace 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify --no-config2 --serve-qps ""
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline_fold.md 2>&1
rm -rf /tmp/prof_k
export KMLS_LEVEL_TRACE_FILE=/tmp/level_trace.bin
KMLS_LEVEL_TRACE=2 step trace2 200 python -u scripts/probe_level_trace.py
KMLS_LEVEL_TRACE=4 step trace4 200 python -u scripts/probe_level_trace.py
KMLS_LEVEL_TRACE=7 step trace7 200 python -u scripts/probe_level_trace.py
step partition 300 python3 scripts/partition_scaling.py
