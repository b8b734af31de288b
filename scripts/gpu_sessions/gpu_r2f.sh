#!/usr/bin/env bash
# Round-2 f: one kernel per level (scan folded into the count's segmented look-back).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_fold 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -k "miner_matches_cpu or max_len or compact or repeat or rule_index or partition"
step pytest_all 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
B=(python3 bench.py --no-config2 --serve-qps "" --steps 50 --warmup 5)
step bench_fold 300 "${B[@]}"
step ktrace 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify --no-config2 --serve-qps ""
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline_fold.md 2>&1
rm -rf /tmp/prof_k
step partition 300 python3 scripts/partition_scaling.py
