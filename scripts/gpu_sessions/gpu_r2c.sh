#!/usr/bin/env bash
# Round-2: rule-map fork/join check + headline A/B + per-step kernel timeline.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_ri 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -k "rule_index or max_len"
step bench_idx 300 python -u bench.py --no-config2 --serve-qps "" --steps 50 --warmup 5
step bench_noidx 300 python -u bench.py --no-rule-map --no-config2 --serve-qps "" --steps 50 --warmup 5
step ktrace 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify --no-config2 --serve-qps ""
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline.md 2>&1
rm -rf /tmp/prof_k
