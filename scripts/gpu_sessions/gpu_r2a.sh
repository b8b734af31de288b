#!/usr/bin/env bash
# Round-2 first check: device rule map + digest tests, then the new headline bench.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_ruleidx 600 python -u -m pytest tests/test_gpu_kernels.py -v -x --timeout 120 --timeout-method thread -k "rule_index or matches_cpu"
step bench_default 900 python -u bench.py
step bench_noidx 240 python -u bench.py --no-rule-map --no-config2 --serve-qps "" --steps 50 --warmup 5
