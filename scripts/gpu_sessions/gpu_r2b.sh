#!/usr/bin/env bash
# Round-2: full GPU suite, then the new headline bench (+config2 +serve) and an A/B without the rule map.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -x --timeout 120 --timeout-method thread
step bench_default 900 python -u bench.py
step bench_noidx 240 python -u bench.py --no-rule-map --no-config2 --serve-qps "" --steps 50 --warmup 5
