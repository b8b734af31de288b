#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step first_call 200 python -u scripts/probe_first_call.py
step bench 240 python -u bench.py --steps 50 --warmup 5
step large10m 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 2
step large100m 600 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --rules
