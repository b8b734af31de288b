#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 800 python -u -m pytest tests -m gpu -q -x --timeout 300
step bench 240 python -u bench.py --steps 30 --warmup 5
step large100m 600 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --min-support 0.001 --steps 3 --warmup 1 --rules
step rocprof_large 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11 -o run --output-format csv -- python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --min-support 0.001 --steps 2 --warmup 1
