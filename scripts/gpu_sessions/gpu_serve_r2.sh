#!/usr/bin/env bash
# Round-2 serving: kernel parity, matcher-only crossover, HTTP p50/p99 per backend.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_serve 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k serve --timeout 120 --timeout-method thread
step matcher 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --matcher-only --pvc /tmp/kmls_pvc
for b in cpu auto hip python; do
  step serve_$b 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend $b --qps 2000,5000,10000 --duration 5 --pvc /tmp/kmls_pvc --workers 4 --clients 4
done
