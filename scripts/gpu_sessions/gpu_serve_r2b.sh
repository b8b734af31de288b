#!/usr/bin/env bash
# Round-2 serving with the GPU-owning matcher process (4 workers → 1 owner).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step owner_tests 300 python -u -m pytest tests/test_api.py -q -x -k owner --timeout 120 --timeout-method thread
for b in hip auto cpu; do
  step serve_owner_$b 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend $b --qps 2000,5000,10000,20000 --duration 5 --pvc /tmp/kmls_pvc --workers 4 --clients 4
done
KMLS_GPU_OWNER=0 step serve_noowner_hip 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend hip --qps 2000,5000,10000,20000 --duration 5 --pvc /tmp/kmls_pvc --workers 4 --clients 4
