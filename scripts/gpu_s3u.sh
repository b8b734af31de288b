#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_sup 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 300 --timeout-method thread -k "support or split_k or txdp"
step large10m 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 2
KMLS_SUPPORT_PARTITIONED=0 step large10m_hash 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 2
step large100m 600 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1
