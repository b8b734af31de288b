#!/usr/bin/env bash
# LDS-staged MFMA gram (KMLS_GRAM_LDS=1): exactness tests, then same-box A/B at 10M and 100M.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gram 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 300 --timeout-method thread -k "pair_gram"
step l10m_direct 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 2
KMLS_GRAM_LDS=1 step l10m_lds 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 2
step l100m_direct 600 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1
KMLS_GRAM_LDS=1 step l100m_lds 600 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1
