#!/usr/bin/env bash
# FP4 (e2m1 block-scaled MFMA) gram vs the i8 MFMA gram: exactness tests, then large-shape A/B.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gram 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 300 --timeout-method thread -k "pair_gram"
for f in 0 1; do
  KMLS_GRAM_FP4=$f step large10m_fp4$f 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 2
done
for f in 1 0; do
  KMLS_GRAM_FP4=$f step large100m_fp4$f 600 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1
done
