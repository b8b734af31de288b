#!/usr/bin/env bash
# Round-2 zb: masked FP4 gram with 2 waves per SIMD (KMLS_GRAM_FP4=mask8) vs the 1-wave default.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_mask8 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "pair_gram and mask8"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
KMLS_GRAM_FP4=mask8 step l100_mask8 600 $L100
step l100_mask 600 $L100
RM="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 10Mx1M"
KMLS_GRAM_FP4=mask8 step rm10_mask8 600 $RM
step rm10_mask 600 $RM
step rm100_mask 900 python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 100Mx1M
