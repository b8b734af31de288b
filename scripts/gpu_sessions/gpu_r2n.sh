#!/usr/bin/env bash
# Round-2 n: LDS-staged FP4 gram (exactness, then A/B against i8 at configs 3 and 5 widths).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gram 900 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "pair_gram"
RM="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 10Mx1M"
step rm10_i8 600 $RM
KMLS_GRAM_FP4=1 step rm10_fp4lds 600 $RM
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
step l100_i8 600 $L100
KMLS_GRAM_FP4=1 step l100_fp4lds 600 $L100
