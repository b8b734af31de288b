#!/usr/bin/env bash
# Round-2 t: wide-tile gram (4x4 MFMA tiles per wave, 256-row blocks), i8 and FP4: exactness, then
# A/B at the 100M x 754 and config-5 widths.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gram 900 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "pair_gram"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
step l100_base 600 $L100
KMLS_GRAM_TILE=256 step l100_wide_i8 600 $L100
KMLS_GRAM_TILE=256 KMLS_GRAM_FP4=1 step l100_wide_fp4 600 $L100
RM="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 10Mx1M"
step rm10_base 600 $RM
KMLS_GRAM_TILE=256 KMLS_GRAM_FP4=1 step rm10_wide_fp4 600 $RM
KMLS_GRAM_TILE=256 step rm10_wide_i8 600 $RM
