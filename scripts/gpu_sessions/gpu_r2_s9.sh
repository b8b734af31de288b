#!/usr/bin/env bash
# Round-2 s9: masked FP4 gram with 16-word stripes (tests, 100M and config-5 10M A/B).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gram 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "mask16"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
step l100_mask 600 $L100
KMLS_GRAM_FP4=mask16 step l100_mask16 600 $L100
RM10="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 10Mx1M"
step rm10_mask 600 $RM10
KMLS_GRAM_FP4=mask16 step rm10_mask16 600 $RM10
KMLS_SUPPORT_TILES=4 step l100_tiles4 600 $L100
