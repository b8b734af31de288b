#!/usr/bin/env bash
# Round-2 w: encode item -> transaction LDS table (KMLS_ENCODE_OWNER) exactness + 100M A/B.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_encode 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "encode"
export KMLS_GRAM_TILE=256 KMLS_GRAM_FP4=1
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
KMLS_ENCODE_OWNER=0 step l100_own0 600 $L100
KMLS_ENCODE_OWNER=12288 step l100_own12k 600 $L100
KMLS_ENCODE_OWNER=16384 KMLS_ENCODE_TW=3 step l100_own16k_tw8 600 $L100
KMLS_ENCODE_OWNER=0 step l100_own0_b 600 $L100
