#!/usr/bin/env bash
# Round-2 s6: encode A/B at 100M: items per thread (8 / 16), tile width (TW 2 / 4 / 8).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_enc 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "encode"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
step l100_u8 600 $L100
KMLS_ENCODE_U=16 step l100_u16 600 $L100
KMLS_ENCODE_TW=1 step l100_tw2 600 $L100
KMLS_ENCODE_TW=3 step l100_tw8 600 $L100
