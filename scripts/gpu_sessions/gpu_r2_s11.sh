#!/usr/bin/env bash
# Round-2 s11: encode block size (more waves per CU on the same LDS): tests, 100M and config-5 A/B.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_enc 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "encode or support"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
step l100_b512 600 $L100
KMLS_ENCODE_BLOCK=256 step l100_b256 600 $L100
KMLS_ENCODE_BLOCK=1024 step l100_b1024 600 $L100
RM10="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 10Mx1M"
step rm10_b1024 600 $RM10
KMLS_ENCODE_BLOCK=256 step rm10_b256 600 $RM10
KMLS_SUPPORT_GRID=1280 step l100_grid1280 600 $L100
KMLS_SUPPORT_GRID=2048 step l100_grid2048 600 $L100
