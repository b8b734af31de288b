#!/usr/bin/env bash
# Round-2 q: one-gather encode tables (group mask + prefix, LDS compact→rank).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_q 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dist.py -q -x --timeout 300 --timeout-method thread -k "encode or txdp or large or dist or tx"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1"
step l100_grp 600 $L100
KMLS_ENCODE_GROUP=0 step l100_nogrp 600 $L100
