#!/usr/bin/env bash
# Round-2 p: encode with next-round prefetch (TW 4, XCD order) at 100M.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_enc 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "encode"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1"
step l100_pf 600 $L100
