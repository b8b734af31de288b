#!/usr/bin/env bash
# Round-2 s8: multi-band encode for wide frequent sets (tests, config 5 rule map at 10M and 100M
# with and without it).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_enc 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "encode or gram"
RM10="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 10Mx1M"
step rm10_mb 600 $RM10
KMLS_ENCODE_MULTIBAND=0 step rm10_nomb 600 $RM10
step rm100_mb 900 python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 100Mx1M
