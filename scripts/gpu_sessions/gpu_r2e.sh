#!/usr/bin/env bash
# Round-2 e: long-merge serve kernel, LDS-hash encode, config-5 rule map (10M, 100M), encode A/B.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_e 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "serve or encode_tiled or rule_map or dist_miner or txdp"
step pytest_dist 300 python -u -m pytest tests/test_gpu_dist.py -q -x --timeout 120 --timeout-method thread
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1"
step l100_mask 600 $L100
RM="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1"
step rm10 600 $RM --shape 10Mx1M
step rm100 900 $RM --shape 100Mx1M
