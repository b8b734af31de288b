#!/usr/bin/env bash
# Round-3 l: serving HIP-vs-C++ crossover evidence (matcher micro-bench, forced HIP, auto at
# high offered load) and config 3 at a support with >10k frequent items (tx-DP, 1 GPU).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
S="-m kubernetes_machine_learning_server_amd.bench.bench_serve"
step matcher 300 python -u $S --matcher-only &&
step serve_hip 400 python -u $S --backend hip --qps 2000,10000,50000 --duration 3 --capacity &&
step serve_auto_hi 400 python -u $S --backend auto --qps 10000,100000,200000,300000 --duration 3 &&
step c3_2e4 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --min-support 0.0002 --mode tx --steps 2 --warmup 1
