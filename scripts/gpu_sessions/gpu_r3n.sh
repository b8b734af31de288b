#!/usr/bin/env bash
# Round-3 n: the N-rank bench path rehearsed with 2 ranks sharing the GPU (gloo + host comm),
# and config 5 (100M x 1M @2e-4, 185 GB of bitmaps) through DistRuleMap at world 1 and world 2.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
TR="python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1"
RM="-m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --shape 100Mx1M --min-support 0.0002 --steps 2 --warmup 1"
KMLS_BENCH_DIST=gloo step bench_w2 600 $TR --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 1 --serve-qps "" &&
step c5_w1 500 python -u $RM &&
KMLS_BENCH_DIST=gloo step c5_w2 700 $TR --master-port 29542 $RM
