#!/usr/bin/env bash
# Round-2 z: bench.py with the config-3 section (10M x 1M tx-DP) at 1 rank, then the N-rank
# rehearsal (gloo process group, ranks sharing the one GPU, host-staged communicator) at 2 and 4.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step bench_c3_n1 600 python3 bench.py --steps 10 --warmup 3 --serve-qps ""
KMLS_BENCH_DIST=gloo step bench_c3_n2 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 2 --steps 10 --warmup 3
KMLS_BENCH_DIST=gloo step bench_c3_n4 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29582 bench.py --gpus 4 --steps 10 --warmup 3
