#!/usr/bin/env bash
# Round-2 re-entry check of HEAD: full GPU suite, smoke(), the driver's default bench line, the
# weak-scaled N-rank bench rehearsed at 2 ranks on one GPU (gloo bracket), encode tx-map A/B.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py --gpus 1 --steps 20 --warmup 5
KMLS_BENCH_DIST=gloo step bench_w2 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-config3
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
step l100_txmap 600 $L100
KMLS_ENCODE_TXMAP=0 step l100_bsearch 600 $L100
KMLS_SUPPORT_COUNT=part step l100_count_part 600 $L100
KMLS_SUPPORT_COUNT=balnd step l100_count_balnd 600 $L100
