#!/usr/bin/env bash
# Round-3 x: item-sharded bitmaps — GPU tests (kernel vs numpy, shard mining world 1 and 2 ranks
# sharing the GPU), config 3 in shard mode at world 1 and 2 (gloo) against tx mode; then the
# full GPU suite on the final deep-miner defaults.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29533"
run shard_tests 300 python -u -m pytest tests/test_item_shard.py -x -q -m gpu --timeout 200 --timeout-method thread &&
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread &&
run c3_shard_w1 400 python -u scripts/c3_shard.py --mode shard --steps 1 --warmup 1 &&
KMLS_BENCH_DIST=gloo step c3_shard_w2 400 $TR --nproc-per-node 2 scripts/c3_shard.py --mode shard --steps 1 --warmup 1
