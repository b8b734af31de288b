#!/usr/bin/env bash
# Round-4 w: item-shard compaction in gather form (tests + config-3 shard step), world-1 mailbox
# interval sweep, then the full GPU suite, smoke and the full bench at this state.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step r4w_shard_tests 400 python -u -m pytest tests/test_item_shard.py -x -q -m gpu --timeout 200 --timeout-method thread
step r4w_c3_shard 500 python -u scripts/c3_shard.py --mode shard --steps 3 --warmup 1 --batch-div 2,4
step r4w_w1_budget 200 python3 -u scripts/deep_probe.py --supports 0.02 --reps 3 --no-parity --sweep 0:4:0:0,0:8:0:0,0:16:0:0,0:32:0:0
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step r4w_bench 900 python -u bench.py --steps 20 --warmup 5
