#!/usr/bin/env bash
# Round-3 g: in-launch work stealing for the deep miner: GPU parity (new waiting loops first,
# bounded), steal vs rounds sweep at ds1 @0.02, 8-rank split simulation; the multi-rank rule map
# (config 5) tests and a 10M x 1M rehearsal at world 1 / 2 (two ranks sharing the GPU); bench.py.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=30
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py"
RM="-m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --shape 10Mx1M --min-support 0.0002 --steps 2 --warmup 1"
run deep_tests 400 python -u -m pytest tests/test_gpu_deep.py -v -x --timeout 120 --timeout-method thread &&
run sweep 400 $P --reps 3 --supports 0.02 --sweep 1024:1024:8:3:0,0:1024:8:3:1:1,0:256:8:3:1:1,0:64:8:3:1:1,0:256:8:3:1:16,0:256:4:3:1:1,0:256:16:3:1:1 &&
run world8 200 $P --no-parity --reps 1 --supports 0.02 --world 8 --budget 256 &&
run world8_rounds 200 $P --no-parity --reps 1 --supports 0.02 --world 8 --rounds --budget 1024 --budget0 1024 &&
run rm_tests 300 python -u -m pytest tests/test_rule_map_dist.py -v -x -m gpu --timeout 280 --timeout-method thread &&
run rm10_w1 300 python -u $RM &&
KMLS_BENCH_DIST=gloo run rm10_w2 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 $RM &&
step bench 600 python -u bench.py --steps 10 --warmup 2
