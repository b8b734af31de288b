#!/usr/bin/env bash
# Round-3 g: in-launch work stealing for the deep miner: GPU parity (new waiting loops first,
# bounded), steal vs rounds sweep at ds1 @0.02, 8-rank split simulation, then the full GPU suite,
# smoke and the shipped bench.py.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=30
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py"
run deep_tests 400 python -u -m pytest tests/test_gpu_deep.py -v -x --timeout 120 --timeout-method thread &&
run sweep 500 $P --reps 3 --supports 0.02 --sweep 1024:1024:8:3:0,0:1024:8:3:1:1,0:256:8:3:1:1,0:64:8:3:1:1,0:256:8:3:1:16,0:256:4:3:1:1,0:256:16:3:1:1 &&
run world8 300 $P --no-parity --reps 1 --supports 0.02 --world 8 --budget 256 &&
run world8_rounds 300 $P --no-parity --reps 1 --supports 0.02 --world 8 --rounds --budget 1024 --budget0 1024 &&
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" &&
step bench 900 python -u bench.py --steps 10 --warmup 2
