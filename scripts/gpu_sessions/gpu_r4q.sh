#!/usr/bin/env bash
# Round-4 q: the last config-2 full-count ranks; the cooc scan with 4 rows in flight (tests,
# config-3 step, config-5 shape count).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
KMLS_DEEP_ROUND_TIMEOUT_S=300 step fc_b4 400 python3 -u scripts/full_count.py --world 256 --ranks 248-255 --out gpurun_out/fc_b4.jsonl
step r4q_cooc_tests 300 python -u -m pytest tests/test_gpu_cooc.py -x -q --timeout 200 --timeout-method thread
step r4q_cooc_c3 300 python3 -u scripts/cooc_probe.py --shape 10Mx1M --reps 3 --step --no-gemm
step r4q_cooc_c5 400 python3 -u scripts/cooc_probe.py --shape 100Mx1M --reps 2 --no-gemm
# the level-3 task order sorted and dealt on the device (deep_order.hip)
step r4q_deep_tests 300 python -u -m pytest tests/test_gpu_deep.py -x -q --timeout 200 --timeout-method thread
step r4q_w1 200 python3 -u scripts/deep_probe.py --supports 0.02 --reps 5
step r4q_w8 200 python3 -u scripts/deep_probe.py --world 8 --supports 0.02 --no-parity --reps 2
