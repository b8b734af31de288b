#!/usr/bin/env bash
# Round-3 c: deep-miner parity + 0.02 probe; native-front serving bench (auto and forced HIP).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=60
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
run pytest_deep 400 python -u -m pytest tests/test_gpu_deep.py -v -x --timeout 120 --timeout-method thread &&
run deep_probe 300 python -u scripts/deep_probe.py --supports 0.02 --reps 2 &&
run serve_auto 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend auto --qps 2000,5000,10000 --duration 4 --capacity --json-out gpurun_out/serve_auto.json &&
run serve_hip 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend hip --qps 2000,5000,10000 --duration 4 --capacity --json-out gpurun_out/serve_hip.json
