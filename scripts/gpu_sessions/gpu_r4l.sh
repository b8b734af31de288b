#!/usr/bin/env bash
# Round-4 l: fused level path with the widened look-back (config 2 max_len 4), then the r4k
# validation (full GPU suite, smoke, traces, PMC).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step kernels_tests 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread &&
step config2 400 python -u bench.py --steps 3 --warmup 1 --serve-qps '' --no-levelwise --no-config3 --no-emit &&
python3 -c "import json; d=json.loads(open('gpurun_out/config2.log').read().strip().splitlines()[-1]); print(json.dumps(d.get('config2',{}).get('mine_max_len4')), d.get('errors'))" &&
bash scripts/gpu_sessions/gpu_r4k.sh
