#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 500 python -u -m pytest tests -m gpu -q -x --timeout 120
step bench 240 python -u bench.py --steps 30 --warmup 5
step bench_mfma 240 python -u bench.py --steps 30 --warmup 5 --mfma
step rocprof 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3
step serve_hip 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend hip --qps 2000,10000 --duration 8 --workers 6 --clients 6 --pvc /tmp/kmls_pvc_box
