#!/usr/bin/env bash
# Round-2 s: serving at 10k QPS — bench.py's serve section vs the standalone serve bench (auto / cpu).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step bench_serve_in_bench 400 python3 bench.py --steps 5 --warmup 2
step serve_auto_a 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend auto --qps 2000,5000,10000 --duration 3 --pvc /tmp/kmls_pvc --workers 4 --clients 4
step serve_cpu 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend cpu --qps 2000,5000,10000 --duration 3 --pvc /tmp/kmls_pvc --workers 4 --clients 4
step serve_auto_b 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend auto --qps 2000,5000,10000 --duration 3 --pvc /tmp/kmls_pvc --workers 4 --clients 4
