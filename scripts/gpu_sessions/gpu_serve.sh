#!/usr/bin/env bash
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
P=/tmp/kmls_pvc_box
step serve_matcher 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --matcher-only --pvc $P
step serve_hip 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend hip --qps 2000,5000,10000 --duration 8 --workers 6 --clients 6 --pvc $P
step serve_cpu 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend cpu --qps 2000,5000,10000 --duration 8 --workers 6 --clients 6 --pvc $P
step serve_python 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend python --qps 2000,5000,10000 --duration 8 --workers 6 --clients 6 --pvc $P
