#!/usr/bin/env bash
# Round-2 s2: support/encode kernel tests, 100M support with the scatter prefetch, a 100M
# kernel trace, serve 10k QPS with more client processes / workers.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_sup 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "support or encode"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
step l100_prefetch 600 $L100
step ktrace100 600 rocprofv3 --kernel-trace --stats -d /tmp/kt100 -o run -- python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 2 --warmup 1 --mfma
cp /tmp/kt100/*kernel_stats.csv gpurun_out/kt100_kernel_stats.csv 2>/dev/null; rm -rf /tmp/kt100
S="python3 -m kubernetes_machine_learning_server_amd.bench.bench_serve --qps 5000,10000 --duration 3"
step serve_auto_w4c4 300 $S --backend auto --workers 4 --clients 4
step serve_auto_w4c8 300 $S --backend auto --workers 4 --clients 8
step serve_auto_w8c8 300 $S --backend auto --workers 8 --clients 8
step serve_cpu_w4c8 300 $S --backend cpu --workers 4 --clients 8
