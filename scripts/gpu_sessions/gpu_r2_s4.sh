#!/usr/bin/env bash
# Round-2 s4: survivor-driven materialize (full GPU suite, 100M A/B vs the candidate-driven grid,
# kernel trace), 10M config-3 shape.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
step l100_surv 600 $L100
KMLS_MATERIALIZE=cand step l100_cand 600 $L100
step ktrace100 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt100 -o run -- python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 2 --warmup 1 --mfma
f=$(find /tmp/kt100 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/kt100_kernel_stats.csv; rm -rf /tmp/kt100
step l10 600 python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 1 --mfma
