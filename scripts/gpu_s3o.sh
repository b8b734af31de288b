#!/usr/bin/env bash
# Large-shape (BASELINE configs 3/5) kernel profile on one GPU.
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step large10m 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 2
step ktrace10m 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_l -o run --output-format csv -- python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 3 --warmup 1
python3 scripts/summarize_rocprof.py /tmp/prof_l/run_kernel_stats.csv 4 > gpurun_out/large10m_kernel_stats.md 2>&1 || find /tmp/prof_l -name "*.csv" > gpurun_out/large10m_files.txt
rm -rf /tmp/prof_l
