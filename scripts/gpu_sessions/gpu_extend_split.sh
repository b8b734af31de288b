#!/usr/bin/env bash
# Split-K level-3+ extend kernels (long rows, few candidates): kernel suite, then 10M / 100M.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_kern 900 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 300 --timeout-method thread
step l10m 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 2
step l100m 600 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1
step ktrace100m 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_l -o run -- python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 2 --warmup 1
f=$(find /tmp/prof_l -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/l100m_kernel_stats.csv
rm -rf /tmp/prof_l
