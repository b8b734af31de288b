#!/usr/bin/env bash
# Round-2 l: support pass 1 vectorised/per-wave bins, encode 16 items per thread; 100M timing.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_l 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "support or encode or txdp or large"
step l100 600 python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step kt100 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt100 -o run -- python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 2 --warmup 1
f=$(find /tmp/kt100 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/kt100_kernel_stats.csv
rm -rf /tmp/kt100
