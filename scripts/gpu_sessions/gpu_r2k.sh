#!/usr/bin/env bash
# Round-2 k: per-kernel times of the 100M x 1M mining call (support passes, encode, gram).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step kt100 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt100 -o run -- python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 2 --warmup 1
f=$(find /tmp/kt100 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/kt100_kernel_stats.csv
rm -rf /tmp/kt100
