#!/usr/bin/env bash
# Round-2 s3: encode LDS lookup tables (tests + 100M A/B vs the group gather), 100M kernel trace.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_enc 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "support or encode"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
step l100_lookup 600 $L100
KMLS_ENCODE_LOOKUP=group step l100_group 600 $L100
step ktrace100 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt100 -o run -- python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 2 --warmup 1 --mfma
f=$(find /tmp/kt100 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/kt100_kernel_stats.csv; rm -rf /tmp/kt100
