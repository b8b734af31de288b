#!/usr/bin/env bash
# Round-2 final check of the tree: full GPU suite, smoke(), the driver's bench line, the 2-rank
# weak-scaled rehearsal, 100M and config-5 (10M) large shapes, a 100M kernel trace.
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py --gpus 1 --steps 20 --warmup 5
KMLS_BENCH_DIST=gloo step bench_w2 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5
step l100 600 python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma
step rm10 600 python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 10Mx1M
step ktrace100 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt100 -o run -- python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 2 --warmup 1 --mfma
f=$(find /tmp/kt100 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/kt100_kernel_stats.csv; rm -rf /tmp/kt100
