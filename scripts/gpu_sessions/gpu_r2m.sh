#!/usr/bin/env bash
# Round-2 m: support pass 3 check, bench.py N-rank rehearsal (gloo, ranks sharing the GPU),
# config-5 gram A/B (i8 LDS-staged vs FP4 block-scaled MFMA) at 10M x 1M, F ~ 14.8k.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_m 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "support or encode or txdp or large or pair_gram"
step l100 600 python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1
for n in 2 4; do
  KMLS_BENCH_DIST=gloo step bench_w$n 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 20 --warmup 3
done
RM="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 10Mx1M"
step rm10_i8 600 $RM
KMLS_GRAM_FP4=1 step rm10_fp4 600 $RM
