#!/usr/bin/env bash
# Level-2 gram kernel A/B on the large shapes: i8 MFMA (default for long rows) vs FP4 MFMA vs
# the VALU popcount bit-GEMM.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
for v in "KMLS_GRAM_POPCOUNT=1" "KMLS_GRAM_FP4=0" "KMLS_GRAM_FP4=1"; do
  tag=$(echo $v | tr -c 'A-Za-z0-9\n' '_')
  env $v python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 2 > gpurun_out/g10m_$tag.log 2>&1 || exit 1
done
env KMLS_GRAM_POPCOUNT=1 timeout -k 10 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 > gpurun_out/g100m_pop.log 2>&1
