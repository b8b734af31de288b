#!/usr/bin/env bash
# Tiled (LDS-slab) encode: exactness tests, then the large shapes with / without it.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_enc 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 300 --timeout-method thread -k "encode or pair_gram or txdp or miner_matches"
for t in 1 0; do
  KMLS_ENCODE_TILED=$t step l10m_enc$t 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 2
done
KMLS_ENCODE_TILED=1 step l100m_enc1 600 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1
