#!/usr/bin/env bash
# Round-2 s7: wide gram with the 2-D XCD-aware remap (tests, 100M A/B, L2 hit counters at 10M).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gram 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "gram"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
step l100_x1d 600 $L100
KMLS_GRAM_XCD=2d step l100_x2d 600 $L100
L10="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 1 --warmup 0 --mfma"
pmc() {  # pmc <name> <counters...>
  local name=$1; shift
  step pmc_$name 200 timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$name -o run -- $L10
  f=$(find /tmp/pmc_$name -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 scripts/summarize_pmc.py "$f" > gpurun_out/pmc_$name.md 2>&1
  rm -rf /tmp/pmc_$name
}
pmc l2_1d TCC_HIT_sum TCC_MISS_sum
KMLS_GRAM_XCD=2d pmc l2_2d TCC_HIT_sum TCC_MISS_sum
