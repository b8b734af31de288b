#!/usr/bin/env bash
# Address-translation and L2 read-latency counters of the large shapes (gram / encode kernels).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
pmc() {  # pmc <name> <counters...>
  local name=$1; shift
  step pmc_$name 300 timeout -s KILL 280 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$name -o run -- $PMC_CMD
  f=$(find /tmp/pmc_$name -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 scripts/summarize_pmc.py "$f" > gpurun_out/pmc_$name.md 2>&1
  rm -rf /tmp/pmc_$name
}
PMC_CMD="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 1 --warmup 0"
pmc tlb10m TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum
PMC_CMD="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 1 --warmup 0"
pmc tlb100m TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum
