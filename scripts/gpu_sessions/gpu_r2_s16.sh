#!/usr/bin/env bash
# Round-2 s16: PMC of the final tree's large-shape kernels at 10M (wave occupancy / wait share of
# the 512-thread encode, L2 traffic), one counter group per pass.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
L10="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 1 --warmup 0 --mfma"
pmc() {  # pmc <name> <counters...>
  local name=$1; shift
  step pmc_$name 200 timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$name -o run -- $L10
  f=$(find /tmp/pmc_$name -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 scripts/summarize_pmc.py "$f" > gpurun_out/pmc_$name.md 2>&1
  rm -rf /tmp/pmc_$name
}
pmc wave SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
pmc mem TCC_HIT_sum TCC_MISS_sum
