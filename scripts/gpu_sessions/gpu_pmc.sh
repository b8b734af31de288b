#!/usr/bin/env bash
# PMC counter passes (each its own run, counters only, no tracing domains).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
L="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 1 --warmup 0"
pmc() {  # pmc <name> <counters...>
  local name=$1; shift
  step pmc_$name 200 timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$name -o run -- $PMC_CMD
  f=$(find /tmp/pmc_$name -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 scripts/summarize_pmc.py "$f" > gpurun_out/pmc_$name.md 2>&1
  rm -rf /tmp/pmc_$name
}
PMC_CMD="$L"
pmc large_sq SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE
pmc large_tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
PMC_CMD="python3 bench.py --steps 3 --warmup 1 --no-verify"
pmc ds1_sq SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
pmc ds1_tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
