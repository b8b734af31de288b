#!/usr/bin/env bash
# Round-2 v: software-pipelined FP4 wide-tile gram (unpack word s+1 before word s's MFMAs).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gram_wide 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "pair_gram and wide"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
KMLS_GRAM_TILE=256 KMLS_GRAM_FP4=1 step l100_wide_fp4p 600 $L100
RM="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 10Mx1M"
KMLS_GRAM_TILE=256 KMLS_GRAM_FP4=1 step rm10_wide_fp4p 600 $RM
pmc() {  # pmc <name> <counters...>: one counter pass, its own run, no tracing domains
  local name=$1; shift
  step pmc_$name 240 timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$name -o run -- $PMC_CMD
  f=$(find /tmp/pmc_$name -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 scripts/summarize_pmc.py "$f" > gpurun_out/pmc_$name.md 2>&1
  rm -rf /tmp/pmc_$name
}
export KMLS_GRAM_TILE=256 KMLS_GRAM_FP4=1
PMC_CMD="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 1 --warmup 0 --mfma"
pmc l100_wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE
pmc l100_mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE
pmc l100_tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
