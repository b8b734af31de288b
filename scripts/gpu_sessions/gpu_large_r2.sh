#!/usr/bin/env bash
# Round-2 large shapes: support/encode A/B at 100M, per-kernel stats, PMC passes (10M).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_sup 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "support_histograms or encode_tiled or serve"
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1"
step l100_default 600 $L100
KMLS_SUPPORT_MODE=atomic step l100_atomic 600 $L100
KMLS_ENCODE_MODE=mp step l100_mp 600 $L100
step ktrace100 600 rocprofv3 --kernel-trace --stats -d /tmp/kt100 -o run -- python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 2 --warmup 1
cp /tmp/kt100/*kernel_stats.csv gpurun_out/kt100_kernel_stats.csv 2>/dev/null; rm -rf /tmp/kt100
L10="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 1 --warmup 0"
pmc() {  # pmc <name> <counters...>
  local name=$1; shift
  step pmc_$name 200 timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$name -o run -- $L10
  f=$(find /tmp/pmc_$name -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 scripts/summarize_pmc.py "$f" > gpurun_out/pmc_$name.md 2>&1
  rm -rf /tmp/pmc_$name
}
pmc sq SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE
pmc fetch FETCH_SIZE TCC_EA0_WRREQ_sum
pmc write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
export KMLS_LEVEL_TRACE_FILE=/tmp/level_trace.bin
KMLS_LEVEL_TRACE=2 step trace2 200 python -u scripts/probe_level_trace.py
KMLS_LEVEL_TRACE=4 step trace4 200 python -u scripts/probe_level_trace.py
KMLS_LEVEL_TRACE=7 step trace7 200 python -u scripts/probe_level_trace.py
