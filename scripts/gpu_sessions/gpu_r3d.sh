#!/usr/bin/env bash
# Round-3 d: deep-miner tuning sweep (budget / split / occupancy), 8-rank split simulation,
# kernel-trace stats + PMC passes on the 0.02 run, and the new level / e2e GPU tests.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=60
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py"
SW=1024:1024:4:3,4096:1024:4:3,1024:1024:4:2,1024:1024:4:4,1024:1024:2:3,1024:1024:8:3,16384:1024:4:3,2048:2048:4:3
pmc() {  # pmc <name> <counters...>
  local name=$1; shift
  run pmc_$name 200 timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$name -o run -- python3 scripts/deep_probe.py --no-parity --reps 1 --supports 0.02 &&
  f=$(find /tmp/pmc_$name -name "*counter_collection.csv" | head -1) && python3 scripts/summarize_pmc.py "$f" > gpurun_out/pmc_$name.md 2>&1; rm -rf /tmp/pmc_$name; true
}
run sweep 400 $P --no-parity --reps 2 --supports 0.02 --sweep $SW &&
run world8 300 $P --no-parity --reps 1 --supports 0.02 --world 8 --budget 1024 --budget0 1024 &&
run bench 600 python -u bench.py --steps 5 --warmup 1 &&
run tests_new 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py::test_level_candidate_total_past_2_28_falls_back tests/test_gpu_e2e.py &&
run ktrace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace_deep -o run -- python3 scripts/deep_probe.py --no-parity --reps 1 --supports 0.02 &&
pmc sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU &&
pmc lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE &&
pmc fetch FETCH_SIZE TCC_HIT_sum &&
pmc write WRITE_SIZE TCC_MISS_sum
