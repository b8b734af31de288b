#!/usr/bin/env bash
# Round-4 k: full GPU suite and smoke at this state; kernel trace and one PMC pass of the headline
# (count-only and emit); config 3 kernel trace (cooc).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread &&
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" &&
step ktrace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4k_ktrace_deep -o run -- python3 scripts/deep_probe.py --no-parity --reps 3 --supports 0.02 &&
step pmc_sq 200 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d /tmp/pmc_sq -o run -- python3 scripts/deep_probe.py --no-parity --reps 1 --supports 0.02 &&
f=$(find /tmp/pmc_sq -name "*counter_collection.csv" | head -1) && python3 scripts/summarize_pmc.py "$f" > gpurun_out/r4k_pmc_sq.md 2>&1 &&
step ktrace_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4k_ktrace_c3 -o run -- python3 scripts/cooc_probe.py --shape 10Mx1M --reps 2 --step --no-gemm
