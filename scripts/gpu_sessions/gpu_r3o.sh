#!/usr/bin/env bash
# Round-3 o: deep batch-step decode tables + cheaper digest: parity, budget sweep, 8-rank split,
# one PMC pass (instruction mix).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_DEEP_ROUND_TIMEOUT_S=30
run() { step "$@"; local rc=$(tail -n1 gpurun_out/steps.log | sed 's/.*rc=//'); [ "$rc" = "0" ]; }
P="python -u scripts/deep_probe.py"
run deep_tests 400 python -u -m pytest tests/test_gpu_deep.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "deep or digest or trie" &&
run sweep 300 $P --reps 3 --supports 0.02 --sweep 0:128:8:3:1:1,0:256:8:3:1:1,0:512:8:3:1:1,0:256:8:4:1:1 &&
run world8 200 $P --no-parity --reps 1 --supports 0.02 --world 8 &&
run pmc_sq 200 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d /tmp/pmc_sq -o run -- python3 scripts/deep_probe.py --no-parity --reps 1 --supports 0.02 &&
f=$(find /tmp/pmc_sq -name "*counter_collection.csv" | head -1) && python3 scripts/summarize_pmc.py "$f" > gpurun_out/pmc_sq.md 2>&1
