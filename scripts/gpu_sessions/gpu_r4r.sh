#!/usr/bin/env bash
# Round-4 r: full GPU suite, smoke, the full bench at this state, headline kernel trace + one SQ
# PMC pass (4 waves/SIMD deep kernel), config-5 rule-map step (cooc scan).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step r4r_bench 900 python -u bench.py --steps 20 --warmup 5
step r4r_ktrace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4r_ktrace_deep -o run -- python3 scripts/deep_probe.py --no-parity --reps 3 --supports 0.02
step r4r_pmc 200 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d /tmp/pmc_sq -o run -- python3 scripts/deep_probe.py --no-parity --reps 1 --supports 0.02
f=$(find /tmp/pmc_sq -name "*counter_collection.csv" | head -1) && python3 scripts/summarize_pmc.py "$f" > gpurun_out/r4r_pmc_sq.md 2>&1
step r4r_config5 600 python3 -u -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 2 --warmup 1 --shape 100Mx1M
