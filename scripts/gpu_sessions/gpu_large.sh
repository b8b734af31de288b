#!/usr/bin/env bash
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gram 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 300 --timeout-method thread -k "gram or split_k or txdp or miner_matches"
step large10m 400 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 5 --warmup 2
step large100m 600 python -u -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1
PMC_CMD="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 10Mx1M --steps 1 --warmup 0"
step pmc_gram 200 timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc_g -o run -- $PMC_CMD
f=$(find /tmp/pmc_g -name "*counter_collection.csv" | head -1); [ -n "$f" ] && python3 scripts/summarize_pmc.py "$f" > gpurun_out/pmc_gram.md 2>&1; rm -rf /tmp/pmc_g
