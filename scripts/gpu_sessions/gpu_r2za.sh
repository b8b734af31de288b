#!/usr/bin/env bash
# Round-2 za: masked-nibble FP4 as the default MFMA gram (whole kernel test file), then the bench
# with the config-3 section at 1, 2 and 4 ranks (scripts/gpu_r2z.sh).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_kernels 900 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread
bash "$(dirname "$0")/gpu_r2z.sh"
