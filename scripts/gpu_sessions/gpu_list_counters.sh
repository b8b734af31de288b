#!/usr/bin/env bash
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
grep -iE "MFMA|SQ_BUSY|SQ_WAVE|VALU|TCC_HIT|TCC_MISS|FETCH_SIZE|WRITE_SIZE|GRBM_GUI|LDS_BANK|SQ_INSTS_LDS" gpurun_out/counters_list.txt | head -80 > gpurun_out/counters_filtered.txt || true
