#!/usr/bin/env bash
# Round-4 p: deep kernel with the 8 KB/wave LDS tables — 3 vs 4 workgroups per CU (the 4-wave/SIMD
# instance at 128 VGPRs), parity first; deep GPU tests; the 8-rank split across mailbox intervals.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step r4p_w1_bpc3 200 python3 -u scripts/deep_probe.py --supports 0.02 --reps 5 --blocks-per-cu 3
step r4p_w1_bpc4 200 python3 -u scripts/deep_probe.py --supports 0.02 --reps 5 --blocks-per-cu 4
step r4p_deep_tests 300 python -u -m pytest tests/test_gpu_deep.py -x -q --timeout 200 --timeout-method thread
for b in 2 8; do
  for bpc in 3 4; do
    step r4p_w8_b${b}_bpc$bpc 200 python3 -u scripts/deep_probe.py --world 8 --supports 0.02 --no-parity --reps 2 --budget $b --blocks-per-cu $bpc --trace
  done
done
