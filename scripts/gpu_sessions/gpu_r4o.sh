#!/usr/bin/env bash
# Round-4 o: the 8-rank split of the headline (simulated rank by rank on one GPU) across the
# stealing launch's mailbox-check interval (budget), with per-wave traces; world 1 at budget 2.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
for b in 1 2 4 8; do
  step r4o_w8_budget$b 200 python3 -u scripts/deep_probe.py --world 8 --supports 0.02 --no-parity --reps 2 --budget $b --trace
done
step r4o_w1_budget2 200 python3 -u scripts/deep_probe.py --world 1 --supports 0.02 --no-parity --reps 3 --budget 2
