#!/usr/bin/env bash
# Same-box A/B: the previous build (ab_old/, not tracked) vs the working tree.
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  step old_$i 240 python -u ab_old/bench.py --steps 50 --warmup 5 --no-verify
  step new_$i 240 python -u bench.py --steps 50 --warmup 5 --no-verify
  KMLS_COPY_BLOCKS=32 step new32_$i 240 python -u bench.py --steps 50 --warmup 5 --no-verify
done
