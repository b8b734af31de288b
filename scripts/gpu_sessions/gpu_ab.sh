#!/usr/bin/env bash
# Generic A/B of the headline bench under environment switches: gpu_ab.sh "ENV=..." "ENV=..." ...
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
i=0
for spec in "$@"; do
  i=$((i+1))
  step ab_$i 240 env $spec python -u bench.py --steps 50 --warmup 5
  echo "$spec" >> gpurun_out/ab_$i.log
done
