#!/usr/bin/env bash
# Round-2 s15: interleaved repeats of the headline with and without the opt-in graph scheduling
# (twin execs + late rule-map nodes), 100 timed steps each.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
B="python3 bench.py --steps 100 --warmup 10 --no-config2 --no-config3 --no-verify --serve-qps "
for i in 1 2 3 4; do
  step old_$i 120 $B ""
  KMLS_GRAPH_TWIN=1 KMLS_RULEMAP_LATE=1 step new_$i 120 $B ""
  KMLS_RULEMAP_LATE=1 step late_$i 120 $B ""
done
