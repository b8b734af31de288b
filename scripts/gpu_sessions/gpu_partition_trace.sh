#!/usr/bin/env bash
# Kernel timelines of single ranks of the replicated mode (world 2): rank 0 vs rank 1.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
WORLD=${WORLD:-2}
for r in ${RANKS:-0 1}; do
  step ktrace_r$r 300 rocprofv3 --kernel-trace -d /tmp/prof_r$r -o run -- python3 scripts/probe_partition_rank.py $WORLD $r
  python3 scripts/rocpd_timeline.py /tmp/prof_r$r/run_results.db --marker k_prologue_init > gpurun_out/timeline_r$r.md 2>&1
  rm -rf /tmp/prof_r$r
done
