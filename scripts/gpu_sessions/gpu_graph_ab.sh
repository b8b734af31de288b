#!/usr/bin/env bash
# Graph replay vs eager launches on one box: kernel timelines for both, then alternating benches.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
for g in 1 0; do
  export KMLS_GRAPH=$g
  step ktrace_g$g 300 rocprofv3 --kernel-trace -d /tmp/prof_g$g -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify
  python3 scripts/rocpd_timeline.py /tmp/prof_g$g/run_results.db > gpurun_out/ktrace_g$g.md 2>&1
  rm -rf /tmp/prof_g$g
done
for g in 1 0 1 0; do
  export KMLS_GRAPH=$g
  step bench_g${g}_$RANDOM 240 python -u bench.py --steps 50 --warmup 5
done
