#!/usr/bin/env bash
# HIP API trace (no counters) of the headline bench: where the host time between steps goes.
# The trace DB is too large to copy back: summarise it on the box and delete it.
source "$(dirname "$0")/gpu_round.sh"
export PYTHONUNBUFFERED=1
step hiptrace 300 rocprofv3 --kernel-trace --hip-trace -d /tmp/prof_s3b -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify
python3 scripts/rocpd_timeline.py /tmp/prof_s3b/run_results.db --api > gpurun_out/hiptrace_timeline.md 2>&1
python3 - <<'PY' >> gpurun_out/hiptrace_timeline.md 2>&1
import sqlite3
db = sqlite3.connect("/tmp/prof_s3b/run_results.db")
print([r[1] for r in db.execute("pragma table_info(regions)")])
PY
rm -rf /tmp/prof_s3b
