#!/usr/bin/env bash
# roctx phase ranges over the kernel timeline of one job run on the GPU miner.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
export KMLS_ROCTX=1
P=/tmp/kmls_roctx_pvc
rm -rf $P && mkdir -p $P
python3 - <<PY
import pathlib
from tests.helpers import make_datasets
make_datasets(pathlib.Path("$P"), shapes=("ds1", "tiny"), seeds=(0, 1))
PY
export BASE_DIR=$P/api-data DATASETS_DIR=$P/datasets MINER=gpu MIN_SUPPORT=0.05
step markers 300 rocprofv3 --marker-trace --kernel-trace -d /tmp/prof_m -o run -- python3 -m kubernetes_machine_learning_server_amd.job
python3 - > gpurun_out/roctx_ranges.md <<'PY'
import sqlite3
db = sqlite3.connect("/tmp/prof_m/run_results.db")
cols = [r[1] for r in db.execute("pragma table_info(regions)")]
rows = list(db.execute("select * from regions where category like 'MARKER%' order by start"))
ia = db.execute("pragma table_info(region_args)").fetchall()
print("| roctx range | duration ms |\n|---|---|")
for r in rows:
    d = dict(zip(cols, r))
    label = d.get("name")
    ex = str(d.get("extdata") or "")
    if "kmls" in ex:
        import re
        m = re.search(r"(kmls[\w.()]+)", ex)
        label = m.group(1) if m else ex[:60]
    print(f"| {label} | {(d['end'] - d['start']) / 1e6:.3f} |")
PY
rm -rf /tmp/prof_m
step first_call 200 python -u scripts/probe_first_call.py
