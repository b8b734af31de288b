#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -q
step bench1 300 python bench.py --steps 30 --warmup 5
step bench1_mfma 300 python bench.py --steps 30 --warmup 5 --mfma
step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2
