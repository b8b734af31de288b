#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 600 python -m pytest tests -m gpu -x -q
step bench1 300 python bench.py --steps 20 --warmup 3
step bench1_mfma 300 python bench.py --steps 20 --warmup 3 --mfma
step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2
