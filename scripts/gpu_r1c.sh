#!/usr/bin/env bash
source "$(dirname "$0")/gpu_round.sh"
step pytest_persist 600 python -m pytest tests/test_gpu_kernels.py -q -k "persistent or matches_cpu or chunked"
step bench_persist 300 python bench.py --steps 30 --warmup 5
step bench_levelwise 300 python bench.py --steps 30 --warmup 5 --level-wise
step pytest_gpu 900 python -m pytest tests -m gpu -q
step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3
