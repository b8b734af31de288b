set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_serve_loop.py > gpurun_out/r5s_serve_tests.log 2>&1 &&
timeout -k 10 200 python3 scripts/serve_loop_probe.py --reps 1000 > gpurun_out/r5s_probe.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5s_prof -o serve -- python3 scripts/serve_loop_probe.py --reps 300 > gpurun_out/r5s_prof.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_hlevels.py tests/test_gpu_cooc.py > gpurun_out/r5s_hl_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/c3_probe.py --steps 5 > gpurun_out/r5s_c3.log 2>&1
echo "rc=$?"
