set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cooc.py tests/test_gpu_hlevels.py tests/test_gpu_dist.py > gpurun_out/r5ab_tests.log 2>&1 &&
timeout -k 10 300 python3 scripts/c3_probe.py --steps 5 > gpurun_out/r5ab_c3.log 2>&1 &&
timeout -k 10 500 python3 scripts/c5_probe.py --steps 3 > gpurun_out/r5ab_c5.log 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r5ab_prof -o c5 -- python3 scripts/c5_probe.py --steps 2 > gpurun_out/r5ab_c5_prof.log 2>&1
echo "rc=$?"
