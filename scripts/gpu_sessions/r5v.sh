set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_cooc.py tests/test_gpu_hlevels.py > gpurun_out/r5v_tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5v_prof -o c3 -- python3 scripts/c3_probe.py --steps 3 > gpurun_out/r5v_c3.log 2>&1 &&
timeout -k 10 300 python3 scripts/c3_probe.py --steps 5 > gpurun_out/r5v_c3_clean.log 2>&1
echo "rc=$?"
