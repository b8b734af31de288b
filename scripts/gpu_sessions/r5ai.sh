set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_cooc.py tests/test_gpu_hlevels.py > gpurun_out/r5ai_tests.log 2>&1 &&
timeout -k 10 300 python3 scripts/c3_probe.py --steps 5 > gpurun_out/r5ai_c3.log 2>&1 &&
timeout -k 10 400 python3 scripts/c5_probe.py --steps 3 > gpurun_out/r5ai_c5.log 2>&1
echo "rc=$?"
