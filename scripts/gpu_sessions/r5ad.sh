set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_serve_loop.py > gpurun_out/r5ad_tests.log 2>&1 &&
timeout -k 10 200 python3 scripts/serve_loop_probe.py --reps 1000 > gpurun_out/r5ad_probe.log 2>&1
echo "rc=$?"
