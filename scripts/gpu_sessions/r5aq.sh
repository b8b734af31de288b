set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5aq_gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5aq_gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5aq_smoke.log 2>&1
echo "smoke rc=$?" >> gpurun_out/r5aq_smoke.log
