set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_cooc.py > gpurun_out/r5ap_tests.log 2>&1 || exit 1
for h in "pl_groups=64" "pl_groups=32" "pl_groups=128" "pl_groups=256" "pl_chunk=131072" "pl_chunk=32768"; do
  timeout -k 10 300 python3 scripts/c5_probe.py --steps 3 --hooks $h > gpurun_out/r5ap_c5_$h.log 2>&1 || exit 1
done
echo "rc=0"
