set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u bench.py > gpurun_out/r5ac_bench.log 2> gpurun_out/r5ac_bench.err
echo "rc=$?"
