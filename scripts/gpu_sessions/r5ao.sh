set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u bench.py > gpurun_out/r5ao_bench.log 2> gpurun_out/r5ao_bench.err
echo "rc=$?"
