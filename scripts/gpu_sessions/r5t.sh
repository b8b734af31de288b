set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5t_prof -o c3 -- python3 scripts/c3_probe.py --steps 2 > gpurun_out/r5t_c3.log 2>&1
echo "rc=$?"
