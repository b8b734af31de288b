set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5r_prof -o serve -- python3 scripts/serve_loop_probe.py --reps 400 > gpurun_out/r5r_prof.log 2>&1; echo "rc=$?" >> gpurun_out/r5r_prof.log
