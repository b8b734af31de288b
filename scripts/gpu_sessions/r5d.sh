set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 3 --no-parity > gpurun_out/r5d_w1.jsonl 2>&1
echo "w1 rc=$?" >> gpurun_out/r5d_w1.jsonl
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --no-parity > gpurun_out/r5d_w8.jsonl 2>&1
echo "w8 rc=$?" >> gpurun_out/r5d_w8.jsonl
KMLS_DEEP_NO_BOARD=1 timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --no-parity > gpurun_out/r5d_w8_noboard.jsonl 2>&1
echo "w8nb rc=$?" >> gpurun_out/r5d_w8_noboard.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5d_prof -o w8 -- python3 scripts/deep_probe.py --supports 0.02 --reps 1 --world 8 --no-parity > gpurun_out/r5d_prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/r5d_prof.log
