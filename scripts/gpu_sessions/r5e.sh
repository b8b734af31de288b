set -o pipefail
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 3 --no-parity > gpurun_out/r5e_w1.jsonl 2>&1
echo "w1 rc=$?" >> gpurun_out/r5e_w1.jsonl
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --no-parity > gpurun_out/r5e_w8.jsonl 2>&1
echo "w8 rc=$?" >> gpurun_out/r5e_w8.jsonl
KMLS_DEEP_NO_BOARD=1 timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --no-parity > gpurun_out/r5e_w8_noboard.jsonl 2>&1
echo "w8nb rc=$?" >> gpurun_out/r5e_w8_noboard.jsonl
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 1 --world 8 --no-parity --trace > gpurun_out/r5e_w8_trace.jsonl 2>&1
echo "w8t rc=$?" >> gpurun_out/r5e_w8_trace.jsonl
