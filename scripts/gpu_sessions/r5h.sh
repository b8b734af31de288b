set -o pipefail
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 1 --world 8 --no-parity --trace > gpurun_out/r5h_w8_trace.jsonl 2>&1
echo "w8t rc=$?" >> gpurun_out/r5h_w8_trace.jsonl
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 1 --no-parity --trace > gpurun_out/r5h_w1_trace.jsonl 2>&1
echo "w1t rc=$?" >> gpurun_out/r5h_w1_trace.jsonl
