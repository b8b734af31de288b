set -o pipefail
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 1 --world 8 --no-parity --trace > gpurun_out/r5f_w8_trace.jsonl 2>&1
echo "w8t rc=$?" >> gpurun_out/r5f_w8_trace.jsonl
KMLS_DEEP_NO_BOARD=1 timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 1 --world 8 --no-parity --trace > gpurun_out/r5f_w8_trace_nb.jsonl 2>&1
echo "w8tnb rc=$?" >> gpurun_out/r5f_w8_trace_nb.jsonl
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --no-parity --trace > gpurun_out/r5f_w1_trace.jsonl 2>&1
echo "w1t rc=$?" >> gpurun_out/r5f_w1_trace.jsonl
KMLS_DEEP_NO_BOARD=1 timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 3 --no-parity > gpurun_out/r5f_w1_nb.jsonl 2>&1
echo "w1nb rc=$?" >> gpurun_out/r5f_w1_nb.jsonl
