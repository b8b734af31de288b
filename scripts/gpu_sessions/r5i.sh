set -o pipefail
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 1 --world 8 --no-parity --trace --presplit-cost 0 > gpurun_out/r5i_w8_nopresplit.jsonl 2>&1
echo "rc=$?" >> gpurun_out/r5i_w8_nopresplit.jsonl
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 1 --world 8 --no-parity --trace --assign 0 --presplit-cost 0 > gpurun_out/r5i_w8_assign0.jsonl 2>&1
echo "rc=$?" >> gpurun_out/r5i_w8_assign0.jsonl
