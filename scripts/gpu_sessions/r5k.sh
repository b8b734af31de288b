set -o pipefail
(cd r4tree && timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 3 --no-parity > ../gpurun_out/r5k_r4_w1.jsonl 2>&1); echo "rc=$?" >> gpurun_out/r5k_r4_w1.jsonl
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 3 --no-parity > gpurun_out/r5k_w1.jsonl 2>&1; echo "rc=$?" >> gpurun_out/r5k_w1.jsonl
(cd r4tree && timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --no-parity > ../gpurun_out/r5k_r4_w8.jsonl 2>&1); echo "rc=$?" >> gpurun_out/r5k_r4_w8.jsonl
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --no-parity > gpurun_out/r5k_w8.jsonl 2>&1; echo "rc=$?" >> gpurun_out/r5k_w8.jsonl
