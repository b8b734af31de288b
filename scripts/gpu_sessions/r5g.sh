set -o pipefail
timeout -k 10 300 python -u scripts/deep_sweep_env.py --world 8 --reps 2 --configs "ASK=8,CAP=2;ASK=8,CAP=2,NO_BOARD=1;ASK=2,CAP=1;ASK=2,CAP=1,NO_BOARD=1;ASK=1,CAP=0;ASK=1,CAP=0,NO_BOARD=1;ASK=4,CAP=1;BUDGET=4,ASK=2,CAP=1;BUDGET=2,ASK=2,CAP=1;BUDGET=16,ASK=2,CAP=1;BUDGET=4,ASK=1,CAP=0" > gpurun_out/r5g_sweep.jsonl 2>&1
echo "rc=$?" >> gpurun_out/r5g_sweep.jsonl
timeout -k 10 200 python -u scripts/deep_sweep_env.py --world 1 --reps 2 --configs "ASK=8,CAP=2;ASK=8,CAP=2,NO_BOARD=1;ASK=2,CAP=1;ASK=1,CAP=0;BUDGET=4,ASK=2,CAP=1" > gpurun_out/r5g_sweep_w1.jsonl 2>&1
echo "rc=$?" >> gpurun_out/r5g_sweep_w1.jsonl
