set -o pipefail
timeout -k 10 300 python -u scripts/deep_sweep_env.py --world 8 --reps 2 --configs "STEAL_IDLE=1;STEAL_IDLE=0;STEAL_IDLE=0,BUDGET=32;STEAL_IDLE=0,BUDGET=64;STEAL_IDLE=0,PRESPLIT_COST=0;STEAL_IDLE=1,SPLIT_MIN=2;STEAL_IDLE=1,SPLIT_MIN=32;STEAL_IDLE=1,BLOCKS_PER_CU=3" > gpurun_out/r5j_sweep.jsonl 2>&1
echo "rc=$?" >> gpurun_out/r5j_sweep.jsonl
timeout -k 10 200 python -u scripts/deep_sweep_env.py --world 1 --reps 2 --configs "STEAL_IDLE=1;STEAL_IDLE=0;STEAL_IDLE=0,BUDGET=32;STEAL_IDLE=0,BUDGET=64" > gpurun_out/r5j_sweep_w1.jsonl 2>&1
echo "rc=$?" >> gpurun_out/r5j_sweep_w1.jsonl
