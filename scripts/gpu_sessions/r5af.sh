set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/c5_probe.py --steps 3 --hooks filter_lds=0 > gpurun_out/r5af_c5_l2mask.log 2>&1 || exit 1
timeout -k 10 300 python3 scripts/c3_probe.py --steps 5 --hooks filter_lds=0 > gpurun_out/r5af_c3_l2mask.log 2>&1 || exit 1
for cfg in "16 1" "16 2" "16 4" "8 2" "4 4"; do
  set -- $cfg
  timeout -k 10 240 python3 scripts/deep_probe.py --world 8 --reps 2 --presplit-cost $1 --presplit-budget $2 --no-parity > gpurun_out/r5af_c$1_b$2.jsonl 2>&1 || exit 1
done
echo "rc=0"
