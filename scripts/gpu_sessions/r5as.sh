set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/deep_probe.py --world 8 --reps 2 > gpurun_out/r5as_w8.jsonl 2>&1
echo "rc=$?"
