set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 2 3 4; do
  timeout -k 10 240 python3 scripts/deep_probe.py --world 8 --reps 2 --blocks-per-cu $b --no-parity > gpurun_out/r5ak_bpc$b.jsonl 2>&1 || exit 1
done
for bud in 8 32; do
  timeout -k 10 240 python3 scripts/deep_probe.py --world 8 --reps 2 --budget $bud --no-parity > gpurun_out/r5ak_bud$bud.jsonl 2>&1 || exit 1
done
echo "rc=0"
