set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --no-parity > gpurun_out/r5m_w1.jsonl 2>&1; echo "rc=$?" >> gpurun_out/r5m_w1.jsonl
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --no-parity > gpurun_out/r5m_w8.jsonl 2>&1; echo "rc=$?" >> gpurun_out/r5m_w8.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5m_prof -o w8 -- python3 scripts/deep_probe.py --supports 0.02 --reps 1 --world 8 --no-parity > gpurun_out/r5m_prof.log 2>&1; echo "prof rc=$?" >> gpurun_out/r5m_prof.log
