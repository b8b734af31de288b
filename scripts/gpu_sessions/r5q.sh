set -o pipefail
timeout -k 10 200 python -u scripts/serve_loop_probe.py > gpurun_out/r5q_loop_probe.jsonl 2>&1; echo "rc=$?" >> gpurun_out/r5q_loop_probe.jsonl
