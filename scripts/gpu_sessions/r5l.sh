set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_deep.py tests/test_gpu_deep_product.py > gpurun_out/r5l_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/r5l_tests.log
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 3 --no-parity > gpurun_out/r5l_w1.jsonl 2>&1; echo "rc=$?" >> gpurun_out/r5l_w1.jsonl
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --no-parity > gpurun_out/r5l_w8.jsonl 2>&1; echo "rc=$?" >> gpurun_out/r5l_w8.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5l_prof -o w8 -- python3 scripts/deep_probe.py --supports 0.02 --reps 1 --world 8 --no-parity > gpurun_out/r5l_prof.log 2>&1; echo "prof rc=$?" >> gpurun_out/r5l_prof.log
