set -o pipefail
timeout -k 10 300 python -u scripts/deep_trie_probe.py --support 0.02 --reps 2 --digest > gpurun_out/r5b_probe.log 2>&1
echo "probe rc=$?" >> gpurun_out/r5b_probe.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_deep_product.py tests/test_gpu_deep.py > gpurun_out/r5b_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5b_tests.log
