set -o pipefail
df -h /tmp . | tee gpurun_out/r5a_df.txt
free -g | tee -a gpurun_out/r5a_df.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_deep_product.py tests/test_gpu_cooc.py tests/test_gpu_e2e.py > gpurun_out/r5a_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/deep_trie_probe.py --support 0.02 --reps 2 --digest > gpurun_out/r5a_probe.log 2>&1
