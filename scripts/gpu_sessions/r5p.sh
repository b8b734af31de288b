set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_serve_loop.py > gpurun_out/r5p_tests.log 2>&1; echo "rc=$?" >> gpurun_out/r5p_tests.log
