set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_serve_loop.py > gpurun_out/r5o_tests.log 2>&1; echo "rc=$?" >> gpurun_out/r5o_tests.log
timeout -k 10 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend loop --qps 2000,10000 --duration 3 > gpurun_out/r5o_serve_loop.log 2>&1; echo "rc=$?" >> gpurun_out/r5o_serve_loop.log
timeout -k 10 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend auto --qps 2000,10000 --duration 3 > gpurun_out/r5o_serve_auto.log 2>&1; echo "rc=$?" >> gpurun_out/r5o_serve_auto.log
