set -o pipefail
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --serve-qps '' --no-emit --no-job --no-levelwise --no-config2 --no-config3 > gpurun_out/r5n_bench_c5.json 2> gpurun_out/r5n_bench_c5.err
echo "rc=$?" >> gpurun_out/r5n_bench_c5.err
