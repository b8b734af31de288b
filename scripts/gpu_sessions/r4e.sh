mkdir -p gpurun_out/r4e
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_cooc.py tests/test_gpu_deep.py > gpurun_out/r4e/tests.log 2>&1; tail -3 gpurun_out/r4e/tests.log
timeout -k 10 300 python -u scripts/cooc_probe.py --shape 10Mx1M --reps 3 --step --no-gemm > gpurun_out/r4e/cooc.jsonl 2>&1; grep probe gpurun_out/r4e/cooc.jsonl | cut -c1-400
timeout -k 10 200 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --trace > gpurun_out/r4e/deep_w1.jsonl 2>&1
timeout -k 10 200 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --trace --no-parity > gpurun_out/r4e/deep_w8.jsonl 2>&1
timeout -k 10 200 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --assign 0 --trace --no-parity > gpurun_out/r4e/deep_w8_a0.jsonl 2>&1
grep split gpurun_out/r4e/deep_w8*.jsonl
