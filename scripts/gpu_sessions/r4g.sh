mkdir -p gpurun_out/r4g
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_cooc.py tests/test_gpu_deep.py > gpurun_out/r4g/tests.log 2>&1; tail -3 gpurun_out/r4g/tests.log
timeout -k 10 300 python -u scripts/cooc_probe.py --shape 10Mx1M --reps 3 --step --no-gemm > gpurun_out/r4g/cooc.jsonl 2>&1; grep probe gpurun_out/r4g/cooc.jsonl | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --serve-qps '' --no-config2 --no-config3 --no-levelwise > gpurun_out/r4g/bench_emit.json 2> gpurun_out/r4g/bench_emit.err; tail -c 1500 gpurun_out/r4g/bench_emit.json
timeout -k 10 200 python -u scripts/deep_probe.py --supports 0.02 --reps 3 --trace > gpurun_out/r4g/deep_w1.jsonl 2>&1
timeout -k 10 200 python -u scripts/deep_probe.py --supports 0.02 --reps 3 --trace --presplit-cost 0 --no-parity > gpurun_out/r4g/deep_w1_nops.jsonl 2>&1
for pc in 16 8 24; do for pb in 1 4; do
timeout -k 10 200 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --trace --no-parity --presplit-cost $pc --presplit-budget $pb > gpurun_out/r4g/deep_w8_pc${pc}_pb${pb}.jsonl 2>&1 || break
done; done
grep -h split gpurun_out/r4g/deep_w8*.jsonl | cut -c1-300
grep -h '"probe": "deep"' gpurun_out/r4g/deep_w1*.jsonl | cut -c1-200
