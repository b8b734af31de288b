mkdir -p gpurun_out/r4i
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_deep.py > gpurun_out/r4i/tests.log 2>&1; tail -3 gpurun_out/r4i/tests.log
for pc in 0 16; do for bu in 16 8; do
timeout -k 10 200 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --trace --no-parity --presplit-cost $pc --budget $bu > gpurun_out/r4i/deep_w8_pc${pc}_b${bu}.jsonl 2>&1 || break
timeout -k 10 200 python -u scripts/deep_probe.py --supports 0.02 --reps 3 --trace --no-parity --presplit-cost $pc --budget $bu > gpurun_out/r4i/deep_w1_pc${pc}_b${bu}.jsonl 2>&1 || break
done; done
grep -h split gpurun_out/r4i/deep_w8*.jsonl | cut -c1-300
for f in gpurun_out/r4i/deep_w1*.jsonl; do echo $f; grep -h '"probe": "deep"' $f | cut -c1-150; done
