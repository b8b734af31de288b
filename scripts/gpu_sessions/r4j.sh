mkdir -p gpurun_out/r4j
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4j/bench.json 2> gpurun_out/r4j/bench.err; tail -c 600 gpurun_out/r4j/bench.json; tail -3 gpurun_out/r4j/bench.err
