set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend loop --qps 2000,5000 --duration 3 --json-out gpurun_out/r5al_loop.json > gpurun_out/r5al_loop.log 2>&1
echo "rc=$?"
