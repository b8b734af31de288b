set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 scripts/make_large_pvc.py --out /tmp/pvc_c5 > gpurun_out/r5an_pvc.log 2>&1 &&
timeout -k 10 300 python3 -m kubernetes_machine_learning_server_amd.bench.bench_serve --pvc /tmp/pvc_c5 --backend loop --qps 10000 --duration 3 --reload-index /tmp/pvc_c5/rules_alt.idx --reload-qps 10000 --reload-duration 10 --reload-at 4 --json-out gpurun_out/r5an_loop_reload.json > gpurun_out/r5an_loop_reload.log 2>&1
echo "rc=$?"
