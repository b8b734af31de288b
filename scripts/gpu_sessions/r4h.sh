mkdir -p gpurun_out/r4h
bash scripts/gpu_sessions/r4g.sh
timeout -k 10 300 python -u scripts/make_large_pvc.py --out /tmp/pvc_c5 > gpurun_out/r4h/pvc.json 2> gpurun_out/r4h/pvc.err; cat gpurun_out/r4h/pvc.json
for be in auto hip cpu; do
timeout -k 10 300 python -u -m kubernetes_machine_learning_server_amd.bench.bench_serve --pvc /tmp/pvc_c5 --backend $be --qps 2000,10000 --duration 4 --reload-index /tmp/pvc_c5/rules_alt.idx --reload-at 4 --reload-qps 10000 --reload-duration 10 > gpurun_out/r4h/serve_c5_$be.jsonl 2> gpurun_out/r4h/serve_c5_$be.err || break
grep -h "reload_under_load\|serve_ready" gpurun_out/r4h/serve_c5_$be.jsonl | cut -c1-600
done
