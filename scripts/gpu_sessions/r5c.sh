set -o pipefail
timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_deep_product.py tests/test_gpu_deep.py tests/test_gpu_cooc.py > gpurun_out/r5c_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5c_tests.log
timeout -k 10 240 python -u scripts/deep_probe.py --supports 0.02 --reps 2 --world 8 --no-parity > gpurun_out/r5c_w8.jsonl 2>&1
echo "w8 rc=$?" >> gpurun_out/r5c_w8.jsonl
timeout -k 10 120 python -u scripts/deep_probe.py --supports 0.02 --reps 3 --no-parity > gpurun_out/r5c_w1.jsonl 2>&1
echo "w1 rc=$?" >> gpurun_out/r5c_w1.jsonl
timeout -k 10 400 python -u -c "
import json
from kubernetes_machine_learning_server_amd.bench import bench_mine as bm
from kubernetes_machine_learning_server_amd.data.synthetic import generate
tx=generate('ds1',seed=0)
print(json.dumps(bm.run_job_full(tx, 0.02, '1d15b1d026fe928d14a65f5b88be8656')))
" > gpurun_out/r5c_job.log 2>&1
echo "job rc=$?" >> gpurun_out/r5c_job.log
