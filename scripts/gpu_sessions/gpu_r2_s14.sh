#!/usr/bin/env bash
# Round-2 s14: twin graph executables + rule-map nodes created after the levels' (opt-in envs):
# graph/prefetch tests with both on, headline A/B, timeline with both on.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
KMLS_GRAPH_TWIN=1 KMLS_RULEMAP_LATE=1 step pytest_graph 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py -q -x --timeout 300 --timeout-method thread -k "graph or prefetch or replay or resident or rule"
B="python3 bench.py --steps 50 --warmup 5 --no-config2 --no-config3 --serve-qps "
step bench_old 300 $B ""
KMLS_GRAPH_TWIN=1 KMLS_RULEMAP_LATE=1 step bench_new 300 $B ""
KMLS_GRAPH_TWIN=1 step bench_twin 300 $B ""
KMLS_RULEMAP_LATE=1 step bench_late 300 $B ""
KMLS_GRAPH_TWIN=1 KMLS_RULEMAP_LATE=1 step bench_new2 300 $B ""
KMLS_GRAPH_TWIN=1 KMLS_RULEMAP_LATE=1 step trace_new 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 30 --warmup 3 --no-verify --no-config2 --no-config3 --serve-qps ""
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline_s14.md 2>&1
cp /tmp/prof_k/run_results.db gpurun_out/tb14_results.db 2>/dev/null
rm -rf /tmp/prof_k
