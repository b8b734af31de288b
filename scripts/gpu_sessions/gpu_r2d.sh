#!/usr/bin/env bash
# Round-2 d: survivors-only level rows, banded/masked encode, device rule map from a caller
# gram; GPU suite, headline A/B + write counters, 100M encode A/B, config-5 rule map (10M, 100M).
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
B=(python3 bench.py --no-config2 --serve-qps "" --steps 50 --warmup 5)
step bench_kb64 300 "${B[@]}"
KMLS_KB18_TILES=100000 step bench_kb_all 300 "${B[@]}"
KMLS_KB18_TILES=0 step bench_kb_none 300 "${B[@]}"
step ktrace 300 rocprofv3 --kernel-trace -d /tmp/prof_k -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify --no-config2 --serve-qps ""
python3 scripts/rocpd_timeline.py /tmp/prof_k/run_results.db > gpurun_out/ktrace_timeline_r2d.md 2>&1
rm -rf /tmp/prof_k
pmc() {  # pmc <name> <counters...>
  local name=$1; shift
  step pmc_$name 200 timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$name -o run -- python3 bench.py --steps 10 --warmup 3 --no-verify --no-config2 --serve-qps ""
  f=$(find /tmp/pmc_$name -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 scripts/summarize_pmc.py "$f" > gpurun_out/pmc_$name.md 2>&1
  rm -rf /tmp/pmc_$name
}
pmc hl_write TCC_EA0_WRREQ_sum WRITE_SIZE
KMLS_KB18_TILES=0 pmc hl_write_old TCC_EA0_WRREQ_sum WRITE_SIZE
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1"
step l100_mask 600 $L100
KMLS_ENCODE_MASK=0 step l100_nomask 600 $L100
RM="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 0"
step rm10 600 $RM --shape 10Mx1M
step rm100 1100 $RM --shape 100Mx1M
