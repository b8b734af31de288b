#!/usr/bin/env bash
# Round-2 s10: mask16 gram + one-tile support A/B at 100M / config 5, then the full GPU suite,
# smoke() and the driver's bench line on this tree.
source "$(dirname "$0")/../gpu_round.sh"
export PYTHONUNBUFFERED=1
L100="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --shape 100Mx1M --steps 3 --warmup 1 --mfma"
step l100_default 600 $L100
KMLS_GRAM_FP4=mask16 step l100_mask16 600 $L100
KMLS_SUPPORT_TILES=4 step l100_tiles4 600 $L100
RM10="python3 -m kubernetes_machine_learning_server_amd.bench.bench_large --rule-map --min-support 0.0002 --steps 1 --warmup 1 --shape 10Mx1M"
KMLS_GRAM_FP4=mask16 step rm10_mask16 600 $RM10
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py --gpus 1 --steps 20 --warmup 5
