set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-include-regex "k_map_filter|k_pl_part|k_pl_split" -d gpurun_out/r5ag_pmc -o c3 -- python3 scripts/c3_probe.py --steps 2 > gpurun_out/r5ag_pmc.log 2>&1
echo "rc=$?"
