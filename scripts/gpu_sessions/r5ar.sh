set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR --kernel-include-regex "k_pl_|k_hl_|k_map_filter|k_csr_refilter" -d gpurun_out/r5ar_sq -o c3 -- python3 scripts/c3_probe.py --steps 2 > gpurun_out/r5ar_sq.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --kernel-include-regex "k_pl_|k_hl_|k_map_filter|k_csr_refilter" -d gpurun_out/r5ar_tcc -o c3 -- python3 scripts/c3_probe.py --steps 2 > gpurun_out/r5ar_tcc.log 2>&1
echo "rc=$?"
