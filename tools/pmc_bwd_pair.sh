#!/bin/bash
# PMC passes over the scan backward at B64 D3072 L1024 (compare profiles/r02/scan_bwd/c4ch_L1024_pmc.txt).
set -u
out=gpurun_out/pmcb; mkdir -p $out
export TMPDIR=/tmp
SHAPE=${SHAPE:-64,3072,1024,16}
run() { timeout -s KILL 120 rocprofv3 "$@" --output-format csv -- python tools/time_scan.py --shape $SHAPE --bwd --iters 2 ; }
run --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $out/p1 -o p > $out/p1.log 2>&1 || { echo p1 failed; tail $out/p1.log; exit 1; }
run --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d $out/p2 -o p > $out/p2.log 2>&1 || { echo p2 failed; tail $out/p2.log; exit 1; }
python3 tools/pmc_summary.py $out/p1 bwd_pair; python3 tools/pmc_summary.py $out/p2 bwd_pair
ls $out/p1
