#!/bin/bash
# rocprofv3 kernel trace + PMC passes over the fused attention at the C2 shape.
set -u
out=gpurun_out/pattn; mkdir -p $out
export TMPDIR=/tmp
run() { timeout -s KILL 120 rocprofv3 "$@" --output-format csv -- python tools/time_attn_bwd.py --iters 5 ; }
run --kernel-trace --stats -d $out/trace -o t > $out/trace.log 2>&1 || { echo trace failed; tail $out/trace.log; exit 1; }
head -12 $out/trace/t_kernel_stats.csv | cut -d, -f1-8
run --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $out/p1 -o p > $out/p1.log 2>&1 || { echo p1 failed; tail $out/p1.log; exit 1; }
run --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $out/p2 -o p > $out/p2.log 2>&1 || { echo p2 failed; tail $out/p2.log; exit 1; }
for k in attn_fwd attn_bwd; do echo "== $k"; python3 tools/pmc_summary.py $out/p1 $k; python3 tools/pmc_summary.py $out/p2 $k; done
