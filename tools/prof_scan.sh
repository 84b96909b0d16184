#!/bin/bash
# Dev profiling recipe for the scan forward (run on the GPU box from the repo root).
# usage: tools/prof_scan.sh <outdir> [extra args for time_scan.py]
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
run() { timeout -k 10 300 rocprofv3 "$@" --output-format csv -- python tools/time_scan.py --iters 3 ${EXTRA:-} ; }
EXTRA="$*"
run --kernel-trace --stats -d "$out/trace" -o t > "$out/trace.log" 2>&1 || exit 1
run --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d "$out/p1" -o p > "$out/p1.log" 2>&1 || exit 2
run --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SMEM GRBM_GUI_ACTIVE -d "$out/p2" -o p > "$out/p2.log" 2>&1 || exit 3
run --pmc FETCH_SIZE -d "$out/p3" -o p > "$out/p3.log" 2>&1 || exit 4
run --pmc WRITE_SIZE -d "$out/p4" -o p > "$out/p4.log" 2>&1 || exit 5
run --pmc SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_UNALIGNED_STALL -d "$out/p5" -o p > "$out/p5.log" 2>&1 || exit 6
echo done
