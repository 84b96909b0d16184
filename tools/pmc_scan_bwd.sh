#!/bin/bash
# Kernel trace + PMC passes over scan fwd+bwd at one shape (run on the GPU box).
#   usage: tools/pmc_scan_bwd.sh <outdir> <shape>
set -u
out=$1; shp=$2
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$out/trace" -o t --output-format csv \
  -- python tools/time_scan.py --shape $shp --iters 3 --bwd > "$out/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass -d "$out/b_$tag" -o p --output-format csv \
    -- python tools/time_scan.py --shape $shp --iters 3 --bwd > "$out/b_$tag.log" 2>&1 || { echo "pmc failed $tag"; exit 2; }
done
echo done
