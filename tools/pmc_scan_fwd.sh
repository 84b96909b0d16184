#!/bin/bash
# PMC passes over the scan forward at one shape for the given variants (run on the GPU box).
#   usage: tools/pmc_scan_fwd.sh <outdir> <shape> <variant>...
set -u
out=$1; shp=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
for v in "$@"; do
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
              "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
    tag=$(echo $pass | cut -d' ' -f1)
    MC_SCAN_FWD_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $pass -d "$out/v${v}_$tag" -o p --output-format csv \
      -- python tools/time_scan.py --shape $shp --iters 3 > "$out/v${v}_$tag.log" 2>&1 || { echo "pmc failed v=$v $tag"; exit 1; }
  done
done
echo done
