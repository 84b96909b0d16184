#!/bin/bash
# Scan backward kernel time at one shape,
# contiguous and channel-major inputs (run on the GPU box).  usage: tools/ab_scan_bwd.sh <outdir> <shape>
set -u
out=$1; shp=$2; mkdir -p "$out"
export TMPDIR=/tmp
for g in 2; do
  for cm in "" "--cm"; do
    tag=g${g}${cm:+_cm}
    MC_SCAN_BWD_GROUP=$g timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out/$tag" -o t --output-format csv \
      -- python tools/time_scan.py --shape $shp --iters 5 --bwd $cm > "$out/$tag.log" 2>&1 || { echo "failed $tag"; exit 1; }
    echo "$tag $(grep scan_bwd_kernel "$out/$tag/t_kernel_stats.csv" | cut -d, -f4) $(grep scan_fwd "$out/$tag/t_kernel_stats.csv" | cut -d, -f4)"
  done
done
