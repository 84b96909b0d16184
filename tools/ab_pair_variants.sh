#!/bin/bash
# Interleaved A/B of the pair-kernel variants on one box (MC_SCAN_FWD_VARIANT 20..23), C4 and C2 training fwd.
set -u
for rep in 1 2 3; do
  for v in ${VARIANTS:-20 22 23 0}; do
    a=$(MC_SCAN_FWD_VARIANT=$v timeout -k 5 60 python tools/time_scan.py --shape 64,3072,4096,16 --iters 10 2>&1 | grep -o "[0-9.]* ms" | head -1) || exit 1
    b=$(MC_SCAN_FWD_VARIANT=$v timeout -k 5 60 python tools/time_scan.py --shape 256,1536,80,16 --cm --train-fwd --iters 20 2>&1 | grep -o "[0-9.]* ms" | head -1) || exit 1
    echo "rep $rep v=$v C4 $a C2-train $b"
  done
done
