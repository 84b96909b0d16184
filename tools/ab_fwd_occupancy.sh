#!/bin/bash
# A/B of the scan-forward kernel variants (MC_SCAN_FWD_VARIANT) at C4 and C2 (dev tool)
set -e
for v in ${VARIANTS:-2 3 4 10}; do
  MC_SCAN_FWD_VARIANT=$v timeout -k 10 120 python tools/time_scan.py --shape 64,3072,4096,16 --iters 10 | sed "s/^/v=$v /"
  MC_SCAN_FWD_VARIANT=$v timeout -k 10 120 python tools/time_scan.py --shape 256,1536,80,16 --cm --iters 20 | sed "s/^/v=$v /"
done
