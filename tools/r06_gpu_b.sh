#!/bin/bash
# Round 6 GPU batch B: op_sel-free broadcast variants of the pair backward -- in-step determinism
# (scan_bwd_localize) and fwd+bwd timing at C2 / C4 shapes against the product build.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06_loc gpurun_out/r06_time
L=mamba-clip_amd/mamba_clip_amd
VARIANTS="sel1 bcastc" RUNS=8 timeout -k 10 300 bash tools/r06_loc_ab.sh || exit 1
for v in prod sel1; do
  so=$PWD/$L/libmamba_clip_amd.so; [ $v != prod ] && so=$PWD/$L/libmamba_clip_amd_v_$v.so
  for rep in 1 2; do
    MAMBA_CLIP_AMD_LIB=$so timeout -k 10 120 python3 -u tools/time_scan.py --shape 256,1536,80,16 --cm --bwd --iters 30 \
      >> gpurun_out/r06_time/c2_bwd_$v.log 2>&1 || exit 1
    MAMBA_CLIP_AMD_LIB=$so timeout -k 10 120 python3 -u tools/time_scan.py --shape 64,3072,4096,16 --bwd --iters 10 \
      >> gpurun_out/r06_time/c4_bwd_$v.log 2>&1 || exit 1
  done
done
