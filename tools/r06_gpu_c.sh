#!/bin/bash
# Round 6 GPU batch C: scan parity with the op_sel-free forward, the two-stream determinism and graph
# tests, and forward timing (old forward = the _v_sel1 build, new = the product build) at C2 / C4.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06_c
L=mamba-clip_amd/mamba_clip_amd
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_scan_gpu.py > gpurun_out/r06_c/scan.log 2>&1 || exit 1
timeout -k 10 700 $T tests/test_determinism_gpu.py tests/test_graph_gpu.py > gpurun_out/r06_c/det_graph.log 2>&1 || exit 1
for v in sel1 prod; do
  so=$PWD/$L/libmamba_clip_amd.so; [ $v != prod ] && so=$PWD/$L/libmamba_clip_amd_v_$v.so
  for rep in 1 2; do
    for f in "" "--train-fwd"; do
      MAMBA_CLIP_AMD_LIB=$so timeout -k 10 120 python3 -u tools/time_scan.py --shape 256,1536,80,16 --cm $f --iters 50 \
        >> gpurun_out/r06_c/c2_fwd_$v.log 2>&1 || exit 1
      MAMBA_CLIP_AMD_LIB=$so timeout -k 10 120 python3 -u tools/time_scan.py --shape 64,3072,4096,16 $f --iters 10 \
        >> gpurun_out/r06_c/c4_fwd_$v.log 2>&1 || exit 1
    done
  done
done
