#!/bin/bash
# Round 6 GPU batch F: scan backward with the fine-state DMA issued in the last sub-tile (product) vs
# the previous build (_v_prev): parity tests, then interleaved C2 / C4 fwd+bwd timing.
cd "$(dirname "$0")/.."
out=gpurun_out/r06_f; mkdir -p $out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_scan_gpu.py tests/test_configs_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
L=mamba-clip_amd/mamba_clip_amd
for rep in 1 2 3; do
  for v in prev prod; do
    so=$PWD/$L/libmamba_clip_amd.so; [ $v != prod ] && so=$PWD/$L/libmamba_clip_amd_v_$v.so
    MAMBA_CLIP_AMD_LIB=$so timeout -k 10 120 python3 -u tools/time_scan.py --shape 256,1536,80,16 --cm --bwd --iters 50 >> $out/c2_$v.log 2>&1 || exit 1
    MAMBA_CLIP_AMD_LIB=$so timeout -k 10 120 python3 -u tools/time_scan.py --shape 64,3072,4096,16 --bwd --iters 10 >> $out/c4_$v.log 2>&1 || exit 1
  done
done
grep -h shape $out/c2_*.log $out/c4_*.log
