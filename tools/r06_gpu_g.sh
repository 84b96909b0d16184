#!/bin/bash
# Round 6 GPU batch G: C5 panel kernel with three B stages (product) vs two (_v_p2): fp8 parity, timing.
cd "$(dirname "$0")/.."
out=gpurun_out/r06_g; mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp8_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
L=mamba-clip_amd/mamba_clip_amd
for rep in 1 2 3; do
  for v in orig p2 prod; do
    so=$PWD/$L/libmamba_clip_amd.so; [ $v != prod ] && so=$PWD/$L/libmamba_clip_amd_v_$v.so
    echo "== $v" >> $out/c5b.log
    MAMBA_CLIP_AMD_LIB=$so timeout -k 10 120 python3 -u tools/time_c5.py >> $out/c5b.log 2>&1 || exit 1
  done
done
grep -E "==|fp8" $out/c5b.log
