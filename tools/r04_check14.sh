#!/bin/bash
set -u
out=gpurun_out/r04c14; mkdir -p $out
for v in base p1only p2only base; do
  if [ $v = base ]; then unset MAMBA_CLIP_AMD_LIB; else export MAMBA_CLIP_AMD_LIB=$PWD/ab_libs/lib_$v.so; fi
  echo -n "$v: " | tee -a $out/summary.txt
  timeout -k 10 120 python tools/time_mixer_proj.py 2>&1 | grep fused | tee -a $out/summary.txt || exit 2
done
