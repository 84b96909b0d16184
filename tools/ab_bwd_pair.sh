#!/bin/bash
# Interleaved same-box A/B of backward variants (ab_libs/lib_<v>.so vs in-tree): C4 and C2 fwd+bwd ms.
set -u
for rep in 1 2; do
  for v in new ${VARIANTS}; do
    if [ $v = new ]; then unset MAMBA_CLIP_AMD_LIB; else export MAMBA_CLIP_AMD_LIB=$PWD/ab_libs/lib_$v.so; fi
    a=$(timeout -k 5 60 python tools/time_scan.py --shape 256,1536,80,16 --cm --bwd --iters 20 2>&1 | grep -o "[0-9.]* ms" | head -1) || exit 2
    b=$(timeout -k 5 90 python tools/time_scan.py --shape 64,3072,4096,16 --bwd --iters 5 2>&1 | grep -o "[0-9.]* ms" | head -1) || exit 3
    echo "rep $rep $v: C2 fwd+bwd $a  C4 fwd+bwd $b"
  done
done
