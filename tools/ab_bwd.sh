#!/bin/bash
# Backward A/B on one box: the in-tree library vs an alternate build (MAMBA_CLIP_AMD_LIB), C2 (channel-major) and C4.
set -u
timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_bwd_pytest.log 2>&1 || { echo "scan tests failed"; tail -30 gpurun_out/ab_bwd_pytest.log; exit 1; }
tail -1 gpurun_out/ab_bwd_pytest.log
for rep in 1 2; do
  for lib in new ${ALT:-ab_libs/lib_bwd_old.so}; do
    if [ $lib = new ]; then unset MAMBA_CLIP_AMD_LIB; else export MAMBA_CLIP_AMD_LIB=$PWD/$lib; fi
    a=$(timeout -k 5 60 python tools/time_scan.py --shape 256,1536,80,16 --cm --bwd --iters 20 2>&1 | grep -o "[0-9.]* ms" | head -1) || exit 2
    b=$(timeout -k 5 90 python tools/time_scan.py --shape 64,3072,4096,16 --bwd --iters 5 2>&1 | grep -o "[0-9.]* ms" | head -1) || exit 3
    echo "rep $rep $lib: C2 fwd+bwd $a  C4 fwd+bwd $b"
  done
done
unset MAMBA_CLIP_AMD_LIB
