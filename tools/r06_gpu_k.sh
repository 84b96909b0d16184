#!/bin/bash
# Round 6 GPU batch K: weight-gradient slab epilogue through LDS with 16-B row stores vs 4-B direct stores.
cd "$(dirname "$0")/.."
out=gpurun_out/r06_k; mkdir -p $out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wgrad_gpu.py tests/test_linear_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2 3; do
  for v in 0 1; do
    echo "== slab_vec $v" >> $out/wgrad.log
    MC_WGRAD_SLAB_VEC=$v timeout -k 10 200 python3 -u tools/time_wgrad_slab.py >> $out/wgrad.log 2>&1 || exit 1
  done
done
grep -E "==|total" $out/wgrad.log
