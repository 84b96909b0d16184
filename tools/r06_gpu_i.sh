#!/bin/bash
# Round 6 GPU batch I: C5 panel kernel, interleaved n-ranges (default) vs contiguous (A/B env), parity + timing.
cd "$(dirname "$0")/.."
out=gpurun_out/r06_i; mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp8_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2 3; do
  for v in 0 1; do
    echo "== interleave $v" >> $out/c5.log
    MAMBA_CLIP_AMD_SIM8_INTERLEAVE=$v timeout -k 10 200 python3 -u tools/time_c5_graph.py >> $out/c5.log 2>&1 || exit 1
  done
done
grep -E "==|logits" $out/c5.log
