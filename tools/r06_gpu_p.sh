#!/bin/bash
# Round 6 GPU batch P: SS2D projections on mc_ss2d_group_proj -- parity tests, then the einsum /
# matmul / group-proj timing at the medmamba stages and the SS2D block A/B.
cd "$(dirname "$0")/.."
out=gpurun_out/r06_p; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ss2d_gpu.py > $out/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $out/tests.log | head -20; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python3 -u tools/time_ss2d_proj.py > $out/proj.log 2>&1 || { tail -20 $out/proj.log; exit 1; }
grep x $out/proj.log
