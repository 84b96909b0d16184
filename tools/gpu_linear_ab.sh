#!/bin/bash
# C2 step A/B: the other Linears' forward / input-gradient GEMMs on mc_linear vs the library.
cd $GRAFT_REPO_ROOT
out=gpurun_out/lin; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_gpu.py tests/test_model_gpu.py > $out/tests2.txt 2>&1 || { tail -20 $out/tests2.txt; exit 1; }
tail -2 $out/tests2.txt
timeout -k 10 400 python -u tools/ab_step.py --toggle ops.LINEAR_HIP_FWD --steps 10 --reps 4 > $out/ab_linear_fwd.txt 2>&1 || exit 3
grep rep $out/ab_linear_fwd.txt
timeout -k 10 400 python -u tools/ab_step.py --toggle ops.LINEAR_HIP_DGRAD --steps 10 --reps 4 > $out/ab_linear_dgrad.txt 2>&1 || exit 4
grep rep $out/ab_linear_dgrad.txt
