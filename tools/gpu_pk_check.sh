#!/bin/bash
# packed GELU / GELU' epilogues: parity tests, epilogue timings, step A/Bs (MLP backward, fused fc1).
cd $GRAFT_REPO_ROOT
out=gpurun_out/pk; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_gpu.py > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
timeout -k 10 200 python tools/time_linear_hip.py --epilogues > $out/epi.txt 2>&1 || exit 2
cat $out/epi.txt
timeout -k 10 400 python -u tools/ab_step.py --toggle ops.MLP_HIP_BWD --steps 10 --reps 4 > $out/ab_bwd.txt 2>&1 || exit 3
grep rep $out/ab_bwd.txt
timeout -k 10 400 python -u tools/ab_step.py --toggle ops.MLP_HIP_FC1 --steps 10 --reps 4 > $out/ab_fc1.txt 2>&1 || exit 4
grep rep $out/ab_fc1.txt
