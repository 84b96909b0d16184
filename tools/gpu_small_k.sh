#!/bin/bash
# mc_gemm_small_k / mc_gemm_skinny_m (dt_proj / x_proj forward): parity tests, timing vs the library, C2 step A/B.  GPU box, repo root.
cd $GRAFT_REPO_ROOT
out=gpurun_out/smallk; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_gpu.py -k 'small_k or skinny_m' > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
timeout -k 10 120 python tools/time_linear_hip.py --small-k > $out/time.txt 2>&1 || { cat $out/time.txt; exit 2; }
cat $out/time.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_mixer_proj_gpu.py > $out/tests_model.txt 2>&1 || { tail -30 $out/tests_model.txt; exit 3; }
tail -2 $out/tests_model.txt
timeout -k 10 400 python -u tools/ab_step.py --toggle ops.SKINNY_M_HIP --steps 10 --reps 4 > $out/ab.txt 2>&1 || exit 4
grep rep $out/ab.txt
