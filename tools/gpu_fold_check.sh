#!/bin/bash
# mc_linear with the slice fold: parity + determinism tests, MLP backward step A/B, bench.
cd $GRAFT_REPO_ROOT
out=gpurun_out/fold; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_linear_gpu.py tests/test_determinism_gpu.py tests/test_reduce_gpu.py > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -2 $out/tests.txt
timeout -k 10 400 python -u tools/ab_step.py --toggle ops.MLP_HIP_BWD --steps 10 --reps 4 > $out/ab_bwd.txt 2>&1 || exit 3
grep rep $out/ab_bwd.txt
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 4; }
cut -c1-400 $out/bench.json
