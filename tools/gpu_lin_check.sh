#!/bin/bash
# mc_linear evidence: parity tests, epilogue timings vs the library chains, and the C2 step
# A/Bs of the MLP / Linear toggles (tools/ab_step.py, interleaved on one box).  GPU box, repo root.
cd $GRAFT_REPO_ROOT
out=gpurun_out/lin; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_gpu.py > $out/tests.txt 2>&1; echo "tests rc=$?" >> $out/tests.txt
tail -4 $out/tests.txt
grep -q "tests rc=0" $out/tests.txt || exit 1
timeout -k 10 200 python tools/time_linear_hip.py --epilogues > $out/epi.txt 2>&1 || exit 2
cat $out/epi.txt
for t in ops.MLP_HIP_BWD ops.MLP_HIP_FC2 ops.MLP_HIP_FC1 ops.LINEAR_HIP_FWD ops.LINEAR_HIP_DGRAD; do
  timeout -k 10 400 python -u tools/ab_step.py --toggle $t --steps 10 --reps 4 > $out/ab_${t#ops.}.txt 2>&1 || exit 3
  grep rep $out/ab_${t#ops.}.txt
done
