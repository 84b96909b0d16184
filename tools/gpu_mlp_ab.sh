#!/bin/bash
# C2 step A/B of the MLP mc_linear toggles (tools/ab_step.py, interleaved, same box).
cd $GRAFT_REPO_ROOT
out=gpurun_out/lin; mkdir -p $out
timeout -k 10 400 python -u tools/ab_step.py --toggle ops.MLP_HIP_BWD --steps 10 --reps 4 > $out/ab_bwd_fc1off.txt 2>&1 || exit 3
grep rep $out/ab_bwd_fc1off.txt
MAMBA_CLIP_AMD_MLP_HIP_BWD=1 timeout -k 10 400 python -u tools/ab_step.py --toggle ops.MLP_HIP_FC2 --steps 10 --reps 3 > $out/ab_fc2_bwdon.txt 2>&1 || exit 4
grep rep $out/ab_fc2_bwdon.txt
