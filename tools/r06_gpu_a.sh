#!/bin/bash
# Round 6 GPU batch A: fp8 panel kernel tests + C5 timing A/B, the scalar-math determinism variant,
# and the three-step two-stream DDP test.  Logs under gpurun_out/r06_c5 / r06_loc.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06_c5 gpurun_out/r06_loc
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_gpu.py -m gpu \
  > gpurun_out/r06_c5/test_fp8.log 2>&1; echo "pytest rc $?" >> gpurun_out/r06_c5/test_fp8.log
timeout -k 10 120 python3 -u tools/time_c5.py > gpurun_out/r06_c5/time_panel.log 2>&1 || exit 1
MAMBA_CLIP_AMD_SIM8_PANEL=0 timeout -k 10 120 python3 -u tools/time_c5.py > gpurun_out/r06_c5/time_tile.log 2>&1 || exit 1
VARIANTS=scalar RUNS=8 timeout -k 10 300 bash tools/r06_loc_ab.sh || exit 1
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 350 --timeout-method thread tests/test_dist_gloo.py -m gpu \
  -k three_steps > gpurun_out/r06_loc/ddp3.log 2>&1; echo "pytest rc $?" >> gpurun_out/r06_loc/ddp3.log
