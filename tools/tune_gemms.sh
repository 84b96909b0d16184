#!/bin/bash
# Re-measure the per-shape library GEMM selection on an MI355X (run on the GPU box
# from the repo root); writes gpurun_out/tunableop_results0.csv -- copy it to
# mamba-clip_amd/mamba_clip_amd/tuning/gemm_gfx950_c2_b256.csv to commit.
set -eu
mkdir -p gpurun_out
MAMBA_CLIP_AMD_NO_GEMM_TUNING=1 PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv \
  timeout -k 10 900 python bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-roofline
