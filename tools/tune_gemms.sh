#!/bin/bash
# Re-measure the per-shape library GEMM selection on an MI355X (run on the GPU box from the repo root),
# with the data-parallel grids the package sets (TENSILE_STREAMK_DATA_PARALLEL=1) and the towers on one
# stream (timing is not shared with the other tower).  Writes gpurun_out/tune_<model>/tunableop_results0.csv
# for C2 (b 256) and C3 (b 64); tools/merge_tuning.py folds them into the committed selection file.
set -eu
for cfg in "vit_b16-mamba130m 256" "biomedclip-vit_b16-pubmedbert256 64"; do
  set -- $cfg
  mkdir -p gpurun_out/tune_$1
  MAMBA_CLIP_AMD_CONCURRENT_TOWERS=0 MAMBA_CLIP_AMD_NO_GEMM_TUNING=1 PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
  PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune_$1/tunableop_results%d.csv \
    timeout -k 10 900 python bench.py --model $1 --batch $2 --steps 2 --warmup 2 --no-cpu-baseline --no-roofline \
    > gpurun_out/tune_$1/bench.log 2>&1 || { echo "tuning $1 failed"; tail -20 gpurun_out/tune_$1/bench.log; exit 1; }
  wc -l gpurun_out/tune_$1/tunableop_results0.csv
done
