#!/bin/bash
# Round-4 check 19: re-tune the GEMM selection with the transposed-weight input gradients (new tn
# shapes), merge with the committed file, A/B on C2 and C3
set -u
bash tools/tune_gemms.sh || exit 1
out=gpurun_out/r04c19; mkdir -p $out
python tools/merge_tuning.py $out/gemm_gfx950_dp_tn.csv mamba-clip_amd/mamba_clip_amd/tuning/gemm_gfx950_dp.csv \
  gpurun_out/tune_vit_b16-mamba130m/tunableop_results0.csv gpurun_out/tune_biomedclip-vit_b16-pubmedbert256/tunableop_results0.csv
old=mamba-clip_amd/mamba_clip_amd/tuning/gemm_gfx950_dp.csv; new=$out/gemm_gfx950_dp_tn.csv
for m in vit_b16-mamba130m:256 biomedclip-vit_b16-pubmedbert256:64; do
  model=${m%%:*}; b=${m##*:}
  for f in new old new old; do
    eval path=\$$f
    MAMBA_CLIP_AMD_GEMM_TUNING_FILE=$path timeout -k 10 300 python bench.py --model $model --batch $b --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/b_${model}_$f.json 2> $out/b_${model}_$f.err || { echo bench failed; tail -20 $out/b_${model}_$f.err; exit 2; }
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'])" $out/b_${model}_$f.json $model $f | tee -a $out/ab.txt
  done
done
