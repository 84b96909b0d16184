#!/bin/bash
# Round-4 check 6: image input path tests; A/B of the GEMM selection files on C2 / C3; C2 fed from host
set -u
out=gpurun_out/r04c6; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_patch_input_gpu.py > $out/pytest.txt 2>&1 || { echo pytest failed; tail -40 $out/pytest.txt; exit 2; }
tail -3 $out/pytest.txt
old=mamba-clip_amd/mamba_clip_amd/tuning/gemm_gfx950_c2_b256.csv  # (removed after this A/B; in git history)
new=mamba-clip_amd/mamba_clip_amd/tuning/gemm_gfx950_dp.csv
for m in vit_b16-mamba130m:256 biomedclip-vit_b16-pubmedbert256:64; do
  model=${m%%:*}; b=${m##*:}
  for f in old new old new; do
    eval path=\$$f
    MAMBA_CLIP_AMD_GEMM_TUNING_FILE=$path timeout -k 10 300 python bench.py --model $model --batch $b --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/bench_${model}_$f.json 2> $out/bench_${model}_$f.err || { echo bench failed; tail -20 $out/bench_${model}_$f.err; exit 2; }
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], r['value'], r['median_pairs_per_sec'])" $out/bench_${model}_$f.json $model $f | tee -a $out/ab.txt
  done
done
timeout -k 10 300 python bench.py --input host --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/bench_c2_host.json 2> $out/bench_c2_host.err || { echo host bench failed; tail -20 $out/bench_c2_host.err; exit 2; }
python -c "import json,sys; r=json.load(open(sys.argv[1])); print('c2 host-fed', r['value'], r['median_pairs_per_sec'])" $out/bench_c2_host.json | tee -a $out/ab.txt
