#!/bin/bash
# Round-4 check 10: fused mixer projections -- tests, kernel times, C2 bench A/B
set -u
out=gpurun_out/r04c10; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_mixer_proj_gpu.py tests/test_model_gpu.py -k "mixer or proj" > $out/pytest.txt 2>&1 || { echo pytest failed; tail -50 $out/pytest.txt; exit 2; }
tail -2 $out/pytest.txt
for v in 11 01 10 11 01 10; do
  f=${v:0:1}; t=${v:1:1}
  MAMBA_CLIP_AMD_FUSE_MIXER_PROJ=$f MAMBA_CLIP_AMD_DGRAD_TN=$t timeout -k 10 300 python bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c2_$v.json 2> $out/c2_$v.err || { echo bench failed; tail -20 $out/c2_$v.err; exit 2; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('fuse_mixer_proj/dgrad_tn', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'])" $out/c2_$v.json $v | tee -a $out/summary.txt
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o t -- python bench.py --steps 4 --warmup 3 --no-roofline --no-cpu-baseline > $out/trace.log 2>&1 || { echo trace failed; tail -20 $out/trace.log; exit 3; }
f=$(find $out/trace -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py $f 60 > $out/breakdown.txt
python tools/stream_overlap.py $f > $out/overlap.txt
find $out/trace -name "*kernel_trace.csv" -delete
head -40 $out/breakdown.txt
