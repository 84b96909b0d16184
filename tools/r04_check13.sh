#!/bin/bash
# Round-4 check 13: mixer projections with 4 chunks in flight (tests, C2 A/B, kernel times); C3 A/B of
# the transposed-weight input gradients
set -u
out=gpurun_out/r04c13; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_mixer_proj_gpu.py > $out/pytest.txt 2>&1 || { echo pytest failed; tail -50 $out/pytest.txt; exit 2; }
tail -2 $out/pytest.txt
for f in 1 0 1 0; do
  MAMBA_CLIP_AMD_FUSE_MIXER_PROJ=$f timeout -k 10 300 python bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c2_$f.json 2> $out/c2_$f.err || { echo bench failed; tail -20 $out/c2_$f.err; exit 2; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('fuse_mixer_proj', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'])" $out/c2_$f.json $f | tee -a $out/summary.txt
done
for t in 1 0 1 0; do
  MAMBA_CLIP_AMD_DGRAD_TN=$t timeout -k 10 300 python bench.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c3_$t.json 2> $out/c3_$t.err || { echo c3 failed; tail -20 $out/c3_$t.err; exit 3; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('c3 dgrad_tn', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'])" $out/c3_$t.json $t | tee -a $out/summary.txt
done
MAMBA_CLIP_AMD_FUSE_MIXER_PROJ=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o t -- python bench.py --steps 4 --warmup 3 --no-roofline --no-cpu-baseline > $out/trace.log 2>&1 || { echo trace failed; tail -20 $out/trace.log; exit 4; }
f=$(find $out/trace -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py $f 60 > $out/breakdown.txt
find $out/trace -name "*kernel_trace.csv" -delete
grep -E "kernels|mixer_proj" $out/breakdown.txt
