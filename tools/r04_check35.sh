#!/bin/bash
# Round-4 check 35: deferred casts (text tower's + transposed copies cast on the text stream after the fork)
# -- GPU suite, C2 / C3 A/B
set -u
out=gpurun_out/r04c35; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest.txt 2>&1 || { echo pytest failed; tail -60 $out/pytest.txt; exit 2; }
tail -2 $out/pytest.txt
for t in 1 0 1 0; do
  MAMBA_CLIP_AMD_DEFER_CASTS=$t timeout -k 10 300 python bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c2_$t.json 2> $out/c2_$t.err || { echo c2 failed; tail -20 $out/c2_$t.err; exit 3; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('c2 defer_casts', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'], r['final_loss'])" $out/c2_$t.json $t | tee -a $out/summary.txt
done
for t in 1 0 1 0; do
  MAMBA_CLIP_AMD_DEFER_CASTS=$t timeout -k 10 300 python bench.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c3_$t.json 2> $out/c3_$t.err || { echo c3 failed; tail -20 $out/c3_$t.err; exit 4; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('c3 defer_casts', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'], r['final_loss'])" $out/c3_$t.json $t | tee -a $out/summary.txt
done
