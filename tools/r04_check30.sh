#!/bin/bash
# Round-4 check 30: text-tower stream at HIP's high priority vs normal -- C2 / C3 A/B, interleaved
set -u
out=gpurun_out/r04c30; mkdir -p $out
export TMPDIR=/tmp
for t in 1 0 1 0; do
  MAMBA_CLIP_AMD_SIDE_PRIORITY=$((-t)) timeout -k 10 300 python bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c2_$t.json 2> $out/c2_$t.err || { echo c2 failed; tail -20 $out/c2_$t.err; exit 3; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('c2 side_high_priority', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'])" $out/c2_$t.json $t | tee -a $out/summary.txt
done
for t in 1 0 1 0; do
  MAMBA_CLIP_AMD_SIDE_PRIORITY=$((-t)) timeout -k 10 300 python bench.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c3_$t.json 2> $out/c3_$t.err || { echo c3 failed; tail -20 $out/c3_$t.err; exit 4; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('c3 side_high_priority', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'])" $out/c3_$t.json $t | tee -a $out/summary.txt
done
