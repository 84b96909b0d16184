#!/bin/bash
# Round-4 check 34: C3 side-stream arrangement, text tower at high priority vs image tower at normal, 3 runs each
set -u
out=gpurun_out/r04c34; mkdir -p $out
export TMPDIR=/tmp
for v in "text -1" "image 0" "text -1" "image 0" "text -1" "image 0"; do
  set -- $v
  MAMBA_CLIP_AMD_SIDE_TOWER=$1 MAMBA_CLIP_AMD_SIDE_PRIORITY=$2 timeout -k 10 300 python bench.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c3_$1_$2.json 2> $out/c3_$1_$2.err || { echo c3 failed; tail -20 $out/c3_$1_$2.err; exit 3; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('c3 side', sys.argv[2], 'prio', sys.argv[3], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'], r['final_loss'])" $out/c3_$1_$2.json $1 $2 | tee -a $out/summary.txt
done
