#!/bin/bash
# Round-4 check 31: text-tower stream priority for C2 (Mamba text tower): low (1) vs normal (0)
set -u
out=gpurun_out/r04c31; mkdir -p $out
export TMPDIR=/tmp
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range()); s=torch.cuda.Stream(priority=1); print('low stream priority', s.priority)" 2>&1 | grep -v amdgpu.ids | tee $out/range.txt
for t in 1 0 1 0; do
  MAMBA_CLIP_AMD_SIDE_PRIORITY=$t timeout -k 10 300 python bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c2_$t.json 2> $out/c2_$t.err || { echo c2 failed; tail -20 $out/c2_$t.err; exit 3; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('c2 side_priority', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'])" $out/c2_$t.json $t | tee -a $out/summary.txt
done
