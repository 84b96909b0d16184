#!/bin/bash
# Round 6 GPU batch M: which tower on the side stream (text = default vs image), interleaved C2 benches.
cd "$(dirname "$0")/.."
out=gpurun_out/r06_m; mkdir -p $out
for rep in 1 2; do
  for v in text image; do
    MAMBA_CLIP_AMD_SIDE_TOWER=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/side_${v}_$rep.json 2> $out/side_${v}_$rep.err || exit 1
  done
done
for f in $out/side_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'])"; done
