#!/bin/bash
# Round-4 check 15: mixer projections with 8 waves per workgroup (K split in halves)
set -u
out=gpurun_out/r04c15; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_mixer_proj_gpu.py > $out/pytest.txt 2>&1 || { echo pytest failed; tail -50 $out/pytest.txt; exit 2; }
tail -2 $out/pytest.txt
timeout -k 10 120 python tools/time_mixer_proj.py 2>&1 | grep fused | tee -a $out/summary.txt || exit 3
for f in 1 0 1 0; do
  MAMBA_CLIP_AMD_FUSE_MIXER_PROJ=$f timeout -k 10 300 python bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c2_$f.json 2> $out/c2_$f.err || { echo bench failed; tail -20 $out/c2_$f.err; exit 2; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('fuse_mixer_proj', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'])" $out/c2_$f.json $f | tee -a $out/summary.txt
done
