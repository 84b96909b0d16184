#!/bin/bash
# Round-4 check 7: fp8 tests (bf16 logits on hipBLASLt), C5 timing, same-box A/B of dt_proj inside the scan (C2)
set -u
out=gpurun_out/r04c7; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_fp8_gpu.py > $out/pytest_fp8.txt 2>&1 || { echo pytest failed; tail -40 $out/pytest_fp8.txt; exit 2; }
tail -2 $out/pytest_fp8.txt
timeout -k 10 200 python -c "
import json, bench
print(json.dumps(bench.similarity_c5()))" > $out/c5.json 2> $out/c5.err || { echo c5 failed; tail $out/c5.err; exit 2; }
cat $out/c5.json
for f in 0 1 0 1; do
  MAMBA_CLIP_AMD_FUSE_DT_PROJ=$f timeout -k 10 300 python bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c2_fuse$f.json 2> $out/c2_fuse$f.err || { echo bench failed; tail -20 $out/c2_fuse$f.err; exit 2; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('fuse_dt_proj', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'])" $out/c2_fuse$f.json $f | tee -a $out/ab_fuse.txt
done
