#!/bin/bash
# Round-4 check 12: forward pair kernel with the compile-time fine branch; mixer projections with the
# Wdt prefetch -- scan + mixer tests, kernel times in the C2 step, C2 A/B of the fused projections
set -u
out=gpurun_out/r04c12; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_scan_gpu.py tests/test_mixer_proj_gpu.py > $out/pytest.txt 2>&1 || { echo pytest failed; tail -50 $out/pytest.txt; exit 2; }
tail -2 $out/pytest.txt
for f in 1 0 1 0; do
  MAMBA_CLIP_AMD_FUSE_MIXER_PROJ=$f timeout -k 10 300 python bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c2_$f.json 2> $out/c2_$f.err || { echo bench failed; tail -20 $out/c2_$f.err; exit 2; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('fuse_mixer_proj', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'])" $out/c2_$f.json $f | tee -a $out/summary.txt
done
for pj in 1 0; do
  MAMBA_CLIP_AMD_FUSE_MIXER_PROJ=$pj timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_$pj -o t -- python bench.py --steps 4 --warmup 3 --no-roofline --no-cpu-baseline > $out/trace_$pj.log 2>&1 || { echo trace failed; tail -20 $out/trace_$pj.log; exit 3; }
  f=$(find $out/trace_$pj -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py $f 60 > $out/breakdown_$pj.txt
  find $out/trace_$pj -name "*kernel_trace.csv" -delete
  echo "proj $pj"; grep -E "kernels|scan_fwd_pair|scan_bwd_pair|mixer_proj" $out/breakdown_$pj.txt
done
