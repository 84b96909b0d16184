#!/bin/bash
# Round-4 check 26: dB / dC partial-store swizzle in scan_bwd_pair_kernel -- scan tests, C2 / C4 per-kernel A/B
# against the previous build (tools/exp_lib/lib_head.so), interleaved
set -u
out=gpurun_out/r04c26; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_scan_gpu.py tests/test_configs_gpu.py > $out/pytest.txt 2>&1 || { echo pytest failed; tail -40 $out/pytest.txt; exit 2; }
tail -2 $out/pytest.txt
for v in new head new head; do
  if [ $v = new ]; then unset MAMBA_CLIP_AMD_LIB; else export MAMBA_CLIP_AMD_LIB=$PWD/tools/exp_lib/lib_head.so; fi
  for shp in "256,1536,80,16 --cm" "64,3072,4096,16"; do
    tag=$(echo $shp | cut -d, -f1-3 | tr ',' 'x')
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${v}_$tag -o p -- python tools/time_scan.py --shape $shp --bwd --iters 10 > $out/${v}_$tag.log 2>&1 || { echo "$v $tag failed"; tail -5 $out/${v}_$tag.log; exit 3; }
    f=$(find $out/${v}_$tag -name "*kernel_stats.csv" | head -1); find $out/${v}_$tag -name "*kernel_trace.csv" -delete
    python -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'scan_bwd_pair' in r['Name']:
        print(sys.argv[2], sys.argv[3], 'avg %.1f us' % (float(r['AverageNs']) / 1e3), r['Calls'], 'calls')
" $f $v $tag | tee -a $out/summary.txt
    rm -rf $out/${v}_$tag
  done
done
