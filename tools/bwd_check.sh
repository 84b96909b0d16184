#!/bin/bash
# Scan backward: parity tests, then kernel times at C4 and C2 (rocprofv3 kernel trace).
set -u
out=gpurun_out/bwd; mkdir -p $out
export TMPDIR=/tmp
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "bwd or c4 or grouped or c2_mamba" > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert" $out/pytest.log | head -30; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for shp in "64,3072,4096,16" "256,1536,80,16 --cm"; do
  tag=$(echo $shp | cut -d, -f1-3 | tr ',' '_' | tr -d ' -')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$tag -o run -- python tools/time_scan.py --shape $shp --bwd --iters 10 > $out/time_$tag.txt 2>&1 || { echo "rocprof failed $shp"; tail -20 $out/time_$tag.txt; exit 1; }
  grep -v amdgpu.ids $out/time_$tag.txt | tail -3
  f=$(find $out/prof_$tag -name "*kernel_stats.csv" | head -1)
  cut -d, -f1-8 "$f" | head -12 | cut -c1-200
done
