#!/bin/bash
# Round-4 check 9: fine saved states with the LDS-DMA prefetch -- scan tests, kernel times, C2 bench A/B
set -u
out=gpurun_out/r04c9; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_scan_gpu.py tests/test_configs_gpu.py > $out/pytest.txt 2>&1 || { echo pytest failed; tail -40 $out/pytest.txt; exit 2; }
tail -2 $out/pytest.txt
for v in fine0 fine; do
  case $v in fine0) export MAMBA_CLIP_AMD_FINE_STATES_MB=0; unset MAMBA_CLIP_AMD_LIB;;
             fine) export MAMBA_CLIP_AMD_FINE_STATES_MB=1024; unset MAMBA_CLIP_AMD_LIB;;
             fnt) export MAMBA_CLIP_AMD_FINE_STATES_MB=1024; export MAMBA_CLIP_AMD_LIB=$PWD/ab_libs/lib_fnt.so;; esac
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c2_$v -o p -- python tools/time_scan.py --shape 256,1536,80,16 --cm --bwd --iters 20 > $out/c2_$v.log 2>&1 || { echo "c2 $v failed"; tail -5 $out/c2_$v.log; exit 2; }
  find $out/c2_$v -name "*kernel_trace.csv" -delete
  f=$(find $out/c2_$v -name "*kernel_stats.csv" | head -1)
  python -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'scan_bwd_pair' in r['Name'] or 'scan_fwd_pair' in r['Name']:
        print(sys.argv[2], r['Name'].split('(')[0][-40:], 'avg %.1f us' % (float(r['AverageNs']) / 1e3), r['Calls'], 'calls')
" $f $v | tee -a $out/summary.txt
done
unset MAMBA_CLIP_AMD_LIB
for f in 1024 0 1024 0; do
  MAMBA_CLIP_AMD_FINE_STATES_MB=$f timeout -k 10 300 python bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/c2_bench_$f.json 2> $out/c2_bench_$f.err || { echo bench failed; tail -20 $out/c2_bench_$f.err; exit 2; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('fine_states_mb', sys.argv[2], r['value'], r['median_pairs_per_sec'], r['median_ms_per_step'])" $out/c2_bench_$f.json $f | tee -a $out/summary.txt
done
