#!/bin/bash
# Round-4 scan-backward levers: per-kernel time of scan_bwd_pair_kernel for timing-only variants
# (ab_libs/lib_<v>.so: norecomp = sub-tile states read instead of recomputed, noy = no Y accumulation)
set -u
out=gpurun_out/r04bx; mkdir -p $out
export TMPDIR=/tmp
for v in base norecomp noy both; do
  if [ $v = base ]; then unset MAMBA_CLIP_AMD_LIB; else export MAMBA_CLIP_AMD_LIB=$PWD/ab_libs/lib_$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o p -- python tools/time_scan.py --shape 256,1536,80,16 --cm --bwd --iters 20 > $out/$v.log 2>&1 || { echo "$v failed"; tail -5 $out/$v.log; exit 2; }
  f=$(find $out/$v -name "*kernel_stats.csv" | head -1); find $out/$v -name "*kernel_trace.csv" -delete
  python -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'scan_bwd_pair' in r['Name'] or 'scan_fwd_pair' in r['Name']:
        print(sys.argv[2], r['Name'].split('(')[0][-40:], 'avg %.1f us' % (float(r['AverageNs']) / 1e3), r['Calls'], 'calls')
" $f $v | tee -a $out/summary.txt
done
