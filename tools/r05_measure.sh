#!/bin/bash
# Round-5 measurement on one GPU: rocprof kernel stats of a short bench, the per-queue C2 step
# breakdown, C4 scan forward / backward timings, and the scan backward's HBM traffic (PMC) at C4.
set -u
cd $GRAFT_REPO_ROOT
out=gpurun_out/r05m; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv \
  -- python -u bench.py --steps 10 --warmup 3 > $out/prof_bench.json 2> $out/prof.log || { echo "rocprof bench failed"; tail -20 $out/prof.log; exit 2; }
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/rocprof_bench_kernel_stats.csv \;
python tools/step_breakdown.py $(ls $out/prof/*/*kernel_trace.csv 2>/dev/null | head -1 || ls $out/prof/*kernel_trace.csv | head -1) 60 > $out/c2_step_breakdown.txt || true
find $out/prof -name "*kernel_trace.csv" -delete
head -5 $out/c2_step_breakdown.txt
for a in "" "--train-fwd" "--bwd"; do
  timeout -k 10 180 python tools/time_scan.py --shape 64,3072,4096,16 --iters 5 $a 2>&1 | grep -v amdgpu.ids >> $out/c4_scan_times.txt || { echo "time_scan $a failed"; exit 4; }
done
cat $out/c4_scan_times.txt
bash tools/pmc_bwd_traffic.sh $out/bwd_traffic 64,3072,4096,16 > $out/c4_scan_bwd_traffic.txt 2>&1 || { echo "bwd traffic failed"; tail -5 $out/c4_scan_bwd_traffic.txt; exit 5; }
rm -rf $out/bwd_traffic/*/
cat $out/c4_scan_bwd_traffic.txt
echo done
