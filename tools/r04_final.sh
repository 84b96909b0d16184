#!/bin/bash
# Round-4 final measurements: default bench (C2 + roofline + CPU baseline), its rocprof kernel stats,
# C3 bench, C4 scan backward rocprof + PMC, scan-forward PMC traffic.  Each step under its own limit.
set -u
out=gpurun_out/${R04_OUT:-r04final}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $out/bench_c2_n1.json 2> $out/bench_c2_n1.err || { echo bench failed; tail -20 $out/bench_c2_n1.err; exit 2; }
cat $out/bench_c2_n1.json
timeout -k 10 400 python bench.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > $out/bench_c3_n1_b64.json 2> $out/bench_c3.err || { echo c3 failed; tail -20 $out/bench_c3.err; exit 3; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/rocprof_bench -o b -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline > $out/rocprof_bench.log 2>&1 || { echo rocprof bench failed; tail -20 $out/rocprof_bench.log; exit 4; }
f=$(find $out/rocprof_bench -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py $f 60 > $out/c2_step_breakdown.txt || true
find $out/rocprof_bench -name "*kernel_trace.csv" -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c4_bwd -o c -- python tools/time_scan.py --shape 64,3072,4096,16 --bwd --iters 5 > $out/c4_bwd.log 2>&1 || { echo c4 bwd failed; tail $out/c4_bwd.log; exit 5; }
find $out/c4_bwd -name "*kernel_trace.csv" -delete
SHAPE=64,3072,4096,16 bash tools/pmc_bwd_pair.sh > $out/c4_bwd_pmc.txt 2>&1 || { echo c4 pmc failed; tail $out/c4_bwd_pmc.txt; exit 6; }
cp -r gpurun_out/pmcb $out/c4_bwd_pmc_raw 2>/dev/null || true
bash tools/pmc_traffic.sh $out/traffic > $out/traffic.txt 2>&1 || { echo traffic failed; tail $out/traffic.txt; exit 7; }
tail -5 $out/traffic.txt
