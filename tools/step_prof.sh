#!/bin/bash
# rocprofv3 kernel trace of a short C2 bench and the per-step, per-queue kernel breakdown.
#   usage: tools/step_prof.sh <outdir> [extra bench args]   (GPU box, repo root)
set -u
out=${1:-gpurun_out/step}; shift || true
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o t -- python bench.py --steps 4 --warmup 3 --no-roofline --no-cpu-baseline "$@" > $out/trace.log 2>&1 || { echo trace failed; tail -20 $out/trace.log; exit 2; }
python tools/step_breakdown.py $(ls $out/trace/*kernel_trace.csv | head -1) 60 > $out/breakdown.txt
find $out/trace -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
rm -f $out/trace/*kernel_trace.csv
head -80 $out/breakdown.txt
