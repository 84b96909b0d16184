#!/bin/bash
# Round-4 check 5: C2 bench kernel trace with the two-stream towers -> per-queue overlap and breakdown
set -u
out=gpurun_out/r04c5; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o t -- python bench.py --steps 4 --warmup 3 --no-roofline --no-cpu-baseline > $out/trace.log 2>&1 || { echo trace failed; tail -20 $out/trace.log; exit 2; }
f=$(ls $out/trace/*kernel_trace.csv | head -1)
python tools/stream_overlap.py $f | tee $out/overlap.txt
python tools/step_breakdown.py $f 60 > $out/breakdown.txt
head -45 $out/breakdown.txt
