#!/bin/bash
# C2 step A/B (fused dt_proj on/off, same box) + a rocprofv3 kernel trace of a short bench for the step breakdown.
set -u
out=gpurun_out/step; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_step.py --toggle fuse_dt_proj --steps 10 --reps 3 > $out/ab_fuse.txt 2>&1 || { echo ab failed; tail -20 $out/ab_fuse.txt; exit 1; }
cat $out/ab_fuse.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o t -- python bench.py --steps 4 --warmup 3 --no-roofline --no-cpu-baseline > $out/trace.log 2>&1 || { echo trace failed; tail -20 $out/trace.log; exit 2; }
python tools/step_breakdown.py $(ls $out/trace/*kernel_trace.csv | head -1) 45 > $out/breakdown.txt
head -50 $out/breakdown.txt
