#!/bin/bash
# rocprofv3 kernel trace of a short C2 bench -> per-step kernel breakdown (tools/step_breakdown.py).
set -u
out=gpurun_out/steptr; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o t -- python bench.py --steps 4 --warmup 3 --no-roofline --no-cpu-baseline > $out/trace.log 2>&1 || { echo trace failed; tail -20 $out/trace.log; exit 2; }
python tools/step_breakdown.py $(ls $out/trace/*kernel_trace.csv | head -1) 45 > $out/breakdown.txt
head -30 $out/breakdown.txt
