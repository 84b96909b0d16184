#!/bin/bash
# Round-4 check 27: C3 step kernel breakdown (rocprofv3 kernel trace of the C3 bench)
set -u
out=gpurun_out/r04c27; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/rp -o c3 -- python bench.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 5 --warmup 3 --no-cpu-baseline --no-roofline > $out/rp.log 2>&1 || { echo rocprof failed; tail -20 $out/rp.log; exit 2; }
f=$(find $out/rp -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py $f 60 > $out/c3_step_breakdown.txt || true
find $out/rp -name "*kernel_trace.csv" -delete
head -45 $out/c3_step_breakdown.txt | cut -c1-160
