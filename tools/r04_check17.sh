#!/bin/bash
# C3 step kernel breakdown (BiomedCLIP ViT-B/16 + PubMedBERT-256, b 64)
set -u
out=gpurun_out/r04c17; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o t -- python bench.py --model biomedclip-vit_b16-pubmedbert256 --batch 64 --steps 4 --warmup 3 --no-roofline --no-cpu-baseline > $out/trace.log 2>&1 || { echo trace failed; tail -20 $out/trace.log; exit 3; }
f=$(find $out/trace -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py $f 60 > $out/breakdown.txt
python tools/stream_overlap.py $f > $out/overlap.txt
find $out/trace -name "*kernel_trace.csv" -delete
head -45 $out/breakdown.txt; cat $out/overlap.txt
