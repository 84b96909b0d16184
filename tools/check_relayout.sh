#!/bin/bash
# GPU suite, then C4 scan timing and a rocprof kernel-stats pass (B/C relayout vs scan kernel).
set -u
out=gpurun_out/relayout; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for i in 1 2; do timeout -k 5 60 python tools/time_scan.py --shape 64,3072,4096,16 --iters 20 2>&1 | grep shape; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof -o c4 --output-format csv -- python tools/time_scan.py --shape 64,3072,4096,16 --iters 20 > $out/prof.log 2>&1 || { echo "rocprof failed"; exit 2; }
cut -d, -f1-4 $out/prof/c4_kernel_stats.csv | head -5
