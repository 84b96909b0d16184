#!/bin/bash
set -u
out=gpurun_out/r04c20; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python tools/torch_prof.py --rows 80 > $out/torch_prof.txt 2>&1 || { echo prof failed; tail -20 $out/torch_prof.txt; exit 2; }
grep -E "copy|contiguous|clone|to_copy|cat|transpose|Name" $out/torch_prof.txt | head -40
