#!/bin/bash
# Round 6 GPU batch O: kernel traces of SS2D's projection einsums (two stages, both formulations).
cd "$(dirname "$0")/.."
out=gpurun_out/r06_o; mkdir -p $out
export TMPDIR=/tmp
for st in 56 14; do
  for f in einsum matmul; do
    STAGE=$st FORMS=$f timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $out/p_${st}_$f -o t --output-format csv -- python3 tools/time_ss2d_proj.py > $out/p_${st}_$f.log 2>&1 || exit 1
    find $out/p_${st}_$f -name "*kernel_stats.csv" -exec cp {} $out/stats_${st}_$f.csv \;
    find $out/p_${st}_$f -name "*kernel_trace.csv" -delete
  done
done
echo done
