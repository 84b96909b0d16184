#!/bin/bash
# Round measurement on one GPU: bench line, rocprof kernel stats of a short bench, PMC HBM traffic of the
# roofline kernel, and C4 scan forward (inference / training) + forward-backward timings.
set -u
out=gpurun_out/meas; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv \
  -- python -u bench.py --steps 10 --warmup 3 > $out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $out/prof.log; exit 2; }
bash tools/pmc_traffic.sh $out/traffic > $out/traffic.log 2>&1 || { echo "traffic failed"; tail -20 $out/traffic.log; exit 3; }
for a in "" "--train-fwd" "--bwd"; do
  timeout -k 10 180 python tools/time_scan.py --shape 64,3072,4096,16 --iters 5 $a 2>&1 | grep -v amdgpu.ids >> $out/times.txt || { echo "time_scan $a failed"; exit 4; }
done
cat $out/times.txt
tail -20 $out/traffic.log
echo done
