#!/bin/bash
# Round-6 final tree on one GPU: full GPU suite + smoke, the bench line, a rocprofv3 kernel-trace summary
# of a short bench with the per-queue step breakdown, and the C2 b256 run-to-run determinism probe.
set -u
cd "$(dirname "$0")/.."
out=gpurun_out/final6; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 2; }
tail -1 $out/smoke.log
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 3; }
cut -c1-300 $out/bench.json
timeout -k 10 600 python -u tools/determinism_probe.py --batch 256 --steps 3 --repeats 6 --variants conc,seq --summary --self-ref \
  > $out/determinism_c2_b256.log 2>&1 || { echo "probe failed"; tail -20 $out/determinism_c2_b256.log; exit 4; }
tail -4 $out/determinism_c2_b256.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv \
  -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof_bench.json 2> $out/prof.log || { echo "rocprof failed"; tail -20 $out/prof.log; exit 5; }
tr=$(find $out/prof -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py "$tr" 60 > $out/c2_step_breakdown.txt || true
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/rocprof_bench_kernel_stats.csv \;
find $out/prof -name "*kernel_trace.csv" -delete
head -3 $out/c2_step_breakdown.txt
echo done
