#!/bin/bash
# Round-end style GPU check (run on the GPU box from the repo root via gpurun):
#   GPU parity tests, smoke(), the bench line, and a rocprofv3 kernel-trace
#   summary of a short bench run.  Every GPU step has its own time limit and
#   the chain stops at the first failure.
#   usage: tools/gpu_check.sh <outdir> [skip-tests]
set -u
out=${1:-gpurun_out/check}
mkdir -p "$out"
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$out/pytest_gpu.log" 2>&1 || { echo "pytest failed: $?"; exit 1; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
    || { echo "smoke failed: $?"; exit 2; }
fi
timeout -k 10 600 python -u bench.py > "$out/bench.log" 2>&1 || { echo "bench failed: $?"; exit 3; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/prof_bench" -o bench --output-format csv \
  -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$out/prof_bench.log" 2>&1 \
  || { echo "rocprof failed: $?"; exit 4; }
tail -n 1 "$out/bench.log"
echo done
