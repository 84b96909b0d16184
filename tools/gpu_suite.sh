#!/bin/bash
# GPU parity suite + smoke (+ optional short bench), each step under its own time limit.
set -u
out=gpurun_out/suite; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $out/pytest_gpu.log | head -20; tail -60 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
grep -E "PASSED|FAILED" $out/pytest_gpu.log | grep -E "configs|durations" | head -20
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -30 $out/bench.err; exit 1; }
  cat $out/bench.json
fi
