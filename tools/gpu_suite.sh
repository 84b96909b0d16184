#!/bin/bash
# GPU parity suite + smoke, each step under its own time limit.
set -u
out=gpurun_out/suite; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
