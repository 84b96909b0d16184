#!/bin/bash
# Round-4: the whole GPU suite + smoke (what the driver runs at round end)
set -u
out=gpurun_out/r04suite; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $out/pytest_gpu.txt 2>&1 || { echo pytest failed; tail -60 $out/pytest_gpu.txt; exit 2; }
tail -3 $out/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { echo smoke failed; tail -30 $out/smoke.txt; exit 3; }
tail -3 $out/smoke.txt
