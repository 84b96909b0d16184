#!/bin/bash
# Full GPU parity suite, then the scan-forward A/B timings at C4.
set -u
out=gpurun_out/round; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
for v in ${VARIANTS:-0 20}; do
  echo "v=$v" >> $out/times.txt
  MC_SCAN_FWD_VARIANT=$v timeout -k 10 120 python tools/time_scan.py --shape 64,3072,4096,16 --iters 10 >> $out/times.txt 2>&1 || { echo "fail v=$v"; exit 2; }
done
grep -v amdgpu.ids $out/times.txt
