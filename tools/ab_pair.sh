#!/bin/bash
# A/B of the long-sequence scan-forward kernels + scan parity with the pair kernel forced.
set -u
out=gpurun_out/pair; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $out/pytest_default.log 2>&1 || { echo "pytest default failed"; tail -40 $out/pytest_default.log; exit 1; }
tail -2 $out/pytest_default.log
MC_SCAN_FWD_VARIANT=20 timeout -k 10 400 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $out/pytest_v20.log 2>&1 || { echo "pytest v20 failed"; tail -40 $out/pytest_v20.log; exit 1; }
tail -2 $out/pytest_v20.log
for v in ${VARIANTS:-0 20}; do
  for shp in ${SHAPES:-64,3072,4096,16}; do
    echo "v=$v $shp" >> $out/times.txt
    MC_SCAN_FWD_VARIANT=$v timeout -k 10 120 python tools/time_scan.py --shape $shp --iters 10 >> $out/times.txt 2>&1 || { echo "fail v=$v $shp"; exit 2; }
  done
done
cat $out/times.txt
