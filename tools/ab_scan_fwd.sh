set -u
out=gpurun_out/ab1; mkdir -p $out
for v in ${VARIANTS:-0 4 5}; do
  for shp in 64,3072,4096,16 256,1536,80,16; do
    MC_SCAN_FWD_VARIANT=$v timeout -k 10 120 python tools/time_scan.py --shape $shp --iters 10 >> $out/times.txt 2>&1 || { echo "fail v=$v $shp"; exit 1; }
    echo "v=$v" >> $out/times.txt
  done
done
MC_SCAN_FWD_VARIANT=${TESTV:-4} timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest_v4.log 2>&1 || { echo "pytest v4 failed"; tail -30 $out/pytest_v4.log; exit 2; }
tail -2 $out/pytest_v4.log
cat $out/times.txt
