set -u
timeout -k 10 400 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c2cmp_default.log 2>&1 || { echo "default tests failed"; tail -30 gpurun_out/c2cmp_default.log; exit 1; }
tail -1 gpurun_out/c2cmp_default.log
MC_SCAN_FWD_VARIANT=20 timeout -k 10 400 python -u -m pytest tests/test_scan_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c2cmp_v20.log 2>&1 || { echo "v20 tests failed"; tail -30 gpurun_out/c2cmp_v20.log; exit 1; }
tail -1 gpurun_out/c2cmp_v20.log
for a in "256,1536,80,16 -1" "256,1536,80,16 20" "256,1536,96,16 20"; do set -- $a; MC_SCAN_FWD_VARIANT=$2 timeout -k 5 60 python tools/time_scan.py --shape $1 --cm --train-fwd --iters 20 2>&1 | grep -v amdgpu.ids; echo "  (variant $2)"; done
for v in -1 20; do MC_SCAN_FWD_VARIANT=$v timeout -k 5 60 python tools/time_scan.py --shape 256,1536,80,16 --cm --iters 20 2>&1 | grep -v amdgpu.ids; echo "  (inference, variant $v)"; done
