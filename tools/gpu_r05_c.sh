set -o pipefail
cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 python -u tools/stress_determinism.py --iters 40 > gpurun_out/stress.log 2>&1; echo "stress rc=$?"
timeout -k 10 300 $T tests/test_wgrad_gpu.py > gpurun_out/wgrad_tests4.log 2>&1 || { echo "wgrad tests failed rc=$?"; tail -30 gpurun_out/wgrad_tests4.log; exit 1; }
timeout -k 10 300 python -u tools/time_wgrad.py > gpurun_out/time_wgrad4.log 2>&1 || { echo "timing failed"; tail -5 gpurun_out/time_wgrad4.log; exit 1; }
echo done
