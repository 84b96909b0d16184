set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/as_gpu_tests.log 2>&1; echo "gpu tests rc=$?"; tail -4 gpurun_out/as_gpu_tests.log
echo done
