set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/av_gpu_tests.log 2>&1; echo "gpu tests rc=$?"; tail -2 gpurun_out/av_gpu_tests.log
timeout -k 10 400 python -u tools/determinism_probe.py --summary --self-ref --steps 3 --repeats 8 --variants seq,conc > gpurun_out/av_det.log 2>&1; echo "det: $(grep '"runs"' gpurun_out/av_det.log | cut -c1-200)"
timeout -k 10 600 python -u bench.py > gpurun_out/av_bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/av_bench.log
echo done
