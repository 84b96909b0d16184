set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_reduce_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py > gpurun_out/ag_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/ag_tests.log
timeout -k 10 400 python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 10 --variants conc > gpurun_out/ag_det.log 2>&1; echo "det rc=$?"; grep -v amdgpu gpurun_out/ag_det.log | cut -c1-500
echo done
