set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_reduce_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py > gpurun_out/af_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/af_tests.log
timeout -k 10 400 python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 10 --variants seq,conc,conc_text > gpurun_out/af_det.log 2>&1; echo "det rc=$?"; grep '"runs"' gpurun_out/af_det.log | cut -c1-400
timeout -k 10 300 python -u tools/sum_under_load.py --iters 30 --loads gemm_vit > gpurun_out/af_sum.log 2>&1; grep '"load"' gpurun_out/af_sum.log | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --no-roofline --no-cpu-baseline > gpurun_out/af_bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/af_bench.log | cut -c1-200
echo done
