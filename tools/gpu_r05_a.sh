set -o pipefail
cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_wgrad_gpu.py > gpurun_out/wgrad_tests.log 2>&1 || { echo "wgrad tests failed rc=$?"; tail -30 gpurun_out/wgrad_tests.log; exit 1; }
timeout -k 10 300 python -u tools/time_wgrad.py > gpurun_out/time_wgrad.log 2>&1 || { echo "timing failed"; tail -5 gpurun_out/time_wgrad.log; exit 1; }
timeout -k 10 300 $T tests/test_guard_gpu.py tests/test_optim_gpu.py > gpurun_out/guard_optim_tests.log 2>&1; echo "guard/optim rc=$?"
timeout -k 10 300 $T tests/test_scan_gpu.py -k "pair_kernels or golden" > gpurun_out/pair_golden_tests.log 2>&1; echo "pair goldens rc=$?"
timeout -k 10 400 python -u tools/determinism_probe.py --compare prev --steps 2 --repeats 4 --variants conc,seq,conc_nofine,conc_noattn,conc_wgradhip --out gpurun_out/det2.json > gpurun_out/det2.log 2>&1 || { echo "probe2 failed rc=$?"; tail -5 gpurun_out/det2.log; exit 1; }
timeout -k 10 300 python -u tools/determinism_probe.py --fill-nan --compare prev --steps 1 --repeats 2 --variants seq,conc --out gpurun_out/det_nan.json > gpurun_out/det_nan.log 2>&1 || { echo "nan probe failed rc=$?"; tail -5 gpurun_out/det_nan.log; exit 1; }
echo done
