set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_wgrad_gpu.py tests/test_guard_gpu.py tests/test_optim_gpu.py > gpurun_out/g_tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 $T tests/test_scan_gpu.py -k "pair_kernels or golden" > gpurun_out/g_pair.log 2>&1; echo "pair rc=$?"
timeout -k 10 500 python -u tools/determinism_probe.py --compare first --steps 2 --repeats 3 --variants seq,conc,conc_sharedcast,conc_text > gpurun_out/g_det.log 2>&1; echo "det rc=$?"
timeout -k 10 300 python -u tools/race_probe.py --concurrent 1 --repeats 4 --watch --out gpurun_out/g_race.json > gpurun_out/g_race.log 2>&1; echo "race rc=$?"
echo done
