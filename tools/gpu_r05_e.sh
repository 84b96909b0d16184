set -o pipefail
cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 python -u tools/race_probe.py --concurrent 1 --repeats 8 --watch --out gpurun_out/race_watch.json > gpurun_out/race_watch.log 2>&1; echo "watch rc=$?"
timeout -k 10 300 $T tests/test_wgrad_gpu.py > gpurun_out/wgrad_tests5.log 2>&1 || { echo "wgrad tests failed rc=$?"; tail -30 gpurun_out/wgrad_tests5.log; exit 1; }
timeout -k 10 300 python -u tools/time_wgrad.py vit_qkv vit_fc1 vit_fc2 vit_proj mamba_in_proj mamba_out_proj > gpurun_out/time_wgrad5.log 2>&1 || { echo "timing failed"; tail -5 gpurun_out/time_wgrad5.log; exit 1; }
echo done
