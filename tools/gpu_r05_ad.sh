set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/layer_under_load.py --iters 40 > gpurun_out/ad_layer.log 2>&1; echo "layer rc=$?"; grep '"load"' gpurun_out/ad_layer.log; tail -3 gpurun_out/ad_layer.log
echo done
