set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/sum_under_load.py --iters 120 > gpurun_out/z_sum.log 2>&1; echo "sum rc=$?"; grep '"load"' gpurun_out/z_sum.log
echo done
