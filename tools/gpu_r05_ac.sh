set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/sum_under_load.py --iters 40 --loads none,gemm_vit > gpurun_out/ac_sum.log 2>&1; echo "sum rc=$?"; grep '"load"' gpurun_out/ac_sum.log
echo done
