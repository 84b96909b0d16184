set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 ./tools/coherence_repro 300 > gpurun_out/x_coh.log 2>&1; echo "coh rc=$?"; cat gpurun_out/x_coh.log
timeout -k 10 300 python -u tools/sum_under_load.py --iters 150 > gpurun_out/x_sum.log 2>&1; echo "sum rc=$?"; grep '"load"' gpurun_out/x_sum.log
echo done
