set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 ./tools/coherence_repro 300 > gpurun_out/y_coh.log 2>&1; echo "coh rc=$?"; cat gpurun_out/y_coh.log
echo done
