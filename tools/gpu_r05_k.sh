set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --steps 2"
timeout -k 10 300 $P --repeats 8 --variants seq,conc,conc_text > gpurun_out/k_det.log 2>&1; echo "det rc=$?"
echo done
