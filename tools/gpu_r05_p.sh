set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2"
timeout -k 10 500 $P --repeats 10 --variants seq,seq_rocblas,conc_rocblas,conc_noattn,conc_text_noattn > gpurun_out/p_det.log 2>&1; echo "det rc=$?"
echo done
