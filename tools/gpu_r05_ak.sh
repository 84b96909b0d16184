set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 12"
timeout -k 10 400 $P --variants conc_nn,conc_text_nn,seq_nn > gpurun_out/ak_det.log 2>&1; echo "det rc=$?"; grep '"runs"' gpurun_out/ak_det.log | cut -c1-500
echo done
