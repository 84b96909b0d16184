set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2"
timeout -k 10 400 $P --repeats 12 --variants conc,conc_nofine,conc_noattn,conc_text,conc_text_nofine > gpurun_out/m_det.log 2>&1; echo "det rc=$?"
echo done
