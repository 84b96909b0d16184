set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/lds_audit.py --out gpurun_out/n_lds_audit.json > gpurun_out/n_lds_audit.log 2>&1; echo "lds audit rc=$?"
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2"
timeout -k 10 400 $P --repeats 10 --variants conc,conc_nofine,conc_text,conc_text_nofine > gpurun_out/m_det.log 2>&1; echo "det rc=$?"
echo done
