set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 10 --variants seq,conc,conc_nofine,conc_text,conc_text_nofine > gpurun_out/v_det.log 2>&1; echo "det rc=$?"
grep '"runs"' gpurun_out/v_det.log | cut -c1-400
echo done
