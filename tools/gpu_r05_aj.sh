set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 12"
timeout -k 10 400 $P --variants seq,conc,conc_text > gpurun_out/aj_det.log 2>&1; echo "det rc=$?"; grep '"runs"' gpurun_out/aj_det.log | cut -c1-500
timeout -k 10 200 python3 tools/list_reductions.py > gpurun_out/aj_red.txt 2>&1; grep -v amdgpu gpurun_out/aj_red.txt
echo done
