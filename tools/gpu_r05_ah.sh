set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 10 --variants conc"
timeout -k 10 400 $P --isolate-aten embedding_dense_backward > gpurun_out/ah_emb.log 2>&1; echo "iso emb rc=$?"; grep '"runs"' gpurun_out/ah_emb.log | cut -c1-300
timeout -k 10 400 $P --isolate mc_scan_bwd > gpurun_out/ah_scan.log 2>&1; echo "iso scan rc=$?"; grep '"runs"' gpurun_out/ah_scan.log | cut -c1-300
timeout -k 10 400 $P --isolate mc_scan_fwd > gpurun_out/ah_scanf.log 2>&1; echo "iso scanfwd rc=$?"; grep '"runs"' gpurun_out/ah_scanf.log | cut -c1-300
echo done
