set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 10 --variants conc,conc_text"
for iso in mc_scan_bwd mc_attn_bwd mc_scan_bwd,mc_attn_bwd mc_attn_fwd,mc_attn_bwd,mc_ce_fused_grad; do
  timeout -k 10 300 $P --isolate $iso > gpurun_out/t_iso_$iso.log 2>&1 || { echo "iso $iso failed rc=$?"; exit 1; }
  echo "== isolate $iso"; grep '"runs"' gpurun_out/t_iso_$iso.log | cut -c1-300
done
echo done
