set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 8 --variants conc,conc_text"
for iso in sum mm,addmm,bmm sum,mm,addmm,bmm,addmm_,mm_; do
  timeout -k 10 400 $P --isolate-aten $iso > gpurun_out/aa_$iso.log 2>&1 || { echo "iso $iso failed rc=$?"; tail -3 gpurun_out/aa_$iso.log; exit 1; }
  echo "== isolate aten $iso"; grep '"runs"' gpurun_out/aa_$iso.log | cut -c1-330
done
echo done
