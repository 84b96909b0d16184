set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 10 --batch 32 --variants conc"
for m in other current device other_event; do
  timeout -k 10 300 $P --pre-sync $m > gpurun_out/ap_$m.log 2>&1; echo "pre-sync=$m: $(grep '"runs"' gpurun_out/ap_$m.log | cut -c1-250)"
done
echo done
