set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 10 --batch 32 --variants conc"
for m in clone_bias clone_D clone_A; do
  timeout -k 10 300 $P --pre-sync $m > gpurun_out/aq_$m.log 2>&1; echo "$m: $(grep '"runs"' gpurun_out/aq_$m.log | cut -c1-250)"
done
echo done
