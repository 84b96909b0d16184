set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 10 --batch 32 --variants conc"
for d in 0 1 2 3; do
  MC_DEBUG_SCAN_BWD_SYNC=$d timeout -k 10 300 $P > gpurun_out/an_$d.log 2>&1; echo "sync=$d: $(grep '"runs"' gpurun_out/an_$d.log | cut -c1-250)"
done
echo done
