set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 10 --batch 32 --variants conc"
for r in 0 1; do
  MC_RECORD_GRAD_STREAM=$r timeout -k 10 300 $P > gpurun_out/ao_$r.log 2>&1; echo "record=$r: $(grep '"runs"' gpurun_out/ao_$r.log | cut -c1-250)"
done
echo done
