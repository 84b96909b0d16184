set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="python -u tools/determinism_probe.py --summary --self-ref --steps 2 --repeats 8 --variants conc,conc_text"
for e in GPU_MAX_HW_QUEUES=1 HIP_FORCE_DEV_KERNARG=0 HIP_FORCE_DEV_KERNARG=1 AMD_SERIALIZE_KERNEL=1 AMD_SERIALIZE_KERNEL=2; do
  env $e timeout -k 10 300 $P > gpurun_out/q_$e.log 2>&1 || { echo "$e failed rc=$?"; exit 1; }
  echo "== $e"; grep '"runs"' gpurun_out/q_$e.log | cut -c1-300
done
echo done
