set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/race_probe.py --light --concurrent 1 --repeats 14 > gpurun_out/o_race_light.log 2>&1; echo "race light rc=$?"
AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 python -u tools/determinism_probe.py --summary --steps 2 --repeats 6 --variants conc,conc_text > gpurun_out/o_det_serialize.log 2>&1; echo "det serialize rc=$?"
echo done
