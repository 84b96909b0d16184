set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/race_probe.py --light --concurrent 1 --repeats 16 > gpurun_out/s_race_light.log 2>&1; echo "race light rc=$?"
echo done
