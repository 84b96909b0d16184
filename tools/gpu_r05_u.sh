set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/determinism_probe.py --fill-nan --compare prev --steps 1 --repeats 2 --variants seq,conc > gpurun_out/u_nan.log 2>&1; echo "nan rc=$?"
echo done
