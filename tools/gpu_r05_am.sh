set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/oob_probe.py --steps 2 > gpurun_out/am_oob.log 2>&1; echo "oob c2 rc=$?"; grep violations gpurun_out/am_oob.log | cut -c1-1500; tail -2 gpurun_out/am_oob.log | cut -c1-300
timeout -k 10 500 python -u tools/oob_probe.py --steps 2 --batch 32 > gpurun_out/am_oob32.log 2>&1; echo "oob c2 b32 rc=$?"; grep violations gpurun_out/am_oob32.log | cut -c1-1500
echo done
