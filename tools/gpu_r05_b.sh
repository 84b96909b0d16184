set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/race_probe.py --concurrent 1 --repeats 5 --out gpurun_out/race_conc.json > gpurun_out/race_conc.log 2>&1; echo "conc rc=$?"
timeout -k 10 300 python -u tools/race_probe.py --concurrent 0 --repeats 3 --out gpurun_out/race_seq.json > gpurun_out/race_seq.log 2>&1; echo "seq rc=$?"
timeout -k 10 300 python -u tools/race_probe.py --side-load gemm --repeats 5 --out gpurun_out/race_gemm.json > gpurun_out/race_gemm.log 2>&1; echo "gemm-load rc=$?"
echo done
