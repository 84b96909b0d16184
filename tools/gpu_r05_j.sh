set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/grad_trace.py --repeats 6 --out gpurun_out/j_trace_image.json > gpurun_out/j_trace_image.log 2>&1; echo "trace image rc=$?"
timeout -k 10 400 python -u tools/grad_trace.py --repeats 6 --side-tower text --out gpurun_out/j_trace_text.json > gpurun_out/j_trace_text.log 2>&1; echo "trace text rc=$?"
echo done
