set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/time_wgrad.py > gpurun_out/at_wgrad.log 2>&1; echo "wgrad rc=$?"; grep shape gpurun_out/at_wgrad.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], 'lib', d['lib_us'], d['lib_tflops'], 'hip', d['hip_us'], d['hip_tflops'], 'pipes', d['pipe_us'], 'err %.1e' % d['rel_err_vs_lib'], 'sweep', d['hip_split_sweep_us'])"
echo done
