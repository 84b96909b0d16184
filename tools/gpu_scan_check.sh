#!/bin/bash
# Scan-kernel GPU check: parity tests, then rocprofv3 kernel stats of the training
# forward + backward at the C2 (channel-major mixer views) and C4 shapes.
#   usage: tools/gpu_scan_check.sh <outdir> [skip-tests]
set -u
out=${1:-gpurun_out/scan}
mkdir -p "$out"
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_model_gpu.py -m gpu -x -v --timeout 120 \
    --timeout-method thread > "$out/pytest_scan.log" 2>&1 || { echo "pytest failed: $?"; tail -30 "$out/pytest_scan.log"; exit 1; }
  tail -3 "$out/pytest_scan.log"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/c2" -o c2 --output-format csv \
  -- python -u tools/time_scan.py --shape 256,1536,80,16 --cm --bwd --iters 10 > "$out/c2.log" 2>&1 \
  || { echo "c2 prof failed: $?"; tail "$out/c2.log"; exit 2; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/c4" -o c4 --output-format csv \
  -- python -u tools/time_scan.py --shape 64,3072,4096,16 --bwd --iters 5 > "$out/c4.log" 2>&1 \
  || { echo "c4 prof failed: $?"; tail "$out/c4.log"; exit 3; }
for f in $(find "$out" -name "*kernel_stats.csv"); do echo "== $f"; cut -d, -f1-4 "$f" | head -8; done
echo done
