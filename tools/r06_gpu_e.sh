#!/bin/bash
# Round 6 GPU batch E: full GPU suite + smoke, then the C4 scan PMC passes (forward traffic and VALU,
# backward traffic) each next to a kernel trace of the same command, so time and bytes pair up.
cd "$(dirname "$0")/.."
out=gpurun_out/r06_e; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -30 $out/smoke.log; exit 1; }
bash tools/pmc_traffic.sh $out/fwd > $out/fwd_traffic.log 2>&1 || { tail -20 $out/fwd_traffic.log; exit 1; }
bash tools/pmc_valu.sh $out/valu > $out/valu.log 2>&1 || { tail -20 $out/valu.log; exit 1; }
bash tools/pmc_bwd_traffic.sh $out/bwd 64,3072,4096,16 > $out/bwd_traffic.log 2>&1 || { tail -20 $out/bwd_traffic.log; exit 1; }
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $out/bwd_trace -o t --output-format csv -- python3 tools/time_scan.py --shape 64,3072,4096,16 --iters 3 --bwd > $out/bwd_trace.log 2>&1 || { tail -20 $out/bwd_trace.log; exit 1; }
find $out/bwd_trace -name "*kernel_stats.csv" -exec cp {} $out/bwd_kernel_stats.csv \;
echo done
