#!/bin/bash
# VALU issue fraction of the scan kernels at C4 (one PMC pass + a kernel trace for the durations).
#   usage: tools/pmc_valu.sh <outdir>    (GPU box, repo root)
set -u
out=${1:-gpurun_out/valu}; mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  -d "$out/pmc" -o p --output-format csv -- python tools/time_scan.py --shape 64,3072,4096,16 --iters 3 > "$out/pmc.log" 2>&1 || { echo "pmc pass failed"; tail -5 "$out/pmc.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$out/trace" -o t --output-format csv -- python tools/time_scan.py --shape 64,3072,4096,16 --iters 5 > "$out/trace.log" 2>&1 || { echo "trace failed"; exit 2; }
python3 tools/pmc_summary.py "$out/pmc" scan_fwd_pair > "$out/fwd_summary.txt"
python3 tools/pmc_summary.py "$out/pmc" scan_bwd_pair > "$out/bwd_summary.txt"
cat "$out/fwd_summary.txt" "$out/bwd_summary.txt"
find "$out/trace" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats.csv" \;
echo done
