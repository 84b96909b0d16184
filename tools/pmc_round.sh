#!/bin/bash
# This round's PMC evidence for the scan kernels (run on the GPU box from the repo root):
#   forward C4 HBM traffic (FETCH_SIZE / WRITE_SIZE, calibrated), forward LDS counters,
#   backward traffic + L2 hits at C2 (channel-major, as in the step) and C4.
#   usage: tools/pmc_round.sh <outdir>
set -u
out=${1:-gpurun_out/pmc}
mkdir -p "$out"
export TMPDIR=/tmp
bash tools/pmc_traffic.sh "$out/fwd_traffic" > "$out/fwd_traffic.txt" 2>&1 || { echo "fwd traffic failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAVES \
  -d "$out/fwd_lds" -o p --output-format csv -- python tools/time_scan.py --shape 64,3072,4096,16 --iters 3 \
  > "$out/fwd_lds.log" 2>&1 || { echo "fwd lds pass failed"; exit 2; }
bash tools/pmc_bwd_traffic.sh "$out/bwd_c2" "256,1536,80,16 --cm" > "$out/bwd_c2.txt" 2>&1 || { echo "bwd c2 failed"; exit 3; }
bash tools/pmc_bwd_traffic.sh "$out/bwd_c4" "64,3072,4096,16" > "$out/bwd_c4.txt" 2>&1 || { echo "bwd c4 failed"; exit 4; }
echo done
