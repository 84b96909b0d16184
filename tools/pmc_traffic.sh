#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter group per run) over tools/pmc_traffic.py.
#   usage: tools/pmc_traffic.sh <outdir>
set -u
out=$1; mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o p --output-format csv -- python tools/pmc_traffic.py > "$out/fetch.log" 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o p --output-format csv -- python tools/pmc_traffic.py > "$out/write.log" 2>&1 || { echo "write pass failed"; exit 2; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d "$out/fcal" -o p --output-format csv -- tools/ubench/fetch_calib > "$out/fcal.log" 2>&1 || { echo "calibration pass failed"; exit 3; }
python tools/pmc_traffic_report.py "$out"
