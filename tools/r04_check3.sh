#!/bin/bash
# Round-4 check 3: non-temporal output stores in the scan forward (interleaved C4 time A/B + PMC
# traffic of the variant); C5 similarity variants incl. hipBLASLt fp32 / bf16 out, DP vs stream-K grids.
set -u
out=gpurun_out/r04c3; mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base ntst; do
    if [ $v = base ]; then lib=""; else lib=ab_libs/lib_$v.so; fi
    r=$(MAMBA_CLIP_AMD_LIB=$lib timeout -k 5 90 python tools/time_scan.py --iters 20 2>&1 | grep -o "[0-9.]* ms" | head -1) || exit 3
    echo "rep $rep $v C4 fwd $r" | tee -a $out/nt_ab.txt
  done
done
MAMBA_CLIP_AMD_LIB=ab_libs/lib_ntst.so bash tools/pmc_traffic.sh $out/pmc_nt > $out/pmc_nt.log 2>&1 || { echo pmc failed; tail -20 $out/pmc_nt.log; exit 4; }
grep -E "scan_fetch_kb|scan_write_kb|over_algorithmic" $out/pmc_nt.log
timeout -k 10 120 python tools/time_c5.py > $out/c5_dp.txt 2>&1 || { echo c5 failed; cat $out/c5_dp.txt; exit 5; }
cat $out/c5_dp.txt
TENSILE_STREAMK_DATA_PARALLEL=0 timeout -k 10 120 python tools/time_c5.py > $out/c5_sk.txt 2>&1 || { echo c5 sk failed; cat $out/c5_sk.txt; exit 6; }
grep scaled_mm $out/c5_sk.txt
