#!/bin/bash
# HBM traffic and L2 hit rate of the scan backward at one shape (run on the GPU box).
#   usage: tools/pmc_bwd_traffic.sh <outdir> <shape>
set -u
out=$1; shp=$2; mkdir -p "$out"
export TMPDIR=/tmp
for pass in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass -d "$out/$tag" -o p --output-format csv \
    -- python tools/time_scan.py --shape $shp --iters 3 --bwd > "$out/$tag.log" 2>&1 || { echo "pass $tag failed"; exit 1; }
done
python - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(f"{out}/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "scan" in k or "relayout" in k:
            acc[(k[:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:60s} {c:14s} {sum(v)/len(v):14.4g}")
PY
