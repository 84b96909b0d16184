"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel (matching a substring)."""
import csv
import glob
import sys
from collections import defaultdict

root, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "scan_fwd")
vals = defaultdict(list)
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        if pat in row.get("Kernel_Name", ""):
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
# several rows per dispatch (per XCD/SE dims are summed already by rocprofv3?) -> report per-dispatch mean
for k, v in sorted(vals.items()):
    print(f"{k:32s} n={len(v):4d} mean={sum(v)/len(v):.4g}")
for f in glob.glob(f"{root}/trace/*kernel_stats.csv"):
    for row in csv.DictReader(open(f)):
        if pat in row["Name"]:
            print("avg duration us:", float(row["AverageNs"]) / 1e3, "calls", row["Calls"])
