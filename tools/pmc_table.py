"""Dev tool: compare PMC counter means per variant directory (rocprofv3 --pmc CSVs).

usage: python tools/pmc_table.py <root> <kernel-substring> <variant-prefix>...
Per-wave numbers are counter / SQ_WAVES; SQ cycle counters are quad-cycles (x4).
"""
import collections
import csv
import glob
import sys

root, pat, variants = sys.argv[1], sys.argv[2], sys.argv[3:]
rows = {}
for v in variants:
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{root}/{v}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows[v] = {k: sum(x) / len(x) for k, x in vals.items()}
names = sorted(set().union(*[r.keys() for r in rows.values()]))
print(f"{'counter':26s}" + "".join(f"{v:>14s}" for v in variants))
for n in names:
    print(f"{n:26s}" + "".join(f"{rows[v].get(n, float('nan')):14.4g}" for v in variants))
for v in variants:
    r = rows[v]
    w = r.get("SQ_WAVES", 1)
    print(f"{v}: per wave: cycles {4 * r.get('SQ_WAVE_CYCLES', 0) / w:.4g}  valu-active {4 * r.get('SQ_ACTIVE_INST_VALU', 0) / w:.4g}"
          f"  wait-any {4 * r.get('SQ_WAIT_ANY', 0) / w:.4g}  wait-inst {4 * r.get('SQ_WAIT_INST_ANY', 0) / w:.4g}"
          f"  valu-insts {r.get('SQ_INSTS_VALU', 0) / w:.4g}  xcd-cycles {r.get('GRBM_GUI_ACTIVE', 0) / 8:.4g}")
