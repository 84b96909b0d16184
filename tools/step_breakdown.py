"""Per-training-step kernel breakdown from a rocprofv3 --kernel-trace CSV of bench.py.

usage: python tools/step_breakdown.py <kernel_trace.csv> [top]
A step is delimited by the fused-AdamW multi_tensor_apply launches.
"""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "multi_tensor_apply" in r["Kernel_Name"]]
groups = []
for i in idx:
    if groups and i - groups[-1][-1] <= 2:
        groups[-1].append(i)
    else:
        groups.append([i])
a, b = groups[-3][-1] + 1, groups[-2][-1] + 1
seq = rows[a:b]
agg = defaultdict(lambda: [0, 0.0])
for r in seq:
    n = re.sub(r"void |at::native::|\(anonymous namespace\)::", "", r["Kernel_Name"])[:110]
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
busy = sum(v[1] for v in agg.values())
wall = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
print(f"kernels {len(seq)}  busy {busy / 1e3:.2f} ms  wall {wall / 1e3:.2f} ms")
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{t / 1e3:7.2f} ms {c:5d} {t / c:8.1f} us  {n}")
