"""Per-training-step kernel breakdown from a rocprofv3 --kernel-trace CSV of bench.py.

usage: python tools/step_breakdown.py <kernel_trace.csv> [top]

A step is delimited by the optimizer launch that ends it: the one-launch HipAdamW (`adamw_kernel`), or
torch's fused AdamW (`multi_tensor_apply` groups) in runs that use it.  The step between the
second-to-last and the last delimiter is reported: its kernels on ALL queues (the towers run on two
HIP streams), busy time per queue, the wall time from its first kernel start to its last kernel end,
and the top kernels by total time.
"""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
if len(idx) < 2:   # torch's fused AdamW: groups of multi_tensor_apply launches
    ids = [i for i, r in enumerate(rows) if "multi_tensor_apply" in r["Kernel_Name"]]
    groups = []
    for i in ids:
        if groups and i - groups[-1][-1] <= 2:
            groups[-1].append(i)
        else:
            groups.append([i])
    idx = [g[-1] for g in groups]
if len(idx) < 2:
    sys.exit("fewer than two optimizer launches in the trace: no complete step")
a, b = idx[-2] + 1, idx[-1] + 1
seq = rows[a:b]
agg = defaultdict(lambda: [0, 0.0])
per_queue = defaultdict(float)
for r in seq:
    n = re.sub(r"void |at::native::|\(anonymous namespace\)::", "", r["Kernel_Name"])[:110]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[n][0] += 1
    agg[n][1] += d
    per_queue[r.get("Queue_Id", "?")] += d
busy = sum(v[1] for v in agg.values())
wall = (int(max(int(r["End_Timestamp"]) for r in seq)) - int(seq[0]["Start_Timestamp"])) / 1e3
print(f"one training step, all queues: kernels {len(seq)}  kernel-busy sum {busy / 1e3:.2f} ms  "
      f"wall {wall / 1e3:.2f} ms")
print("busy per queue: " + ", ".join(f"queue {q}: {t / 1e3:.2f} ms" for q, t in sorted(per_queue.items())))
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{t / 1e3:8.2f} ms  {c:5d}  {t / c:9.1f} us  {n}")
qagg = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))
for r in seq:
    n = re.sub(r"void |at::native::|\(anonymous namespace\)::", "", r["Kernel_Name"])[:110]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    e = qagg[r.get("Queue_Id", "?")][n]
    e[0] += 1
    e[1] += d
for q, kern in sorted(qagg.items()):
    print(f"\nqueue {q}: busy {per_queue[q] / 1e3:.2f} ms")
    for n, (c, t) in sorted(kern.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{t / 1e3:8.2f} ms  {c:5d}  {t / c:9.1f} us  {n}")
