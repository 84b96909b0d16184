"""Per-step stream overlap from a rocprofv3 kernel trace of bench.py (two-stream towers).

usage: python tools/stream_overlap.py <kernel_trace.csv>
Steps are delimited by the fused-AdamW launches.  Prints, for the second-to-last full step: wall,
busy time per HIP queue, the time both queues had a kernel running, and the time only one did.
"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "multi_tensor_apply" in r["Kernel_Name"]]
groups = []
for i in idx:
    if groups and i - groups[-1][-1] <= 2:
        groups[-1].append(i)
    else:
        groups.append([i])
a, b = groups[-3][-1] + 1, groups[-2][-1] + 1
seq = rows[a:b]
t0 = int(seq[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in seq)
ivs = defaultdict(list)
for r in seq:
    ivs[r.get("Queue_Id", "0")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def total(iv):
    return sum(e - s for s, e in iv)


u = {q: union(v) for q, v in ivs.items()}
print(f"step wall {(t1 - t0) / 1e6:.2f} ms, {len(seq)} kernels")
for q, v in sorted(u.items()):
    print(f"  queue {q}: {len(ivs[q])} kernels, busy {total(v) / 1e6:.2f} ms")
allu = union([x for v in ivs.values() for x in v])
print(f"  any queue busy {total(allu) / 1e6:.2f} ms, idle {((t1 - t0) - total(allu)) / 1e6:.2f} ms")
qs = sorted(u)
if len(qs) >= 2:
    both = 0
    A, B = u[qs[0]], u[qs[1]]
    i = j = 0
    while i < len(A) and j < len(B):
        s, e = max(A[i][0], B[j][0]), min(A[i][1], B[j][1])
        if s < e:
            both += e - s
        if A[i][1] < B[j][1]:
            i += 1
        else:
            j += 1
    print(f"  both queues busy {both / 1e6:.2f} ms")
    # last kernel end per queue: who finishes the step
    for q in qs:
        print(f"  queue {q} last kernel ends at +{(max(e for _, e in ivs[q]) - t0) / 1e6:.2f} ms")
