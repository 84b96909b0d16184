"""Join tools/sk_probe.py's GEMM call log with a rocprofv3 kernel trace of the same run.

usage: python tools/sk_probe_report.py <kernel_trace.csv> <calls.json> [--label X]
Prints, per library GEMM dispatch of the step: op, output shape (batch, M, N), tower (from the token
count), kernel macro tile, whether the kernel name carries a stream-K tag (_SK<n>_), the launched
workgroup count and the output tile count.  A grid equal to the tile count is a data-parallel launch:
every workgroup owns whole tiles and none waits on another; fewer workgroups than tiles on an _SK
kernel is a stream-K launch (partial tiles fixed up across workgroups -> needs co-residency).
"""
import csv
import json
import math
import re
import sys

trace, calls_path = sys.argv[1], sys.argv[2]
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "spin" in r["Kernel_Name"].lower() or "sleep" in r["Kernel_Name"].lower()]
if len(marks) < 2:
    sys.exit(f"expected two spin-kernel markers, found {len(marks)}")
seg = rows[marks[-2] + 1: marks[-1]]
gemms = [r for r in seg if "Cijk_" in r["Kernel_Name"]]
log = json.load(open(calls_path))
calls = log["calls"]
print(f"model {log['model']} batch {log['batch']} tuned {log['tuned']} env {log['env']}")
# the run's tag names the grid mode it meant to measure (c*_default / c*_dp): flag a mismatch (the
# package sets TENSILE_STREAMK_DATA_PARALLEL=1 at import when the variable is unset)
_dp = log["env"].get("TENSILE_STREAMK_DATA_PARALLEL")
if "_default" in calls_path and _dp != "0":
    print(f"WARNING: default-grid leg ran with TENSILE_STREAMK_DATA_PARALLEL={_dp!r} (expected '0')")
if "_dp" in calls_path and _dp != "1":
    print(f"WARNING: data-parallel leg ran with TENSILE_STREAMK_DATA_PARALLEL={_dp!r} (expected '1')")
print(f"{len(gemms)} GEMM dispatches in the step, {len(calls)} aten GEMM calls logged")

TOWER = {}


def tower_of(dims):
    tok = {50432: "vit", 50176: "vit(patch)", 12608: "vit", 12544: "vit(patch)", 20480: "mamba", 16384: "bert"}
    for d in dims:
        if d in tok:
            return tok[d]
        for t, name in tok.items():
            if d * 16 == t or d * 8 == t or d * 4 == t:   # split-K slabs of a token dim
                return name + "(splitK)"
    return "head/loss"


def out_shape(c):
    s = c["shapes"]
    op = c["op"].split(".")[0]
    if op in ("mm", "_scaled_mm"):
        return 1, s[0][0], s[1][1]
    if op in ("addmm", "addmm_"):
        return 1, s[1][0], s[2][1]
    if op in ("bmm",):
        return s[0][0], s[0][1], s[1][2]
    if op in ("baddbmm",):
        return s[1][0], s[1][1], s[2][2]
    return 1, -1, -1


def wgs(r):
    n = 1
    for ax in "XYZ":
        g, w = int(r[f"Grid_Size_{ax}"]), int(r[f"Workgroup_Size_{ax}"])
        n *= max(1, math.ceil(g / max(w, 1)))
    return n


# map kernels to calls: by order on one stream; per stream (HIP queue <-> logged stream) otherwise
order = list(range(len(gemms)))
queues = sorted({r.get("Queue_Id", "0") for r in gemms})
streams = sorted({c["stream"] for c in calls})
call_of = {}
if len(queues) > 1 or len(streams) > 1:
    kq = {q: [i for i, r in enumerate(gemms) if r.get("Queue_Id", "0") == q] for q in queues}
    cs = {s_: [j for j, c in enumerate(calls) if c["stream"] == s_] for s_ in streams}
    used = set()
    for q, ks in kq.items():
        match = [s_ for s_ in streams if len(cs[s_]) == len(ks) and s_ not in used]
        if not match:
            sys.exit(f"queue {q}: {len(ks)} GEMM kernels, no logged stream with that many calls "
                     f"({ {s_: len(v) for s_, v in cs.items()} })")
        used.add(match[0])
        for i, j in zip(ks, cs[match[0]]):
            call_of[i] = j
    print("per-stream match:", {q: len(ks) for q, ks in kq.items()})
else:
    call_of = {i: i for i in range(min(len(gemms), len(calls)))}
n_sk_partial = 0
print(f"{'#':>3} {'op':10} {'b':>3} {'M':>6} {'N':>6} {'K':>6} {'tower':14} {'MT':14} {'SK':4} {'queue':>5} {'WGs':>6} "
      f"{'tiles':>6} mode")
for i, r in enumerate(gemms):
    name = r["Kernel_Name"]
    mt = re.search(r"MT(\d+)x(\d+)x(\d+)", name)
    sk = re.search(r"_SK(\d+)_", name)
    gsu = re.search(r"_GSU(\d+)", name)
    c = calls[call_of[i]] if i in call_of else None
    b, M, N = out_shape(c) if c else (0, -1, -1)
    K = -1
    if c:
        sh = c["shapes"]
        op = c["op"].split(".")[0]
        K = sh[0][1] if op in ("mm", "_scaled_mm") else (sh[1][1] if op.startswith("addmm") else sh[-1][-2] if op.endswith("bmm") else -1)
    t0, t1 = (int(mt.group(1)), int(mt.group(2))) if mt else (0, 0)
    tiles = b * math.ceil(N / t0) * math.ceil(M / t1) if (mt and M > 0) else -1   # BLAS view: C^T is N x M
    tiles_sw = b * math.ceil(M / t0) * math.ceil(N / t1) if (mt and M > 0) else -1
    w = wgs(r)
    if tiles > 0 and w in (tiles, tiles_sw):
        mode = "data-parallel"
    elif tiles > 0 and (tiles % w == 0 or tiles_sw % w == 0):
        mode = "persistent, whole tiles per workgroup"
    elif gsu and tiles > 0 and w in (tiles * int(gsu.group(1)), tiles_sw * int(gsu.group(1))):
        mode = f"GSU{gsu.group(1)}"
    else:
        mode = "STREAM-K (grid != tiles)" if sk else "?"
        if sk:
            n_sk_partial += 1
    print(f"{i:3d} {c['op'] if c else '?':10} {b:3d} {M:6d} {N:6d} {K:6d} {tower_of([M, N, K]) if c else '?':14} "
          f"{(mt.group(0) if mt else '-'):14} {(sk.group(1) if sk else '-'):4} {r.get('Queue_Id', '?'):>5} {w:6d} "
          f"{max(tiles, tiles_sw) if tiles > 0 else -1:6d} {mode}")
print(f"stream-K launches (grid != tile count): {n_sk_partial} of {len(gemms)}")
