set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ae_prof -o step -- python3 tools/one_step.py > gpurun_out/ae.log 2>&1; echo "rc=$?"
f=$(find gpurun_out/ae_prof -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
n = len(rows) // 3
c = collections.Counter()
for r in rows[-n:]:
    k = r["Kernel_Name"]
    if "reduce_kernel" in k or "Reduce" in k or "lookback" in k or "scan_kernel" in k:
        c[(k[:140], r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"], r["Workgroup_Size_Y"])] += 1
for k, v in c.items():
    print(v, k)
PY
echo done
