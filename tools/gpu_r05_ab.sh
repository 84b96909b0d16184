set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_prof -o sum0 -- python3 tools/sum0_probe.py > gpurun_out/ab.log 2>&1; echo "rc=$?"; tail -2 gpurun_out/ab.log
f=$(find gpurun_out/ab_prof -name "*kernel_trace.csv" | head -1); echo $f
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Kernel_Name"]
    if "reduce" in n or "Reduce" in n:
        print(n[:110], r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Workgroup_Size_X"), r.get("Workgroup_Size_Y"), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
PY
echo done
