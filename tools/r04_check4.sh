#!/bin/bash
# Round-4 check 4: SS2D fused cross-scan glue -- kernel tests, the reference goldens (ss2d_*, VSSM),
# block timing fused vs reference construction, and the kernel list of one fused SS2D fwd+bwd.
set -u
out=gpurun_out/r04c4; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ss2d_gpu.py \
    "tests/test_model_gpu.py::test_ss2d_matches_reference_golden" "tests/test_model_gpu.py::test_ss_conv_ssm_matches_reference_golden" \
    "tests/test_model_gpu.py::test_ss2d_c1_shape_matches_reference_golden" "tests/test_model_gpu.py::test_vssm_tiny_matches_reference_golden" \
    tests/test_scan_gpu.py > $out/pytest.log 2>&1 || { echo pytest failed; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python tools/ss2d_block.py > $out/block.txt 2>&1 || { echo block timing failed; tail -20 $out/block.txt; exit 2; }
cat $out/block.txt
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o k -- python tools/ss2d_block.py --trace > $out/trace.log 2>&1 || { echo trace failed; tail -20 $out/trace.log; exit 3; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04c4/trace/*kernel_trace.csv")[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
m = [i for i, r in enumerate(rows) if "spin" in r["Kernel_Name"].lower() or "sleep" in r["Kernel_Name"].lower()]
seg = rows[m[-2] + 1: m[-1]]
with open("gpurun_out/r04c4/ss2d_kernels.txt", "w") as o:
    o.write("one fused SS2D fwd+bwd (B 32, 56x56, d_model 32, fp32), kernels in launch order:\n")
    for r in seg:
        o.write("%8.1f us  %s\n" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Kernel_Name"][:150]))
print(open("gpurun_out/r04c4/ss2d_kernels.txt").read())
PY
