"""Workload for the HBM-traffic PMC passes of the roofline kernel (run under rocprofv3 --pmc).

Runs (1) a calibration stream: a 2 GiB bf16 tensor clone (known bytes: 2 GiB
read + 2 GiB written) and (2) the C4 selective_scan forward (bench.py's
roofline call).  tools/pmc_traffic.sh collects FETCH_SIZE and WRITE_SIZE in
separate passes and tools/pmc_traffic_report.py turns them into per-launch
HBM bytes, calibrating the read side on the clone (MI355X_MICROARCH.md: on
gfx950 FETCH_SIZE under-counts wide streaming reads; calibrate on a known
byte count).
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

calib = torch.empty(1 << 30, dtype=torch.bfloat16, device="cuda").normal_()
for _ in range(3):
    c = calib.clone()
    del c
torch.cuda.synchronize()
del calib
torch.cuda.empty_cache()
r = bench.scan_roofline(iters=3, warmup=1)
print("scan ms/call", r["ms_per_call"])
