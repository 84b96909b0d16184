"""ISA guards for the scan pair kernels (CPU: hipcc cross-compiles gfx950 assembly, no GPU needed).

* No packed-fp32 op with op_sel[src] = 1 (the low result reading a source's high half) in any kernel of
  scan_fwd_pair.hip / scan_bwd_pair.hip: that form, issued from inline asm, made the two-stream
  training step non-reproducible; scan_common.h rejects it at compile time in our own
  helpers and this test also catches the compiler choosing it.
* The fine-state backward instances (the C2 / C4 training path) and every forward pair instance run
  without VGPR spills.
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _asm(src, tmp_path):
    out = tmp_path / (os.path.basename(src) + ".s")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                    os.path.join(ROOT, "mamba-clip_amd", "csrc", src), "-o", str(out)],
                   check=True, capture_output=True, timeout=600)
    return str(out)


def _spills(path):
    text = open(path).read()
    out = {}
    for m in re.finditer(r"\.name:\s+(\S+)\s*\n(.*?)\.vgpr_spill_count:\s+(\d+)", text, re.S):
        out[m.group(1)] = int(m.group(3))
    return out


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
@pytest.mark.parametrize("src", ["scan_fwd_pair.hip", "scan_bwd_pair.hip"])
def test_scan_pair_kernels_have_no_packed_opsel_high_broadcast(src, tmp_path):
    import hazard_scan
    path = _asm(src, tmp_path)
    bad = [f for f in hazard_scan.main(path) if f[0] == "pk_f32 op_sel hi->lo"]
    assert not bad, [(f[1][:80], f[3]) for f in bad[:4]]
    spills = _spills(path)
    assert spills, "no kernel metadata found"
    if src == "scan_fwd_pair.hip":
        hot = {k: v for k, v in spills.items() if "scan_fwd_pair_kernel" in k}
    else:   # <TI, softplus, z, projected delta, fine>: the fine instances end in Lb1EEE
        hot = {k: v for k, v in spills.items() if "scan_bwd_pair_kernel" in k and k.endswith("Lb1EEEvNS0_11BwdPairArgsE")}
    assert hot, sorted(spills)[:4]
    assert all(v == 0 for v in hot.values()), {k: v for k, v in hot.items() if v}
