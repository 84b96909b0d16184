"""Offline GEMM selection for the library GEMMs (hipBLASLt / rocBLAS via PyTorch TunableOp).

The dense projections of the towers stay plain library GEMMs.  Their default
hipBLASLt heuristic picks non-split-K tiles for the long-K weight gradients
(K = batch * tokens = 50432 at C2) and leaves most of the 256 CUs idle, so
the step loads a per-shape selection measured on MI355X (gfx950) once with
PYTORCH_TUNABLEOP_TUNING=1 (tools/tune_gemms.sh) and committed here.  Shapes
not in the file fall back to the default heuristic; nothing is tuned at run
time.
"""
import os
import tempfile

import torch

_DIR = os.path.dirname(os.path.abspath(__file__))
# C2 (b 256) and C3 (b 64) shapes, measured with the data-parallel grids the package sets
# (tools/tune_gemms.sh); MAMBA_CLIP_AMD_GEMM_TUNING_FILE overrides (A/B runs)
DEFAULT_FILE = os.environ.get("MAMBA_CLIP_AMD_GEMM_TUNING_FILE") or os.path.join(_DIR, "gemm_gfx950_dp.csv")


def load_gemm_tuning(path=DEFAULT_FILE):
    """Enable TunableOp in lookup-only mode with the committed selections; returns True if loaded."""
    if not (torch.cuda.is_available() and os.path.exists(path)):
        return False
    if os.environ.get("MAMBA_CLIP_AMD_NO_GEMM_TUNING"):
        return False
    tun = torch.cuda.tunable
    tun.set_filename(os.path.join(tempfile.gettempdir(), "mamba_clip_amd_tunableop%d.csv"))  # never write in-tree
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    return bool(tun.read_file(path))
