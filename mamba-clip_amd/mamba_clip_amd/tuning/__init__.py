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
# per-model selections where a step A/B chose another file: the C3 pair, re-tuned with the transposed-
# weight input gradients' shapes (profiles/r04/gemm_tuning_tn_ab.txt: C3 25.95 -> 25.60 ms; the same
# merged file costs C2 0.8 ms, so C2 keeps the default)
MODEL_FILES = {"biomedclip-vit_b16-pubmedbert256": os.path.join(_DIR, "gemm_gfx950_dp_c3.csv")}


def tuning_file(model=None):
    if os.environ.get("MAMBA_CLIP_AMD_GEMM_TUNING_FILE"):
        return os.environ["MAMBA_CLIP_AMD_GEMM_TUNING_FILE"]
    return MODEL_FILES.get(model, DEFAULT_FILE)


def load_gemm_tuning(path=None, model=None):
    """Enable TunableOp in lookup-only mode with the committed selections (the model's file, else the
    default); returns True if loaded."""
    path = path or tuning_file(model)
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
