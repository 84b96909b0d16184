"""mamba_clip_amd -- MI355X-native hot path of psmyth94/mamba-clip.

Host layer in Python (mirrors the reference's operator/module surface) over
the C ABI of libmamba_clip_amd.so (include/*.h), whose kernels are hand-written
HIP for gfx950.  See DESIGN.md.
"""
import os as _os
import sys as _sys

__version__ = "0.1.0"

# Library GEMM grids.  hipBLASLt's gfx950 GEMM kernels are stream-K builds (_SK3_):
# by default a launch may run fewer workgroups than output tiles and split a tile's K range over
# several workgroups, the first of which waits for the others' partial sums -- so every workgroup of
# the launch must be co-resident.  Two such launches on two streams can each hold part of the CUs and
# wait forever (the round-3 C3 hang).  TENSILE_STREAMK_DATA_PARALLEL=1 makes hipBLASLt launch one
# workgroup per tile (tools/sk_probe.sh, profiles/r04/sk_probe/: with it 0 of the 440 C2 / 299 C3
# step GEMM dispatches split a tile's K range, against 36 / 13 by default -- the sweeps' larger
# 253 / 121 counts also include stream-K launches that run whole tiles -- GEMM time unchanged), and
# then no GEMM workgroup waits on another.
# hipBLASLt reads the variable once, on its first GEMM, so it is set here, before this process can
# have run one -- unless CUDA was already live at import, in which case it may be too late.
_SK_ENV = "TENSILE_STREAMK_DATA_PARALLEL"
_sk_preset = _os.environ.get(_SK_ENV)
_os.environ.setdefault(_SK_ENV, "1")
_torch = _sys.modules.get("torch")
_cuda_live = bool(_torch is not None and _torch.cuda.is_initialized())

#: True when every library GEMM of this process launches data-parallel (no co-residency
#: dependence): the condition for running ClipModel's two towers on two HIP streams.
GEMM_GRIDS_DATA_PARALLEL = _os.environ.get(_SK_ENV) == "1" and (_sk_preset == "1" or not _cuda_live)
