"""mamba_clip_amd -- MI355X-native hot path of psmyth94/mamba-clip.

Host layer in Python (mirrors the reference's operator/module surface) over
the C ABI of libmamba_clip_amd.so (include/*.h), whose kernels are hand-written
HIP for gfx950.  See DESIGN.md.
"""
__version__ = "0.1.0"
