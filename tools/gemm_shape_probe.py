"""Same tile count (4096 tiles of 128x128), K = 16 fp8, different output row strides:
separates a per-tile cost tied to the C row stride (page crossings) from a plain per-tile cost."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd.ops import gemm_nt, quant_rows_fp8  # noqa: E402

for M, N in ((8192, 8192), (65536, 1024), (1024, 65536), (32768, 2048), (2048, 32768)):
    qa, sa = quant_rows_fp8(torch.randn(M, 16, device="cuda"))
    qb, sb = quant_rows_fp8(torch.randn(N, 16, device="cuda"))
    fn = lambda: gemm_nt(qa, qb, scale_a=sa, scale_b=sb)  # noqa: E731
    for _ in range(3):
        fn()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0.record()
    for _ in range(10):
        fn()
    t1.record()
    torch.cuda.synchronize()
    us = t0.elapsed_time(t1) / 10 * 1e3
    print(f"M={M} N={N} (row stride {N * 4 // 1024} KB): {us:.1f} us, write {M * N * 4 / us / 1e3:.0f} GB/s", flush=True)
