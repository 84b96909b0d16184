"""fp8 / bf16 gemm_nt at N = 8192 over K: separates the logit-write floor (small K) from the K loop."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd.ops import gemm_nt, quant_rows_fp8  # noqa: E402

n = 8192
for K in (16, 64, 128, 256, 512, 1024):
    A = torch.randn(n, K, device="cuda")
    qa, sa = quant_rows_fp8(A)
    res = []
    for name, fn in (("fp8", lambda: gemm_nt(qa, qa, scale_a=sa, scale_b=sa)),
                     ("bf16", lambda: gemm_nt(A.bfloat16(), A.bfloat16())),
                     ("fp8->bf16 out", lambda: gemm_nt(qa, qa, scale_a=sa, scale_b=sa, out_dtype=torch.bfloat16))):
        for _ in range(3):
            fn()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0.record()
        for _ in range(10):
            fn()
        t1.record()
        torch.cuda.synchronize()
        res.append(f"{name} {t0.elapsed_time(t1) / 10 * 1e3:.1f} us")
    print(f"K={K}: " + ", ".join(res), flush=True)
