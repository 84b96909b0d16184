import os, sys, torch
sys.path.insert(0, "/root/repo/mamba-clip_amd")
from mamba_clip_amd.ops import gemm_nt, quant_rows_fp8
for n in (8192, 8064, 8128, 8256, 8320, 4096, 16384):
    A = torch.randn(n, 16, device="cuda"); qa, sa = quant_rows_fp8(A)
    fn = lambda: gemm_nt(qa, qa, scale_a=sa, scale_b=sa)
    for _ in range(3): fn()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); t0.record()
    for _ in range(10): fn()
    t1.record(); torch.cuda.synchronize()
    us = t0.elapsed_time(t1) / 10 * 1e3
    print(f"N={n} K=16 fp8: {us:.1f} us  write {n*n*4/us/1e3:.0f} GB/s", flush=True)
