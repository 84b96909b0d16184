"""Dev tool: HIP-event time of mc_gemm_wgrad (ops.wgrad_hip, split-K slabs + mc_sum_slabs) at the C2
weight-gradient shapes; MC_WGRAD_SLAB_VEC=0 / 1 selects the slab epilogue (A/B in separate processes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd import ops  # noqa: E402

dev = "cuda"
SHAPES = [("vit_qkv", 2304, 768, 50432, False, False), ("vit_proj", 768, 768, 50432, False, False),
          ("vit_fc1", 3072, 768, 50432, False, False), ("vit_fc2", 768, 3072, 50432, False, False),
          ("mamba_in_proj", 3072, 768, 20480, True, True), ("mamba_out_proj", 768, 1536, 20480, False, True)]
tot = 0.0
for name, N, K, T, a_fm, b_fm in SHAPES:
    g = torch.Generator(device=dev).manual_seed(N + K)
    G = torch.randn(N, T, device=dev, generator=g).bfloat16() if a_fm else torch.randn(T, N, device=dev, generator=g).bfloat16().t()
    X = torch.randn(K, T, device=dev, generator=g).bfloat16().t() if b_fm else torch.randn(T, K, device=dev, generator=g).bfloat16()
    for _ in range(3):
        out = ops.wgrad_hip(G, X)
    ref = (G.float() @ X.float())
    err = float((out - ref).abs().max() / ref.abs().max())
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(10):
        ops.wgrad_hip(G, X)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 10 * 1e3
    tot += us
    print(f"{name:16s} {us:8.1f} us  {2 * N * K * T / us / 1e6:7.1f} TFLOP/s  rel err {err:.2e}", flush=True)
print(f"total {tot:.1f} us")
