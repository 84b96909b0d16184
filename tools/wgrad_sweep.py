"""Dev tool: split factor sweep of the towers' weight-gradient GEMMs (ops.wgrad's formulation:
strided-batched bf16 GEMM with fp32 output over s slabs of the token dim, then a sum), C2 shapes,
with the committed TunableOp selection loaded as in bench.py.  HIP events, us per call."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd.tuning import load_gemm_tuning  # noqa: E402

load_gemm_tuning()
dev, bf = "cuda", torch.bfloat16


def t(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def wg(G, X, s):
    N, M = G.shape
    if s == 1:
        return torch.mm(G, X).float()
    Gs = G.unflatten(1, (s, M // s)).transpose(0, 1)
    Xs = X.unflatten(0, (s, M // s))
    return torch.bmm(Gs, Xs, out_dtype=torch.float32).sum(0)


def wg_t(G, X, s):
    """the transposed product X^T G (K x N) per slab, summed, transposed back"""
    N, M = G.shape
    Xs = X.unflatten(0, (s, M // s)).transpose(1, 2)        # (s, K, M/s)
    Gs = G.t().unflatten(0, (s, M // s))                    # (s, M/s, N)
    return torch.bmm(Xs, Gs, out_dtype=torch.float32).sum(0).t().contiguous()


shapes = [("vit qkv", 50432, 2304, 768), ("vit proj", 50432, 768, 768), ("vit fc1", 50432, 3072, 768),
          ("vit fc2", 50432, 768, 3072), ("patch", 50176, 768, 768),
          ("mamba in_proj", 20480, 3072, 768), ("mamba out_proj", 20480, 768, 1536),
          ("mamba x_proj", 20480, 80, 1536), ("mamba dt_proj", 20480, 1536, 48)]
for name, M, N, K in shapes:
    g = torch.randn(M, N, device=dev, dtype=bf)   # gradient rows (tokens x out)
    x = torch.randn(M, K, device=dev, dtype=bf)   # input rows (tokens x in)
    G = g.t()
    res = []
    for s in (1, 2, 4, 8, 16):
        if M % s == 0:
            us = t(lambda s=s: wg(G, x, s))
            res.append(f"s{s} {us:6.1f} us ({2 * M * N * K / us / 1e6:5.0f} TF/s)")
            if "--t" in sys.argv:
                ut = t(lambda s=s: wg_t(G, x, s))
                res.append(f"T{s} {ut:6.1f}")
    print(f"{name:15s} N{N} K{K} M{M}: " + " | ".join(res), flush=True)
