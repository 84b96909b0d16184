"""Dev tool: the towers' weight-gradient GEMMs (dW = g^T x over the token dim, fp32 out, s slabs as
ops.wgrad) with each operand either as the forward leaves it (token-major rows) or as a contiguous
transposed copy (reduction dim contiguous).  Copies are made outside the timed region: this prices
the GEMM forms only.  HIP events, us per call, C2 shapes."""
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


def slabs(G, X, s):
    N, M = G.shape
    if s == 1:
        return torch.mm(G, X, out_dtype=torch.float32)
    Gs = G.unflatten(1, (s, M // s)).transpose(0, 1)
    Xs = X.unflatten(0, (s, M // s))
    return torch.bmm(Gs, Xs, out_dtype=torch.float32)


shapes = [("vit qkv", 50432, 2304, 768), ("vit proj", 50432, 768, 768), ("vit fc1", 50432, 3072, 768),
          ("vit fc2", 50432, 768, 3072), ("mamba in_proj", 20480, 3072, 768), ("mamba out_proj", 20480, 768, 1536),
          ("c3 vit fc1", 12608, 3072, 768), ("c3 vit qkv", 12608, 2304, 768)]
for name, M, N, K in shapes:
    g = torch.randn(M, N, device=dev, dtype=bf)
    x = torch.randn(M, K, device=dev, dtype=bf)
    gT = g.t().contiguous()          # (N, M)
    xT = x.t().contiguous()          # (K, M)
    forms = {"rows": (g.t(), x), "gT": (gT, x), "xT": (g.t(), xT.t()), "gT+xT": (gT, xT.t())}
    fl = 2 * M * N * K
    for fname, (G, X) in forms.items():
        res = []
        for s in (1, 2, 4, 8, 16):
            if M % s == 0:
                us = t(lambda s=s: slabs(G, X, s))
                res.append(f"s{s} {us:6.1f} ({fl / us / 1e6:4.0f})")
        print(f"{name:14s} {fname:6s} N{N} K{K} M{M}: " + " | ".join(res), flush=True)
    del g, x, gT, xT
