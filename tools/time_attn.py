"""Dev tool: fused attention (mc_attn) vs torch SDPA at a tower shape, HIP events (not the bench contract).

usage: python tools/time_attn.py [--shape B,N,H] [--iters 20]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd.model import _gpu_sdpa_backends  # noqa: E402
from mamba_clip_amd.ops import packed_attention  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="256,197,12")
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
B, N, H = map(int, args.shape.split(","))
D, C = 64, H * 64
dev = "cuda"
qkv = torch.randn(B, N, 3 * C, device=dev, dtype=torch.bfloat16).requires_grad_(True)
go = torch.randn(B, N, C, device=dev, dtype=torch.bfloat16)


def fused(bwd):
    o = packed_attention(qkv, H)
    if bwd:
        o.backward(go)


def sdpa(bwd):
    q, k, v = qkv.view(B, N, 3, H, D).unbind(2)
    with _gpu_sdpa_backends():
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2))
    o = o.transpose(1, 2).reshape(B, N, C)
    if bwd:
        o.backward(go)


def t(fn, bwd):
    for _ in range(3):
        fn(bwd)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(args.iters):
        fn(bwd)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / args.iters


io_fwd = (B * N * 3 * C + B * N * C) * 2
for name, fn in (("fused", fused), ("sdpa", sdpa)):
    f = t(fn, False)
    fb = t(fn, True)
    print(f"{name:6s} B{B} N{N} H{H}: fwd {f * 1e3:.1f} us ({io_fwd / f / 1e6:.0f} GB/s of q,k,v,o)  "
          f"fwd+bwd {fb * 1e3:.1f} us  bwd {(fb - f) * 1e3:.1f} us", flush=True)
