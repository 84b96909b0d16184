"""SS2D core: flips inside the kernels' addressing (grouped_scan_fn, u = [x, x^T]) vs the reference's explicit
stack / flip / transpose copies around selective_scan_fn (model.py:510-565), fwd + bwd.

    python tools/time_ss2d.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd.selective_scan_interface import grouped_scan_fn, selective_scan_fn  # noqa: E402


def explicit(x, dts, A, Bs, Cs, D, bias, H, W):
    Bsz, d, L = x.shape
    x4 = x.view(Bsz, d, H, W)
    x_hw, x_wh = x, x4.transpose(2, 3).reshape(Bsz, d, L)
    xs = torch.stack([x_hw, x_wh, x_hw.flip(-1), x_wh.flip(-1)], 1).reshape(Bsz, 4 * d, L)
    # per-direction delta / B / C already in scan order in the reference (computed from xs)
    out = selective_scan_fn(xs, dts, A, Bs, Cs, D, None, bias, delta_softplus=True).view(Bsz, 4, d, L)
    y_inv = out[:, 2:4].flip(-1)
    y_wh = out[:, 1].reshape(Bsz, d, W, H).transpose(2, 3).reshape(Bsz, d, L)
    y_invwh = y_inv[:, 1].reshape(Bsz, d, W, H).transpose(2, 3).reshape(Bsz, d, L)
    return out[:, 0] + y_inv[:, 0] + y_wh + y_invwh


def fused(x, dts, A, Bs, Cs, D, bias, H, W):
    Bsz, d, L = x.shape
    u = torch.stack([x, x.view(Bsz, d, H, W).transpose(2, 3).reshape(Bsz, d, L)], 1).view(Bsz, 2 * d, L)
    out = grouped_scan_fn(u, dts, A, Bs, Cs, D, bias, True, 0b1100, 2).view(Bsz, 4, d, L)
    return out[:, 0] + out[:, 2] + (out[:, 1] + out[:, 3]).view(Bsz, d, W, H).transpose(2, 3).reshape(Bsz, d, L)


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for (Bsz, d, H, W) in [(32, 64, 56, 56), (32, 128, 28, 28), (32, 256, 14, 14)]:
    L, N = H * W, 16
    x = torch.randn(Bsz, d, L, device="cuda", requires_grad=True)
    dts = (0.5 * torch.randn(Bsz, 4 * d, L, device="cuda")).requires_grad_(True)
    A = -torch.exp(torch.log(torch.arange(1, N + 1, device="cuda").float()).repeat(4 * d, 1))
    Bs = torch.randn(Bsz, 4, N, L, device="cuda", requires_grad=True)
    Cs = torch.randn(Bsz, 4, N, L, device="cuda", requires_grad=True)
    D = torch.ones(4 * d, device="cuda")
    bias = torch.rand(4 * d, device="cuda") * 4 - 5
    gy = torch.randn(Bsz, d, L, device="cuda")
    res = {}
    for name, f in (("explicit copies", explicit), ("flip-free grouped scan", fused)):
        res[name] = timed(lambda: f(x, dts, A, Bs, Cs, D, bias, H, W).backward(gy))
    print(f"B{Bsz} d{d} {H}x{W} fp32 fwd+bwd: " + ", ".join(f"{k} {v:.3f} ms" for k, v in res.items()))

# the scan alone: plain vs grouped addressing (isolates the kernels' mirrored / shared-u costs)
for (Bsz, d, H, W) in [(32, 64, 56, 56)]:
    L, N = H * W, 16
    u4 = torch.randn(Bsz, 4 * d, L, device="cuda", requires_grad=True)
    u2 = torch.randn(Bsz, 2 * d, L, device="cuda", requires_grad=True)
    dts = (0.5 * torch.randn(Bsz, 4 * d, L, device="cuda")).requires_grad_(True)
    A = -torch.exp(torch.log(torch.arange(1, N + 1, device="cuda").float()).repeat(4 * d, 1))
    Bs = torch.randn(Bsz, 4, N, L, device="cuda", requires_grad=True)
    Cs = torch.randn(Bsz, 4, N, L, device="cuda", requires_grad=True)
    D = torch.ones(4 * d, device="cuda")
    bias = torch.rand(4 * d, device="cuda") * 4 - 5
    gy = torch.randn(Bsz, 4 * d, L, device="cuda")
    cases = [("plain selective_scan_fn", lambda: selective_scan_fn(u4, dts, A, Bs, Cs, D, None, bias, True)),
             ("grouped rev=0000 u_groups=4", lambda: grouped_scan_fn(u4, dts, A, Bs, Cs, D, bias, True, 0, 4)),
             ("grouped rev=1100 u_groups=4", lambda: grouped_scan_fn(u4, dts, A, Bs, Cs, D, bias, True, 0b1100, 4)),
             ("grouped rev=1100 u_groups=2", lambda: grouped_scan_fn(u2, dts, A, Bs, Cs, D, bias, True, 0b1100, 2))]
    for name, f in cases:
        tf = timed(lambda: f())
        tb = timed(lambda: f().backward(gy))
        print(f"B{Bsz} 4x{d} L{L} {name}: fwd {tf:.3f} ms, fwd+bwd {tb:.3f} ms")
