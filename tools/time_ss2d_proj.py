"""Dev tool: SS2D's x_proj / dt_proj einsums (model.py:519-528; model.SS2D._scan_u) fwd+bwd in fp32 at the
medmamba stage shapes (B 32): torch.einsum as written vs broadcast matmuls on the u = [x, x^T] layout
(no operand permutes).  Prints us per fwd+bwd and the max relative difference between the two."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
dev = "cuda"


def einsum_form(u, w, wdt, R, N):
    Bsz, _, d, L = u.shape
    x_dbl = torch.einsum("bjdl,ijcd->bijcl", u, w.view(2, 2, -1, d)).reshape(Bsz, 4, -1, L)
    dts, Bs, Cs = torch.split(x_dbl, [R, N, N], dim=2)
    return torch.einsum("bkrl,kdr->bkdl", dts, wdt), Bs, Cs


def matmul_form(u, w, wdt, R, N):
    Bsz, _, d, L = u.shape
    w4 = w.view(2, 2, -1, d)                                           # [i][j]: direction k = 2 i + j
    x_dbl = torch.stack([torch.matmul(w4[0], u), torch.matmul(w4[1], u)], dim=1).reshape(Bsz, 4, -1, L)
    dts, Bs, Cs = torch.split(x_dbl, [R, N, N], dim=2)
    return torch.matmul(wdt, dts), Bs, Cs


def group_form(u, w, wdt, R, N):
    from mamba_clip_amd.ops import ss2d_proj
    return ss2d_proj(u, w, wdt, R, N)


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


STAGES = [(56, 32), (28, 64), (14, 128), (7, 256)]
only = os.environ.get("STAGE")          # e.g. STAGE=56 for one stage (profiling)
forms = os.environ.get("FORMS", "einsum,matmul,group").split(",")
for (hw, dm) in [s for s in STAGES if only is None or s[0] == int(only)]:
    Bsz, d, L, N = 32, 2 * dm, hw * hw, 16
    R = -(-dm // 16)
    g = torch.Generator(device=dev).manual_seed(hw)
    u = torch.randn(Bsz, 2, d, L, device=dev, generator=g).requires_grad_(True)
    w = (torch.randn(4, R + 2 * N, d, device=dev, generator=g) * d ** -0.5).requires_grad_(True)
    wdt = (torch.randn(4, d, R, device=dev, generator=g) * R ** -0.5).requires_grad_(True)
    gd = torch.randn(Bsz, 4, d, L, device=dev, generator=g)
    gb = torch.randn(Bsz, 4, N, L, device=dev, generator=g)
    gc = torch.randn(Bsz, 4, N, L, device=dev, generator=g)
    res = {}
    for name, f in [x for x in (("einsum", einsum_form), ("matmul", matmul_form), ("group", group_form)) if x[0] in forms]:
        def step():
            u.grad = w.grad = wdt.grad = None
            outs = f(u, w, wdt, R, N)
            torch.autograd.backward(outs, [gd, gb, gc])
        us = timed(step)
        step()
        res[name] = (us, [t.detach().clone() for t in f(u, w, wdt, R, N)] + [u.grad.clone(), w.grad.clone(), wdt.grad.clone()])
    ref = res.get("einsum")
    diffs = {k: max(float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(v[1], ref[1]))
             for k, v in res.items() if ref is not None and k != "einsum"}
    print(f"{hw}x{hw} d_inner {d}: " + ", ".join(f"{k} {v[0]:.1f} us" for k, v in res.items())
          + "".join(f", {k} max rel diff {v:.1e}" for k, v in diffs.items()), flush=True)
