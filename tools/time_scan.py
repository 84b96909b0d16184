"""Dev tool: time mc_scan_fwd at a given shape with HIP events (not the bench contract)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd.selective_scan_interface import selective_scan_fn  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="64,3072,4096,16")
ap.add_argument("--dtype", default="bf16")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--noz", action="store_true")
ap.add_argument("--bwd", action="store_true", help="time forward+backward (training) instead")
ap.add_argument("--train-fwd", action="store_true", help="time the training forward (saves the chunk states)")
ap.add_argument("--cm", action="store_true",
                help="channel-major views like the Mamba mixer: (B, D, L) with strides (L, B*L, 1)")
args = ap.parse_args()
Bsz, D, L, N = map(int, args.shape.split(","))
dt = {"bf16": torch.bfloat16, "f32": torch.float32}[args.dtype]
dev = "cuda"
torch.manual_seed(0)


def act(scale=1.0):
    if args.cm:
        return (scale * torch.randn(D, Bsz, L, device=dev)).to(dt).transpose(0, 1)
    return (scale * torch.randn(Bsz, D, L, device=dev)).to(dt)


u = act()
delta = act(0.5)
z = None if args.noz else act()
A = -torch.exp(torch.log(torch.arange(1, N + 1, dtype=torch.float32, device=dev)).repeat(D, 1))
Bm = torch.randn(Bsz, 1, N, L, device=dev, dtype=dt)
Cm = torch.randn(Bsz, 1, N, L, device=dev, dtype=dt)
Dv = torch.ones(D, device=dev)
bias = torch.rand(D, device=dev) * 4 - 5
if args.bwd:
    for t in (u, delta, A, Bm, Cm, Dv, bias) + ((z,) if z is not None else ()):
        t.requires_grad_(True)
    g_out = act()


def step():
    if args.train_fwd:
        from mamba_clip_amd.selective_scan_interface import scan_fwd
        return scan_fwd(u, delta, A, Bm, Cm, Dv, z, bias, True, True, False)
    out = selective_scan_fn(u, delta, A, Bm, Cm, Dv, z, bias, delta_softplus=True)
    if args.bwd:
        out.backward(g_out)


for _ in range(3):
    step()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(args.iters):
    step()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / args.iters
es = u.element_size()
nbytes = Bsz * D * L * es * (4 if z is not None else 3) + 2 * Bsz * N * L * es + (D * N + 2 * D) * 4
print(f"shape {args.shape} {args.dtype} z={z is not None} bwd={args.bwd} train_fwd={args.train_fwd}: {ms:.3f} ms  {nbytes / ms / 1e6:.1f} GB/s "
      f"({nbytes / ms / 1e6 / 8000 * 100:.1f}% of 8 TB/s)")
