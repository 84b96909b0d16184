"""Dev tool: HIP-event times of mc_mixer_proj_fwd / _bwd at the C2 mixer shape (D 1536, T 20480, R 48)
and of the library-GEMM chain they replace.  MAMBA_CLIP_AMD_LIB selects an A/B build."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
from mamba_clip_amd.ops import GradHandoff, mixer_proj  # noqa: E402

D, T, R = 1536, 20480, 48
P = R + 32
dev = "cuda"
torch.manual_seed(0)
x = torch.randn(D, T, device=dev, dtype=torch.bfloat16, requires_grad=True)
wx = (torch.randn(P, D, device=dev) * D ** -0.5).requires_grad_(True)
wdt = (torch.randn(D, R, device=dev) * R ** -0.5).requires_grad_(True)
gb, gc = torch.randn(16, T, device=dev, dtype=torch.bfloat16), torch.randn(16, T, device=dev, dtype=torch.bfloat16)
gd = torch.randn(D, T, device=dev, dtype=torch.bfloat16)
du = torch.randn(1, D, T, device=dev, dtype=torch.bfloat16)


def timed(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def fused_fwd():
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        mixer_proj(x, wx, wdt)


def fused_fwd_bwd():
    h = GradHandoff()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        b, c, d = mixer_proj(x, wx, wdt, h)
    h.du = du
    torch.autograd.backward([b, c, d], [gb, gc, gd], inputs=[x])


wxb, wdtb = wx.detach().bfloat16(), wdt.detach().bfloat16()


def lib_fwd():
    xd = wxb @ x.detach()
    wdtb @ xd[:R]


print(f"fused fwd {timed(fused_fwd):.1f} us, fused fwd+bwd(dx only) {timed(fused_fwd_bwd):.1f} us, "
      f"library fwd chain {timed(lib_fwd):.1f} us", flush=True)
