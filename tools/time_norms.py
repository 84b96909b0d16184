"""Dev tool: the ViT's add + LayerNorm (ops.add_layernorm -> mc_add_layernorm_fwd / _bwd) and the Mamba
tower's add + RMSNorm at the C2 shapes, forward and forward + backward, HIP events, us per call.
MAMBA_CLIP_AMD_LIB selects the build."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
import torch  # noqa: E402
from mamba_clip_amd.ops import add_layernorm  # noqa: E402


def t(fn, iters=20):
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


B, N, C = 256, 197, 768
x = torch.randn(B, N, C, device="cuda", dtype=torch.bfloat16, requires_grad=True)
r = torch.randn(B, N, C, device="cuda", dtype=torch.bfloat16, requires_grad=True)
w = torch.randn(C, device="cuda", requires_grad=True)
b = torch.randn(C, device="cuda", requires_grad=True)
g1 = torch.randn(B, N, C, device="cuda", dtype=torch.bfloat16)
with torch.no_grad():
    fwd = t(lambda: add_layernorm(x, r, w, b))


def fb():
    y, h = add_layernorm(x, r, w, b)
    torch.autograd.backward([y, h], [g1, g1])
both = t(fb)
byt = 4 * x.numel() * 2
print(f"add_layernorm {B}x{N}x{C} bf16: fwd {fwd:6.1f} us ({byt / fwd / 1e3:.0f} GB/s) | fwd+bwd {both:6.1f} us", flush=True)

from mamba_clip_amd.ops import add_rmsnorm  # noqa: E402
T, D = 256 * 80, 768
hs = torch.randn(256, 80, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
rs = torch.randn(256, 80, D, device="cuda", dtype=torch.float32, requires_grad=True)
wn = torch.randn(D, device="cuda", requires_grad=True)
gy = torch.randn(256, 80, D, device="cuda", dtype=torch.bfloat16)
gr = torch.randn(256, 80, D, device="cuda", dtype=torch.float32)
with torch.no_grad():
    fwd = t(lambda: add_rmsnorm(hs, rs, wn, 1e-5))


def fb2():
    y, res = add_rmsnorm(hs, rs, wn, 1e-5)
    torch.autograd.backward([y, res], [gy, gr])
both = t(fb2)
byt = T * D * (2 + 4 + 2 + 4)
print(f"add_rmsnorm {T}x{D} bf16 (fp32 residual): fwd {fwd:6.1f} us ({byt / fwd / 1e3:.0f} GB/s) | fwd+bwd {both:6.1f} us",
      flush=True)
