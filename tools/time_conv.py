"""Dev tool: causal conv1d (+SiLU) forward / forward+backward at the C2 mixer shape, channel-major
views as in MambaMixer (x = rows [0, d_inner) of the (2 d_inner, B L) in_proj output).
MAMBA_CLIP_AMD_LIB selects an A/B build of the library."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
import torch
from mamba_clip_amd.ops import causal_conv1d

B, D, L = 256, 1536, 80
xz = torch.randn(2 * D, B * L, device="cuda").bfloat16()
x = xz[:D].view(D, B, L).transpose(0, 1)
w = torch.randn(D, 1, 4, device="cuda") * 0.3
b = torch.randn(D, device="cuda") * 0.1
gy = torch.randn(B, D, L, device="cuda").bfloat16()


def t(fn, n=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


with torch.no_grad():
    f = t(lambda: causal_conv1d(x, w, b, True))
xg = x.detach().requires_grad_(True)
wg, bg = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
fb = t(lambda: causal_conv1d(xg, wg, bg, True).backward(gy))
mb = B * D * L * 2 / 1e6
print(f"conv1d C2: fwd {f:.1f} us ({2 * mb / f / 1e3:.2f} TB/s)  fwd+bwd {fb:.1f} us  bwd ~{fb - f:.1f} us "
      f"({3 * mb / (fb - f) / 1e3:.2f} TB/s on x, dy, dx)")
