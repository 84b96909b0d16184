"""Dev tool: A/B of the ViT-B/16 attention and MLP glue at C2 (b=256, 197 tokens, 12 x 64, bf16), fwd+bwd.

Times torch SDPA (default backend selection), the math backend, an explicit
bmm + softmax path, and Linear+GELU vs the fused-epilogue addmm.
"""
import time

import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel

dev = "cuda"
B, N, Hh, D = 256, 197, 12, 64
bf = torch.bfloat16


def bench(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


q, k, v = (torch.randn(B, Hh, N, D, device=dev, dtype=bf, requires_grad=True) for _ in range(3))
go = torch.randn(B, Hh, N, D, device=dev, dtype=bf)


def sdpa_default():
    o = F.scaled_dot_product_attention(q, k, v)
    o.backward(go)


def sdpa_math():
    with sdpa_kernel(SDPBackend.MATH):
        o = F.scaled_dot_product_attention(q, k, v)
    o.backward(go)


def explicit():
    s = torch.matmul(q, k.transpose(-1, -2)) * (D ** -0.5)
    p = torch.softmax(s.float(), dim=-1).to(bf)
    o = torch.matmul(p, v)
    o.backward(go)


for name, fn in [("sdpa default", sdpa_default), ("sdpa math", sdpa_math), ("bmm+softmax(fp32)", explicit)]:
    for backend in (None,):
        try:
            print(f"{name:22s} fwd+bwd {bench(fn):8.3f} ms")
        except Exception as e:  # noqa: BLE001
            print(f"{name:22s} failed: {type(e).__name__}: {e}")
for be in (SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION, SDPBackend.CUDNN_ATTENTION):
    def f(be=be):
        with sdpa_kernel(be):
            o = F.scaled_dot_product_attention(q, k, v)
        o.backward(go)
    try:
        print(f"{str(be):22s} fwd+bwd {bench(f):8.3f} ms")
    except Exception as e:  # noqa: BLE001
        print(f"{str(be):22s} failed: {type(e).__name__}: {str(e)[:100]}")

# MLP: fc1 + GELU at (B*N, 768) -> 3072
x = torch.randn(B * N, 768, device=dev, dtype=bf, requires_grad=True)
w = torch.randn(3072, 768, device=dev, dtype=bf, requires_grad=True)
bb = torch.randn(3072, device=dev, dtype=bf, requires_grad=True)
g2 = torch.randn(B * N, 3072, device=dev, dtype=bf)


def mlp_plain():
    y = F.gelu(F.linear(x, w, bb))
    y.backward(g2)


def mlp_fused():
    y = torch._addmm_activation(bb, x, w.t(), use_gelu=True)
    y.backward(g2)


def mlp_tanh():
    y = F.gelu(F.linear(x, w, bb), approximate="tanh")
    y.backward(g2)


for name, fn in [("linear+gelu", mlp_plain), ("addmm_activation gelu", mlp_fused), ("linear+gelu(tanh)", mlp_tanh)]:
    try:
        print(f"{name:22s} fwd+bwd {bench(fn):8.3f} ms")
    except Exception as e:  # noqa: BLE001
        print(f"{name:22s} failed: {type(e).__name__}: {str(e)[:100]}")
