"""Dev tool: the ViT attention sub-block (qkv Linear -> SDPA -> proj) at C2, fwd+bwd, variants of the q/k/v split and SDPA backend."""
import time

import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel

dev, bf = "cuda", torch.bfloat16
B, N, C, Hh = 256, 197, 768, 12
D = C // Hh
torch.manual_seed(0)
qkv_l = torch.nn.Linear(C, 3 * C).to(dev, bf)
proj = torch.nn.Linear(C, C).to(dev, bf)
x = torch.randn(B, N, C, device=dev, dtype=bf, requires_grad=True)
go = torch.randn(B, N, C, device=dev, dtype=bf)


def permute_default():
    qkv = qkv_l(x).reshape(B, N, 3, Hh, D).permute(2, 0, 3, 1, 4)
    o = F.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2])
    return proj(o.transpose(1, 2).reshape(B, N, C))


def unbind(backend=None):
    def f():
        q, k, v = qkv_l(x).view(B, N, 3, Hh, D).unbind(2)
        q, k, v = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
        if backend is None:
            o = F.scaled_dot_product_attention(q, k, v)
        else:
            with sdpa_kernel(backend):
                o = F.scaled_dot_product_attention(q, k, v)
        return proj(o.transpose(1, 2).reshape(B, N, C))
    return f


def bench(fn, iters=10):
    def step():
        fn().backward(go)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


ref = permute_default().float()
for name, fn in [("permute+default", permute_default), ("unbind+default", unbind()),
                 ("unbind+efficient", unbind(SDPBackend.EFFICIENT_ATTENTION)),
                 ("unbind+flash", unbind(SDPBackend.FLASH_ATTENTION))]:
    try:
        err = float((fn().float() - ref).abs().max())
        print(f"{name:20s} {bench(fn):8.3f} ms   max|diff| vs permute+default {err:.2e}")
    except Exception as e:  # noqa: BLE001
        print(f"{name:20s} failed: {type(e).__name__}: {str(e)[:120]}")
