"""Deterministic reductions that replace torch's in the towers' glue: mc_colsum (bias /
position / cls gradients) and mc_l2norm (F.normalize of the features), against fp64 torch references,
plus the autograd wrappers (TokenEmbedFn, AddPosFn, L2NormalizeFn) against torch autograd."""
import pytest
import torch

from mamba_clip_amd import ops

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


@pytest.mark.parametrize("rows,cols,dtype,ld_pad", [
    (256, 197 * 768, torch.bfloat16, 0),      # the ViT pos_embed gradient (C2)
    (50432, 768, torch.bfloat16, 0),          # a ViT bias gradient
    (1000, 513, torch.float32, 3),            # ragged: scalar path, padded row stride
    (7, 64, torch.float16, 8),
    (1, 8, torch.float32, 0),
    (0, 16, torch.float32, 0),                # empty batch: zeros
])
def test_colsum_matches_fp64(rows, cols, dtype, ld_pad):
    g = torch.Generator(device=dev).manual_seed(rows + cols)
    base = torch.randn(rows, cols + ld_pad, device=dev, generator=g).to(dtype)
    x = base[:, :cols]
    got = ops.colsum(x)
    ref = x.double().sum(0)
    assert got.dtype == torch.float32 and got.shape == (cols,)
    tol = 1e-5 * max(1.0, rows ** 0.5)
    assert torch.allclose(got.double(), ref, atol=tol * 4, rtol=1e-5), float((got.double() - ref).abs().max())
    # bitwise repeatable
    assert torch.equal(got, ops.colsum(x))


@pytest.mark.parametrize("rows,cols,dtype", [(256, 512, torch.bfloat16), (64, 512, torch.float32),
                                             (33, 100, torch.float16), (5, 1, torch.float32)])
def test_l2_normalize_matches_torch(rows, cols, dtype):
    g = torch.Generator(device=dev).manual_seed(rows)
    x = torch.randn(rows, cols, device=dev, generator=g).to(dtype)
    if dtype != torch.float16:
        x[0] = 0      # the clamp branch: zero row (its gradient g / eps overflows fp16)
    gy = torch.randn(rows, cols, device=dev, generator=g)
    xa = x.clone().requires_grad_(True)
    y = ops.l2_normalize(xa)
    y.backward(gy)
    xr = x.double().requires_grad_(True)
    yr = torch.nn.functional.normalize(xr, dim=-1)
    yr.backward(gy.double())
    # torch's dtype rule: the input's dtype outside autocast, fp32 under it (ops.l2_normalize)
    assert y.dtype == dtype
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ya = ops.l2_normalize(x)
    assert ya.dtype == torch.float32
    assert torch.allclose(ya.double(), yr, atol=1e-6, rtol=1e-5)
    ytol = 1e-5 if dtype == torch.float32 else (4e-3 if dtype == torch.bfloat16 else 5e-4)
    assert torch.allclose(y.double(), yr, atol=ytol, rtol=ytol)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    scale = float(xr.grad.abs().max()) + 1e-30
    assert float((xa.grad.double() - xr.grad).abs().max()) / scale < tol
    assert xa.grad.dtype == dtype


def test_token_embed_and_add_pos_match_autograd():
    g = torch.Generator(device=dev).manual_seed(3)
    B, N, C = 8, 196, 768
    cls = torch.randn(1, 1, C, device=dev, generator=g).requires_grad_(True)
    pos = torch.randn(1, N + 1, C, device=dev, generator=g).requires_grad_(True)
    x = torch.randn(B, N, C, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    gm = torch.randn(B, N + 1, C, device=dev, generator=g).to(torch.bfloat16)
    m = ops.TokenEmbedFn.apply(cls, x, pos)
    m.backward(gm)
    cr, pr, xr = (t.detach().clone().requires_grad_(True) for t in (cls, pos, x))
    mr = torch.cat([cr.to(xr.dtype).expand(B, -1, -1), xr], 1) + pr.to(xr.dtype)
    assert torch.equal(m, mr)
    mr.backward(gm)
    assert torch.equal(x.grad, xr.grad)
    ref_pos = gm.double().sum(0, keepdim=True)
    assert torch.allclose(pos.grad.double(), ref_pos, atol=1e-3, rtol=1e-5)
    assert torch.allclose(cls.grad.double(), ref_pos[:, :1], atol=1e-3, rtol=1e-5)
    # BERT-style table longer than the sequence
    tab = torch.randn(1, 300, C, device=dev, generator=g).requires_grad_(True)
    h = torch.randn(B, 256, C, device=dev, generator=g).requires_grad_(True)
    gh = torch.randn(B, 256, C, device=dev, generator=g)
    out = ops.AddPosFn.apply(h, tab)
    out.backward(gh)
    assert torch.equal(out, h.detach() + tab.detach()[:, :256])
    assert torch.equal(h.grad, gh)
    assert torch.allclose(tab.grad[:, :256].double(), gh.double().sum(0, keepdim=True), atol=1e-4, rtol=1e-5)
    assert bool((tab.grad[:, 256:] == 0).all())
