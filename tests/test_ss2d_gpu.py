"""SS2D cross-scan glue kernels (include/mc_ss2d.h) vs the reference's own construction, restated in
oracle/cpu_model.py (model.py:510-517 stack / transpose, 553-565 flips back, 630-647 conv, merge,
out_norm, gate): forward and every gradient, fp64 on the same inputs."""
import pytest
import torch

from oracle.cpu_model import ss2d_conv_stack_ref, ss2d_merge_ln_gate_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [(2, 6, 5, 16), (2, 16, 16, 64), (1, 7, 7, 96), (2, 14, 14, 40), (1, 56, 56, 128), (3, 17, 33, 8),
          (2, 14, 14, 256), (2, 7, 7, 512), (1, 5, 6, 1024)]   # merge tiles 16 / 8 / 4, conv tiles 16 / 8


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_stack_matches_reference_construction(shape, dtype):
    from mamba_clip_amd.ops import ss2d_conv_stack
    Bsz, H, W, C = shape
    g = torch.Generator().manual_seed(sum(shape))
    # the in_proj output's x half: a channels-last view with pixel stride 2C
    xz = torch.randn(Bsz, H, W, 2 * C, generator=g).to(dtype)
    w = torch.randn(C, 1, 3, 3, generator=g) * 0.3
    b = torch.randn(C, generator=g) * 0.1
    du = torch.randn(Bsz, 2, C, H * W, generator=g)
    x = xz[..., :C]
    # reference: fp64 autograd through the reference construction on the same (rounded) inputs
    xr = x.double().requires_grad_(True)
    wr, br = w.double().requires_grad_(True), b.double().requires_grad_(True)
    ur = ss2d_conv_stack_ref(xr, wr, br).double()
    ur.backward(du.double())
    # HIP
    xg = xz.to(DEV)[..., :C].detach().requires_grad_(True)
    wg, bg = w.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    u = ss2d_conv_stack(xg, wg, bg)
    assert u.dtype == torch.float32 and u.shape == (Bsz, 2, C, H * W)
    u.backward(du.to(DEV))
    assert _rel(u.cpu(), ur.detach()) < 1e-5
    tol = 1e-5 if dtype == torch.float32 else 8e-3     # dx is stored in x's dtype
    assert _rel(xg.grad.cpu(), xr.grad) < tol
    assert _rel(wg.grad.cpu(), wr.grad) < 1e-5
    assert _rel(bg.grad.cpu(), br.grad) < 1e-5


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_merge_ln_gate_matches_reference_construction(shape, dtype):
    from mamba_clip_amd.ops import SS2DMergeFn
    Bsz, H, W, C = shape
    L = H * W
    g = torch.Generator().manual_seed(7 + sum(shape))
    out = torch.randn(Bsz, 4 * C, L, generator=g)
    xz = torch.randn(Bsz, H, W, 2 * C, generator=g).to(dtype)
    lw = 1 + 0.2 * torch.randn(C, generator=g)
    lb = 0.1 * torch.randn(C, generator=g)
    dy = torch.randn(Bsz, H, W, C, generator=g).to(dtype)
    z = xz[..., C:]
    orr = out.double().requires_grad_(True)
    zr = z.double().requires_grad_(True)
    lwr, lbr = lw.double().requires_grad_(True), lb.double().requires_grad_(True)
    yr = ss2d_merge_ln_gate_ref(orr, zr, lwr, lbr, 1e-5)
    yr.backward(dy.double())
    og = out.to(DEV).requires_grad_(True)
    zg = xz.to(DEV)[..., C:].detach().requires_grad_(True)
    lwg, lbg = lw.to(DEV).requires_grad_(True), lb.to(DEV).requires_grad_(True)
    y = SS2DMergeFn.apply(og, zg, lwg, lbg, 1e-5, dtype)
    assert y.dtype == dtype and y.shape == (Bsz, H, W, C)
    y.backward(dy.to(DEV))
    ty = 2e-5 if dtype == torch.float32 else 8e-3       # y (and dz) are stored in the 16-bit dtype
    assert _rel(y.cpu(), yr.detach()) < ty
    assert _rel(og.grad.cpu(), orr.grad) < 5e-5
    assert _rel(zg.grad.cpu(), zr.grad) < ty
    assert _rel(lwg.grad.cpu(), lwr.grad) < 5e-5
    assert _rel(lbg.grad.cpu(), lbr.grad) < 5e-5


def test_ss2d_block_fused_equals_reference_construction_autocast():
    """The whole SS2D block under bf16 autocast, fused kernels vs the same module on the reference
    construction (oracle restatements of the conv / stack and the merge, HIP scan in both): outputs and
    the input gradient agree within bf16 rounding."""
    import mamba_clip_amd.model as M
    from mamba_clip_amd.model import SS2D
    torch.manual_seed(0)
    m = SS2D(d_model=32).to(DEV)
    x = torch.randn(2, 12, 10, 32, device=DEV)
    res = []
    for fused in (True, False):
        saved = (M.ss2d_conv_stack, M.ss2d_merge_ln_gate)
        if not fused:
            M.ss2d_conv_stack, M.ss2d_merge_ln_gate = ss2d_conv_stack_ref, ss2d_merge_ln_gate_ref
        try:
            xg = x.clone().requires_grad_(True)
            m.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = m(xg)
            y.float().sum().backward()
            res.append((y.float().detach(), xg.grad.clone(), m.conv2d.weight.grad.clone(), m.out_norm.weight.grad.clone()))
        finally:
            M.ss2d_conv_stack, M.ss2d_merge_ln_gate = saved
    for a, b in zip(res[0], res[1]):
        assert _rel(a, b) < 3e-2


def test_ss2d_kernels_reject_bad_shapes():
    from mamba_clip_amd.ops import ss2d_conv_stack
    x = torch.randn(1, 4, 4, 6, device=DEV)        # 6 channels: not a multiple of 4
    with pytest.raises(RuntimeError, match="multiples of 4"):
        ss2d_conv_stack(x, torch.randn(6, 1, 3, 3, device=DEV), None)
    x = torch.randn(1, 4, 4, 8, device=DEV)
    with pytest.raises(RuntimeError, match="ksize"):
        ss2d_conv_stack(x, torch.randn(8, 1, 5, 5, device=DEV), None)


PROJ_SHAPES = [(2, 64, 2, 3136), (2, 128, 4, 784), (3, 256, 8, 196), (2, 512, 16, 49), (1, 48, 3, 37),
               (2, 16, 1, 5)]   # (B, d_inner, dt_rank, L): the medmamba stages + ragged / tiny cases


@pytest.mark.parametrize("shape", PROJ_SHAPES)
def test_ss2d_proj_matches_reference_einsums(shape):
    """ops.SS2DProjFn (mc_ss2d_group_proj) vs the reference's two einsums (model.py:519-528) in fp64 on
    the same fp32 inputs: x_dbl's B / C rows, delta, and the gradients of u, x_proj and dt_proj; and two
    runs give the same bits (in-order sums, fixed-order batch reduction)."""
    from mamba_clip_amd.ops import ss2d_proj
    Bsz, d, R, L = shape
    N = 16
    c = R + 2 * N
    g = torch.Generator().manual_seed(d + L)
    u = torch.randn(Bsz, 2, d, L, generator=g)
    wx = torch.randn(4, c, d, generator=g) * d ** -0.5
    wdt = torch.randn(4, d, R, generator=g) * R ** -0.5
    gd, gb, gc = (torch.randn(Bsz, 4, m, L, generator=g) for m in (d, N, N))
    # reference: the model's einsum form in fp64 (direction k = 2 i + j reads frame j)
    ur, wxr, wdtr = (t.double().requires_grad_(True) for t in (u, wx, wdt))
    x_dbl = torch.einsum("bjdl,ijcd->bijcl", ur, wxr.view(2, 2, c, d)).reshape(Bsz, 4, c, L)
    dts, Br, Cr = torch.split(x_dbl, [R, N, N], dim=2)
    dr = torch.einsum("bkrl,kdr->bkdl", dts, wdtr)
    torch.autograd.backward([dr, Br, Cr], [gd.double(), gb.double(), gc.double()])
    runs = []
    for _ in range(2):
        ug, wxg, wdtg = (t.to(DEV).requires_grad_(True) for t in (u, wx, wdt))
        delta, Bs, Cs = ss2d_proj(ug, wxg, wdtg, R, N)
        torch.autograd.backward([delta, Bs, Cs], [gd.to(DEV), gb.to(DEV), gc.to(DEV)])
        runs.append([t.detach().clone() for t in (delta, Bs, Cs, ug.grad, wxg.grad, wdtg.grad)])
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    for got, ref, tol in zip(runs[0], (dr, Br, Cr, ur.grad, wxr.grad, wdtr.grad), (1e-5, 1e-5, 1e-5, 1e-5, 2e-5, 2e-5)):
        assert got.shape == ref.shape
        assert _rel(got.cpu(), ref.detach()) < tol


def test_ss2d_block_uses_group_proj():
    """The SS2D block's forward takes the mc_ss2d_group_proj path for fp32 activations, and its result
    equals the einsum path's within fp32 rounding (fwd + every parameter gradient)."""
    import mamba_clip_amd.model as M
    torch.manual_seed(3)
    m = M.SS2D(d_model=32).to(DEV)
    x = torch.randn(2, 14, 14, 32, device=DEV)
    calls = []
    real = M.ss2d_proj
    M.ss2d_proj = lambda *a: calls.append(1) or real(*a)
    try:
        xa = x.clone().requires_grad_(True)
        m(xa).square().sum().backward()
    finally:
        M.ss2d_proj = real
    assert calls, "SS2D did not take the group-projection path"
    grads = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad()
    ok = M.ss2d_proj_ok
    M.ss2d_proj_ok = lambda *a: False
    try:
        xb = x.clone().requires_grad_(True)
        m(xb).square().sum().backward()
    finally:
        M.ss2d_proj_ok = ok
    assert _rel(xa.grad, xb.grad) < 1e-4
    for n, p in m.named_parameters():
        assert _rel(grads[n], p.grad) < 1e-4, n
