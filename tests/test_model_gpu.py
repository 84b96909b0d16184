"""GPU checks of the encoder kernels and modules (HIP path) against fp64/fp32 oracles
and the reference SS2D golden vectors."""
import pytest
import torch
import torch.nn.functional as F

from conftest import load_golden
from oracle import models_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_add_rmsnorm_fwd_bwd():
    from mamba_clip_amd.ops import add_rmsnorm
    g = torch.Generator().manual_seed(0)
    for dt in (torch.float32, torch.bfloat16):
        for rows, cols in [(7, 768), (160, 1536), (3, 64)]:
            x = torch.randn(rows, cols, generator=g).to(dt)
            res = torch.randn(rows, cols, generator=g)
            w = torch.randn(cols, generator=g)
            xd = x.to(DEV).requires_grad_(True)
            rd = res.to(DEV).requires_grad_(True)
            wd = w.to(DEV).requires_grad_(True)
            y, h = add_rmsnorm(xd, rd, wd)
            dy = torch.randn(rows, cols, generator=g).to(dt)
            dh = torch.randn(rows, cols, generator=g)
            (y.float() * dy.to(DEV).float()).sum().add_((h * dh.to(DEV)).sum()).backward()
            xr = x.double().requires_grad_(True)
            rr = res.double().requires_grad_(True)
            wr = w.double().requires_grad_(True)
            yr, hr = R.rmsnorm_ref(xr, rr, wr)
            ((yr * dy.double()).sum() + (hr * dh.double()).sum()).backward()
            tol = 1e-5 if dt == torch.float32 else 1e-2
            torch.testing.assert_close(y.float().cpu(), yr.float(), rtol=tol, atol=tol)
            torch.testing.assert_close(h.cpu(), hr.float(), rtol=1e-6, atol=1e-6)
            torch.testing.assert_close(xd.grad.float().cpu(), xr.grad.float(), rtol=tol, atol=tol * 4)
            torch.testing.assert_close(rd.grad.cpu(), rr.grad.float(), rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(wd.grad.cpu(), wr.grad.float(), rtol=1e-3, atol=1e-3 * rows ** 0.5)


def test_add_layernorm_fwd_bwd():
    from mamba_clip_amd.ops import add_layernorm
    g = torch.Generator().manual_seed(5)
    for dt in (torch.float32, torch.bfloat16):
        for rows, cols, with_res, with_bias in [(9, 768, True, True), (197, 768, False, True), (5, 64, True, False)]:
            x = torch.randn(rows, cols, generator=g).to(dt)
            res = torch.randn(rows, cols, generator=g).to(dt) if with_res else None
            w = 1 + 0.1 * torch.randn(cols, generator=g)
            b = 0.1 * torch.randn(cols, generator=g) if with_bias else None
            dy = torch.randn(rows, cols, generator=g).to(dt)
            dh = torch.randn(rows, cols, generator=g).to(dt)
            xd = x.to(DEV).requires_grad_(True)
            rd = res.to(DEV).requires_grad_(True) if with_res else None
            wd = w.to(DEV).requires_grad_(True)
            bd = b.to(DEV).requires_grad_(True) if with_bias else None
            y, h = add_layernorm(xd, rd, wd, bd)
            loss = (y.float() * dy.to(DEV).float()).sum()
            if with_res:
                loss = loss + (h.float() * dh.to(DEV).float()).sum()
            loss.backward()
            xr = x.double().requires_grad_(True)
            rr = res.double().requires_grad_(True) if with_res else None
            wr = w.double().requires_grad_(True)
            br = b.double().requires_grad_(True) if with_bias else None
            yr, hr = R.add_layernorm_ref(xr, rr, wr, br)
            lr = (yr * dy.double()).sum()
            if with_res:
                lr = lr + (hr * dh.double()).sum()
            lr.backward()
            tol = 1e-5 if dt == torch.float32 else 2e-2
            torch.testing.assert_close(y.float().cpu(), yr.float(), rtol=tol, atol=tol)
            torch.testing.assert_close(h.float().cpu(), hr.to(dt).float(), rtol=tol, atol=tol)
            torch.testing.assert_close(xd.grad.float().cpu(), xr.grad.float(), rtol=tol, atol=tol * 4)
            if with_res:
                torch.testing.assert_close(rd.grad.float().cpu(), rr.grad.float(), rtol=tol, atol=tol * 4)
            gtol = 1e-3 if dt == torch.float32 else 3e-2
            torch.testing.assert_close(wd.grad.cpu(), wr.grad.float(), rtol=gtol, atol=gtol * rows ** 0.5)
            if with_bias:
                torch.testing.assert_close(bd.grad.cpu(), br.grad.float(), rtol=gtol, atol=gtol * rows ** 0.5)


def test_vit_block_matches_unfused_math():
    """Fused (m, h) ViT blocks == x = x + attn(norm1(x)); x = x + mlp(norm2(x)) in fp32."""
    from mamba_clip_amd.model import VisionTransformer
    torch.manual_seed(0)
    vit = VisionTransformer(img_size=32, patch=8, width=64, layers=2, heads=4, output_dim=16).to(DEV)
    img = torch.randn(3, 3, 32, 32, device=DEV)
    out = vit(img)
    with torch.no_grad():
        x = vit.patch_embed.proj(img).flatten(2).transpose(1, 2)
        x = torch.cat([vit.cls_token.expand(3, -1, -1), x], 1) + vit.pos_embed
        for blk in vit.blocks:
            x = x + blk.attn(blk.norm1(x))
            x = x + blk.fc2(F.gelu(blk.fc1(blk.norm2(x))))
        ref = vit.head(vit.norm(x)[:, 0])
    torch.testing.assert_close(out.detach(), ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fc1_gelu_fused_backward(dt):
    """mc_gelu_bwd (gh = ga * gelu'(h) + the fc1 bias gradient in one pass) vs torch's unfused
    GELU backward + sum, same weights, fp32 and bf16 (rows not a multiple of the slice size)."""
    from mamba_clip_amd.ops import fc1_gelu
    torch.manual_seed(3)
    x = torch.randn(5, 77, 96, device=DEV).to(dt).requires_grad_(True)
    w = (0.1 * torch.randn(256, 96, device=DEV)).requires_grad_(True)
    b = (0.1 * torch.randn(256, device=DEV)).requires_grad_(True)
    ga = torch.randn(5, 77, 256, device=DEV).to(dt)
    a = fc1_gelu(x, w, b)
    a.backward(ga)
    xr, wr, br = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    h = F.linear(xr, wr.to(dt), br.to(dt))
    ar = F.gelu(h)
    ar.backward(ga)
    tol = dict(rtol=1e-5, atol=1e-5) if dt == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(a, ar, **tol)
    torch.testing.assert_close(x.grad, xr.grad, **tol)
    torch.testing.assert_close(w.grad, wr.grad, **(dict(rtol=1e-4, atol=1e-4) if dt == torch.float32
                                                   else dict(rtol=2e-2, atol=5e-2)))
    # the bias gradient: sum of the stored gh (bf16-rounded for bf16) -- vs torch's gelu_backward output summed
    gh = torch.ops.aten.gelu_backward(ga.reshape(-1, 256), h.detach().reshape(-1, 256))
    # bf16: an element of gh may round one ulp apart from torch's (erf evaluated differently)
    btol = dict(rtol=1e-5, atol=1e-4) if dt == torch.float32 else dict(rtol=1e-3, atol=2e-3)
    torch.testing.assert_close(b.grad, gh.sum(0, dtype=torch.float32), **btol)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_qkv_proj_fused_pack(dt):
    """mc_qkv_grad_pack packs the attention's dq / dk / dv (strides as SDPA returns them) into the
    qkv output gradient and sums the qkv bias gradient: vs linear + unbind + stack."""
    from mamba_clip_amd.ops import qkv_proj
    torch.manual_seed(4)
    Bsz, N, C, H = 3, 50, 128, 4
    x = torch.randn(Bsz, N, C, device=DEV).to(dt).requires_grad_(True)
    w = (0.05 * torch.randn(3 * C, C, device=DEV)).requires_grad_(True)
    b = (0.05 * torch.randn(3 * C, device=DEV)).requires_grad_(True)
    go = torch.randn(Bsz, H, N, C // H, device=DEV).to(dt)
    q, k, v = qkv_proj(x, w, b, H)
    F.scaled_dot_product_attention(q, k, v).backward(go)
    xr, wr, br = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    qr, kr, vr = F.linear(xr, wr.to(dt), br.to(dt)).view(Bsz, N, 3, H, C // H).unbind(2)
    F.scaled_dot_product_attention(qr.transpose(1, 2), kr.transpose(1, 2), vr.transpose(1, 2)).backward(go)
    # bf16: torch's reference bias / weight gradients are rounded to bf16 before the fp32 cast
    tol = dict(rtol=1e-4, atol=1e-4) if dt == torch.float32 else dict(rtol=1e-2, atol=2e-2)
    for got, want in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        torch.testing.assert_close(got, want, **tol)


def test_vit_bias_grads_from_layernorm_colsum():
    """fc2 / attention-proj bias gradients come from the column sums the LayerNorm backward takes
    of dx (mc_add_layernorm_bwd dx_colsum); they equal the direct column sums of the gradient."""
    from mamba_clip_amd import ops
    from mamba_clip_amd.model import VisionTransformer
    torch.manual_seed(5)
    vit = VisionTransformer(img_size=32, patch=8, width=64, layers=3, heads=4, output_dim=16).to(DEV)
    img = torch.randn(4, 3, 32, 32, device=DEV)
    seen = []
    orig = ops.LinearSK.backward

    def spy(ctx, gy):
        pre = getattr(gy, ops.COLSUM_ATTR, None)
        out = orig(ctx, gy)
        if pre is not None and pre[1] == gy._version:
            seen.append(float((out[2] - gy.reshape(-1, gy.shape[-1]).sum(0, dtype=torch.float32)).abs().max()))
        return out

    ops.LinearSK.backward = staticmethod(spy)
    try:
        vit(img).square().sum().backward()
    finally:
        ops.LinearSK.backward = orig
    # fc2 of blocks 0..1 and the attention proj of every block feed a following add+LayerNorm
    assert len(seen) >= 5 and max(seen) < 1e-4, seen


def test_causal_conv1d_fwd_bwd():
    from mamba_clip_amd.ops import causal_conv1d
    g = torch.Generator().manual_seed(1)
    for dt in (torch.float32, torch.bfloat16):
        for (B, D, L, K, silu) in [(2, 64, 80, 4, True), (3, 40, 17, 3, False), (1, 8, 1, 4, True)]:
            big = torch.randn(B, 2 * D, L, generator=g).to(dt)
            x = big[:, :D]                       # strided view, as in the Mamba mixer
            w = torch.randn(D, 1, K, generator=g)
            b = torch.randn(D, generator=g)
            xd = big.to(DEV)[:, :D].detach().requires_grad_(True)
            wd = w.to(DEV).requires_grad_(True)
            bd = b.to(DEV).requires_grad_(True)
            y = causal_conv1d(xd, wd, bd, silu)
            gy = torch.randn(B, D, L, generator=g).to(dt)
            y.backward(gy.to(DEV))
            xr = x.double().requires_grad_(True)
            wr = w.double().requires_grad_(True)
            br = b.double().requires_grad_(True)
            yr = R.causal_conv1d_ref(xr, wr, br, silu)
            yr.backward(gy.double())
            tol = 1e-5 if dt == torch.float32 else 2e-2
            torch.testing.assert_close(y.float().cpu(), yr.float(), rtol=tol, atol=tol)
            torch.testing.assert_close(xd.grad.float().cpu(), xr.grad.float(), rtol=tol, atol=tol)
            torch.testing.assert_close(wd.grad.cpu(), wr.grad.float(), rtol=1e-3, atol=1e-3 * (B * L) ** 0.5)
            torch.testing.assert_close(bd.grad.cpu(), br.grad.float(), rtol=1e-3, atol=1e-3 * (B * L) ** 0.5)


def test_causal_conv1d_channel_major_layout():
    """x as the channel-major (dim, batch*L) GEMM output viewed (B, D, L): y / dx keep that layout."""
    from mamba_clip_amd.ops import causal_conv1d
    g = torch.Generator().manual_seed(2)
    for dt in (torch.bfloat16, torch.float32):
        # the last three: the backward's halo kernel over several slices and 63-item wave steps, with
        # rows of 1 and 2 vectors (every / every other neighbouring lane in another row)
        for (B, D, L, K) in [(4, 96, 80, 4), (3, 16, 24, 8), (2, 24, 13, 4), (256, 6, 80, 4), (200, 4, 8, 4),
                             (130, 4, 16, 4)]:
            xz = torch.randn(2 * D, B * L, generator=g).to(dt)
            w = torch.randn(D, 1, K, generator=g)
            b = torch.randn(D, generator=g)
            xd = xz.to(DEV).requires_grad_(True)
            x = xd[:D].view(D, B, L).transpose(0, 1)
            wd = w.to(DEV).requires_grad_(True)
            bd = b.to(DEV).requires_grad_(True)
            y = causal_conv1d(x, wd, bd, True)
            assert y.stride() == x.stride()
            gy = torch.randn(B, D, L, generator=g).to(dt)
            y.backward(gy.to(DEV))
            xr = xz[:D].view(D, B, L).transpose(0, 1).double().requires_grad_(True)
            wr = w.double().requires_grad_(True)
            br = b.double().requires_grad_(True)
            yr = R.causal_conv1d_ref(xr, wr, br, True)
            yr.backward(gy.double())
            tol = 1e-5 if dt == torch.float32 else 2e-2
            torch.testing.assert_close(y.float().cpu(), yr.float(), rtol=tol, atol=tol)
            gx = xd.grad[:D].view(D, B, L).transpose(0, 1)
            torch.testing.assert_close(gx.float().cpu(), xr.grad.float(), rtol=tol, atol=tol)
            assert torch.count_nonzero(xd.grad[D:]) == 0
            torch.testing.assert_close(wd.grad.cpu(), wr.grad.float(), rtol=1e-3, atol=1e-3 * (B * L) ** 0.5)
            torch.testing.assert_close(bd.grad.cpu(), br.grad.float(), rtol=1e-3, atol=1e-3 * (B * L) ** 0.5)


def test_scan_channel_major_layout():
    """selective_scan_fn on channel-major views: out and du/ddelta/dz keep the input layout."""
    from mamba_clip_amd.selective_scan_interface import selective_scan_fn
    from oracle.scan_ref import selective_scan_ref
    g = torch.Generator().manual_seed(3)
    B, D, L, N = 3, 128, 48, 16
    for dt in (torch.bfloat16, torch.float32):
        big = torch.randn(3 * D, B * L, generator=g)
        big[D:2 * D] *= 0.5
        bc = torch.randn(2 * N, B * L, generator=g)
        A = -torch.exp(torch.log(torch.arange(1, N + 1).float()).repeat(D, 1))
        Dv = torch.randn(D, generator=g)
        bias = torch.randn(D, generator=g) * 0.3 - 2.0

        def views(t, tbc):
            u, dl, z = (t[i * D:(i + 1) * D].view(D, B, L).transpose(0, 1) for i in range(3))
            Bm, Cm = (tbc[i * N:(i + 1) * N].view(N, B, L).transpose(0, 1) for i in range(2))
            return u, dl, z, Bm, Cm

        bd = big.to(dt).to(DEV).requires_grad_(True)
        bcd = bc.to(dt).to(DEV).requires_grad_(True)
        u, dl, z, Bm, Cm = views(bd, bcd)
        out = selective_scan_fn(u, dl, A.to(DEV), Bm, Cm, Dv.to(DEV), z=z, delta_bias=bias.to(DEV),
                                delta_softplus=True)
        assert out.stride() == u.stride()
        dout = torch.randn(B, D, L, generator=g).to(dt)
        out.backward(dout.to(DEV))
        br = big.to(dt).double().requires_grad_(True)
        bcr = bc.to(dt).double().requires_grad_(True)
        ur, dlr, zr, Br, Cr = views(br, bcr)
        ref = selective_scan_ref(ur, dlr, A.double(), Br, Cr, Dv.double(), z=zr, delta_bias=bias.double(),
                                 delta_softplus=True, compute_dtype=torch.float64)
        ref.backward(dout.double())
        tol = 2e-2 if dt == torch.bfloat16 else 1e-4
        scale = ref.abs().max().item()
        torch.testing.assert_close(out.double().cpu(), ref.to(dt).double(), rtol=tol, atol=tol * scale)
        gs = br.grad.abs().max().item()
        torch.testing.assert_close(bd.grad.double().cpu(), br.grad, rtol=tol, atol=tol * gs)
        gs = bcr.grad.abs().max().item()
        torch.testing.assert_close(bcd.grad.double().cpu(), bcr.grad, rtol=tol, atol=tol * gs)


def test_patch_im2col_exact():
    from mamba_clip_amd.ops import patch_im2col
    img = torch.randn(2, 3, 32, 48)
    for P in (4, 16):
        torch.testing.assert_close(patch_im2col(img.to(DEV), P).cpu(), R.im2col_ref(img, P), rtol=0, atol=0)
    imgb = img.bfloat16()
    assert torch.equal(patch_im2col(imgb.to(DEV), 16).cpu(), R.im2col_ref(imgb.float(), 16).bfloat16())


def test_mamba_mixer_matches_oracle():
    from mamba_clip_amd.model import MambaMixer
    torch.manual_seed(0)
    m = MambaMixer(64, d_state=16).to(DEV)
    h = torch.randn(2, 40, 64, device=DEV, requires_grad=True)
    out = m(h)
    ref = R.mamba_mixer_ref(m, h.detach().cpu())
    torch.testing.assert_close(out.detach().cpu().double(), ref, rtol=1e-4, atol=1e-4)
    out.sum().backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())
    # gradients vs fp64 autograd of the oracle for the input
    hr = h.detach().cpu().double().requires_grad_(True)
    R.mamba_mixer_ref(m, hr).sum().backward()
    torch.testing.assert_close(h.grad.cpu().double(), hr.grad, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("amp", [False, True])
def test_mamba_mixer_gradient_slabs_no_concat(amp):
    """The conv / scan backward kernels write dx / dz into one slab (the in_proj split's gradient),
    and dt_proj's backward GEMM plus the scan's dB / dC reduction write into another (the x_proj
    split's gradient): no transpose copies or concatenation, and every gradient bitwise the same as
    the copying path.  amp: bf16 autocast at a C2-like width (the lane-pair scan kernels)."""
    from mamba_clip_amd import ops
    from mamba_clip_amd.model import MambaMixer
    import mamba_clip_amd.model as M
    torch.manual_seed(1)
    d = 256 if amp else 64
    m = MambaMixer(d, d_state=16).to(DEV)
    h = torch.randn(3, 48, d, device=DEV, requires_grad=True)

    def run():
        m.zero_grad()
        h.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            y = m(h)
        y.float().square().sum().backward()
        return [h.grad.clone()] + [p.grad.clone() for p in m.parameters()]

    made = []
    orig = ops.GradSlab.__init__

    def spy(self, *a, **k):
        orig(self, *a, **k)
        made.append(self)

    ops.GradSlab.__init__ = spy
    try:
        with_slab = run()
    finally:
        ops.GradSlab.__init__ = orig
    assert len(made) == 2 and all(getattr(s, "shared", False) for s in made)
    real = M.GradSlab
    M.GradSlab = lambda *a, **k: None     # the same step with plain concatenation
    try:
        plain = run()
    finally:
        M.GradSlab = real
    for a, b in zip(with_slab, plain):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_mamba_mixer_du_handoff(dt):
    """The scan hands du to x_proj's backward (ops.GradHandoff), which adds its dX in the GEMM
    epilogue: the same gradients as autograd summing the two producers (one rounding instead of two
    in bf16), and the handoff is consumed."""
    import mamba_clip_amd.model as M
    from mamba_clip_amd import ops
    torch.manual_seed(2)
    m = M.MambaMixer(128, d_state=16).to(DEV)
    h = torch.randn(4, 64, 128, device=DEV)
    gy = torch.randn(4, 64, 128, device=DEV)
    made = []
    real = M.GradHandoff

    def spy():
        made.append(real())
        return made[-1]

    runs = []
    for hand in (spy, lambda: None):
        M.GradHandoff = hand
        try:
            m.zero_grad()
            hh = h.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dt == torch.bfloat16):
                y = m(hh)
            (y.float() * gy).sum().backward()
        finally:
            M.GradHandoff = real
        runs.append((hh.grad.clone(), {n: p.grad.clone() for n, p in m.named_parameters()}))
    assert len(made) == 1 and made[0].du is None          # handed over and taken
    (gh, gp), (gh0, gp0) = runs
    tol = dict(rtol=1e-5, atol=1e-5) if dt == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(gh, gh0, **tol)
    for n in gp0:
        torch.testing.assert_close(gp[n], gp0[n], **tol, msg=n)
    assert isinstance(ops.GradHandoff(), ops.GradHandoff)


def test_text_tower_neg_exp_many_bitwise():
    """The tower forms every mixer's A = -exp(A_log) in one launch (ops.NegExpManyFn): values and
    A_log gradients bitwise equal to the per-mixer expression."""
    from mamba_clip_amd.ops import neg_exp_many
    torch.manual_seed(3)
    logs = [torch.randn(96, 16, device=DEV, requires_grad=True) for _ in range(5)]
    gs = [torch.randn(96, 16, device=DEV) for _ in range(5)]
    As = neg_exp_many(logs)
    torch.autograd.backward([a for a in As if True][:4], gs[:4])   # one output without a gradient
    for i, (l, a) in enumerate(zip(logs, As)):
        ref_l = l.detach().clone().requires_grad_(True)
        ref = -torch.exp(ref_l.float())
        assert torch.equal(a, ref.detach())
        if i < 4:
            ref.backward(gs[i])
            assert torch.equal(l.grad, ref_l.grad)
        else:
            assert l.grad is None


@pytest.mark.parametrize("fname", ["ss2d_d32_h6w5.safetensors", "ss2d_d16_h4w4.safetensors"])
def test_ss2d_matches_reference_golden(fname):
    from mamba_clip_amd.model import SS2D
    g = load_golden(fname)
    sd = {k[3:]: v for k, v in g.items() if k.startswith("sd.")}
    m = SS2D(d_model=g["x"].shape[-1]).to(DEV).eval()
    m.load_state_dict(sd)
    x = g["x"].to(DEV).requires_grad_(True)
    y = m(x)
    torch.testing.assert_close(y.detach().cpu(), g["y"], rtol=1e-4, atol=1e-5)
    y.backward(g["gy"].to(DEV))
    torch.testing.assert_close(x.grad.cpu(), g["gx"], rtol=1e-3, atol=1e-5)


def test_ss_conv_ssm_matches_reference_golden():
    from mamba_clip_amd.model import SS_Conv_SSM
    g = load_golden("ss_conv_ssm_h32.safetensors")
    sd = {k[3:]: v for k, v in g.items() if k.startswith("sd.")}
    m = SS_Conv_SSM(hidden_dim=32).to(DEV).eval()
    m.load_state_dict(sd)
    torch.testing.assert_close(m(g["x"].to(DEV)).detach().cpu(), g["y"], rtol=1e-4, atol=1e-5)


def test_tiny_clip_train_step():
    from mamba_clip_amd.model import init_model
    from mamba_clip_amd.loss import ClipLoss
    # seeded, lr 3e-4 over 5 steps: at lr 1e-3 / 3 steps the loss rose on some seeds with or
    # without any given fusion (tools/dbg_tiny.py), i.e. the old form was a flaky check
    torch.manual_seed(0)
    model, _, _, _ = init_model("tiny-mamba-clip")
    model = model.to(DEV)
    opt = torch.optim.AdamW(model.parameters(), lr=3e-4)
    img = torch.randn(8, 3, 32, 32, device=DEV)
    tok = torch.randint(1, 1000, (8, 16), device=DEV)
    losses = []
    for _ in range(5):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(img, tok)
            loss = ClipLoss()(**out)["contrastive_loss"]
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss))
        assert torch.allclose(out["image_features"].float().norm(dim=-1), torch.ones(8, device=DEV), atol=1e-2)
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]          # it learns the (fixed) batch


@pytest.mark.parametrize("stage", [1, 2])
def test_cli_synthetic_tiny(stage, capsys):
    from mamba_clip_amd.cli import main
    rc = main(["--synthetic", "--model", "tiny-mamba-clip", "--batch-size", "8", "--train-num-samples", "24",
               "--stage", str(stage), "--benchmark", "--log-every-n-steps", "1", "--warmup", "1"])
    assert rc == 0
    import json
    line = [l for l in capsys.readouterr().out.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["pairs_per_sec"] > 0 and out["final"]["loss"] is not None


def test_split_k_weight_grad_matches_fp32():
    """wgrad (strided-batched split-K, fp32 partial sums) vs an fp64 product, at a C2 tower shape."""
    import torch
    from mamba_clip_amd.ops import wgrad
    torch.manual_seed(0)
    M, N, K = 50432, 768, 768
    g = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    got = wgrad(g.t(), x)
    ref = (g.double().t() @ x.double()).float()
    assert got.dtype == torch.float32
    rel = float((got - ref).abs().max() / ref.abs().max())
    assert rel < 1e-4, rel          # fp32 accumulation of exact bf16 products
    # channel-major operand (the mixer's in_proj: X = H^T view)
    X = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
    got2 = wgrad(g.t(), X.t())
    ref2 = (g.double().t() @ X.double().t()).float()
    assert float((got2 - ref2).abs().max() / ref2.abs().max()) < 1e-4


def test_ss2d_c1_shape_matches_reference_golden():
    """C1's exact SS2D (BASELINE configs[0]: d_model 128, 16x16 -> L 256, batch 8) on the HIP scan:
    output, input gradient and every parameter gradient vs the reference module."""
    from mamba_clip_amd.model import SS2D
    g = load_golden("ss2d_c1_d128_h16w16.safetensors")
    gen = torch.Generator().manual_seed(2025)
    x = torch.randn(8, 16, 16, 128, generator=gen)
    gy = torch.randn(8, 16, 16, 128, generator=gen)
    chk = torch.stack([x.double().sum(), x.double().abs().sum(), gy.double().sum()])
    torch.testing.assert_close(chk, g["x_checksum"], rtol=0, atol=0)
    m = SS2D(d_model=128).to(DEV).eval()
    m.load_state_dict({k[3:]: v for k, v in g.items() if k.startswith("sd.")})
    xd = x.to(DEV).requires_grad_(True)
    y = m(xd)
    torch.testing.assert_close(y.detach().cpu(), g["y"], rtol=1e-4, atol=1e-5)
    y.backward(gy.to(DEV))
    torch.testing.assert_close(xd.grad.cpu(), g["gx"], rtol=1e-3, atol=1e-5)
    for n, p in m.named_parameters():
        ref = g[f"grad.{n}"]
        torch.testing.assert_close(p.grad.cpu(), ref, rtol=1e-3, atol=1e-4 * float(ref.abs().max()), msg=n)


def test_vssm_tiny_matches_reference_golden():
    """A reduced VSSM end to end (PatchEmbed2D, PatchMerging2D, SS_Conv_SSM stages down to a 1x1 map,
    avgpool head; model.py:868-995): forward, input gradient and head gradient vs the reference."""
    from mamba_clip_amd.model import VSSM
    g = load_golden("vssm_tiny_d16.safetensors")
    m = VSSM(patch_size=4, in_chans=3, num_classes=2, depths=[1, 1, 2, 1], dims=[16, 32, 64, 128]).to(DEV).eval()
    m.load_state_dict({k[3:]: v for k, v in g.items() if k.startswith("sd.")})
    x = g["x"].to(DEV).requires_grad_(True)
    y = m(x)
    torch.testing.assert_close(y.detach().cpu(), g["y"], rtol=1e-4, atol=1e-5)
    y.backward(g["gy"].to(DEV))
    torch.testing.assert_close(x.grad.cpu(), g["gx"], rtol=1e-3, atol=1e-6)
    torch.testing.assert_close(m.head.weight.grad.cpu(), g["grad.head.weight"], rtol=1e-3, atol=1e-6)


def _tiny_bert_clip():
    from mamba_clip_amd.model import BertTextEncoder, ClipModel, VisionTransformer
    return ClipModel(VisionTransformer(img_size=32, patch=8, width=64, layers=2, heads=4, output_dim=32),
                     BertTextEncoder(vocab_size=500, context_length=24, width=64, layers=2, heads=4, output_dim=32))


def test_bert_clip_tiny_matches_cpu_restatement():
    """The BiomedCLIP-shaped tower pair (ViT + PubMedBERT-style encoder, config C3) at tiny width:
    HIP path on cuda vs the same weights on the CPU restatement (oracle_ops), fwd + ClipLoss + bwd."""
    from mamba_clip_amd.loss import ClipLoss
    from oracle.cpu_model import oracle_clip_loss, oracle_ops
    torch.manual_seed(3)
    cpu = _tiny_bert_clip()
    gpu = _tiny_bert_clip()
    gpu.load_state_dict(cpu.state_dict())
    gpu = gpu.to(DEV)
    g = torch.Generator().manual_seed(4)
    img = torch.randn(6, 3, 32, 32, generator=g)
    tok = torch.randint(1, 500, (6, 24), generator=g)
    out = gpu(img.to(DEV), tok.to(DEV))
    loss = ClipLoss()(**out)["contrastive_loss"]
    loss.backward()
    with oracle_ops():
        ref = cpu(img, tok)
        ref_loss = oracle_clip_loss(**ref)["contrastive_loss"]
        ref_loss.backward()
    torch.testing.assert_close(out["text_features"].detach().cpu(), ref["text_features"].detach(), rtol=1e-4,
                               atol=1e-5)
    assert abs(float(loss) - float(ref_loss)) <= 1e-5 * max(1.0, abs(float(ref_loss)))
    rp = dict(cpu.named_parameters())
    for n, p in gpu.named_parameters():
        if p.grad is None:
            continue
        want = rp[n].grad
        err = float((p.grad.cpu() - want).abs().max()) / max(float(want.abs().max()), 1e-12)
        assert err < 5e-3, (n, err)


def test_biomedclip_c3_full_size_trains_on_one_gpu():
    """C3 (BiomedCLIP ViT-B/16 + PubMedBERT-256, BASELINE configs[2]) at its per-GPU shape: batch 64,
    256-token context, amp_bf16, the product train_step.  Tower parity vs open_clip is unpinned
    (absent offline; see test_bert_clip_tiny_matches_cpu_restatement for the arithmetic), so the
    full size is checked by properties: finite, normalised features and a decreasing loss on a fixed batch."""
    from types import SimpleNamespace
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.loss import ClipLoss
    from mamba_clip_amd.model import build_clip
    from mamba_clip_amd.train import create_optimizer, train_step
    torch.manual_seed(0)
    model = build_clip("biomedclip-vit_b16-pubmedbert256").to(DEV)
    assert model.context_length == 256
    args = SimpleNamespace(precision="amp_bf16", lr=1e-4, wd=0.2, beta1=0.9, beta2=0.98, eps=1e-6,
                           grad_clip_norm=None)
    opt = create_optimizer(model, args)
    images, texts, targets = synthetic_batch(64, 224, 256, model.vocab_size, device=DEV, seed=1000)
    losses = [float(train_step(model, images, texts, targets, ClipLoss(), opt, None, args)["loss"])
              for _ in range(4)]
    assert all(torch.isfinite(torch.tensor(losses))), losses
    assert losses[-1] < losses[0], losses
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        out = model(images, texts)
    for k in ("image_features", "text_features"):
        assert out[k].shape == (64, 512)
        torch.testing.assert_close(out[k].float().norm(dim=-1), torch.ones(64, device=DEV), rtol=0, atol=1e-2)


def test_clip_classifier_head_on_frozen_features():
    """Stage-2 (model.py:1174-1192, config C5's head): frozen CLIP features -> MLP logits on the GPU vs
    the CPU restatement; only the head gets gradients; classify = (argmax, softmax)."""
    from mamba_clip_amd.loss import cross_entropy_loss
    from mamba_clip_amd.model import ClipClassifier, build_clip
    from oracle.cpu_model import oracle_ops
    torch.manual_seed(1)
    clip = build_clip("tiny-mamba-clip")
    heads = {}
    for variant in ({}, {"use_inner_prod": True, "feature_dim": 32}, {"use_visual_only": True, "feature_dim": 32}):
        torch.manual_seed(2)
        cpu = ClipClassifier(clip, num_classes=2, **variant)
        gpu = ClipClassifier(build_clip("tiny-mamba-clip"), num_classes=2, **variant)
        gpu.load_state_dict(cpu.state_dict())
        gpu = gpu.to(DEV)
        g = torch.Generator().manual_seed(3)
        img, tok = torch.randn(8, 3, 32, 32, generator=g), torch.randint(1, 999, (8, 16), generator=g)
        tgt = torch.tensor([0, 1, 1, 0, 1, 0, 0, 1])
        logits = gpu(img.to(DEV), tok.to(DEV))
        cross_entropy_loss(logits, tgt.to(DEV), weight=torch.tensor([1.0, 3.0], device=DEV)).backward()
        with oracle_ops():
            ref = cpu(img, tok)
            cross_entropy_loss(ref, tgt, weight=torch.tensor([1.0, 3.0])).backward()
        torch.testing.assert_close(logits.detach().cpu(), ref.detach(), rtol=1e-4, atol=1e-5)
        assert all(p.grad is None for p in gpu.clip_model.parameters())
        rp = dict(cpu.fc.named_parameters())
        for n, p in gpu.fc.named_parameters():
            torch.testing.assert_close(p.grad.cpu(), rp[n].grad, rtol=1e-4, atol=1e-6)
        pred, prob = gpu.classify(img.to(DEV), tok.to(DEV))
        torch.testing.assert_close(prob.sum(1).cpu(), torch.ones(8))
        assert torch.equal(pred.cpu(), ref.argmax(1))
        heads[str(variant)] = logits


def test_glue_ops_take_the_hip_path_for_unaligned_views_and_raise_on_odd_widths():
    """fc1_gelu / qkv_proj backward on the GPU run the HIP kernels (mc_gelu_bwd, mc_qkv_grad_pack)
    for any layout -- an unaligned view is copied to aligned rows first, there is no ATen fallback --
    and a width the kernels cannot tile raises instead of silently leaving the HIP path."""
    from mamba_clip_amd import ops
    torch.manual_seed(5)
    w = torch.randn(64, 40, device=DEV, requires_grad=True)
    bias = torch.randn(64, device=DEV, requires_grad=True)
    base = torch.randn(7 * 41 + 1, device=DEV)
    x = base[1:].view(7, 41)[:, :40].requires_grad_(False)     # unaligned rows (offset 4 B, stride 41)
    calls = []
    orig_load = ops._lib.load
    lib = orig_load()

    class Spy:
        def __getattr__(self, n):
            return getattr(lib, n)

        def mc_gelu_bwd(self, *a):
            calls.append(1)
            return lib.mc_gelu_bwd(*a)
    ops._lib.load = lambda: Spy()
    M = torch.randn(64, 7, device=DEV)
    try:   # the gradient reaching fc1_gelu is M.t(): a transposed (column-major) view
        (ops.fc1_gelu(x, w, bias).t() * M).sum().backward()
    finally:
        ops._lib.load = orig_load
    assert calls, "mc_gelu_bwd was not called"
    xr, wr, br = x.double(), w.detach().double().requires_grad_(True), bias.detach().double().requires_grad_(True)
    (torch.nn.functional.gelu(xr @ wr.T + br).t() * M.double()).sum().backward()
    torch.testing.assert_close(w.grad.double(), wr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bias.grad.double(), br.grad, rtol=1e-4, atol=1e-4)
    w3 = torch.randn(66, 40, device=DEV, requires_grad=True)         # 66 columns: not a multiple of 4
    with pytest.raises(RuntimeError):
        ops.fc1_gelu(x, w3, torch.zeros(66, device=DEV, requires_grad=True)).sum().backward()


@pytest.mark.parametrize("d_model,L", [(256, 64), (768, 80)])
def test_mamba_mixer_projected_delta_matches_unfused_and_oracle(d_model, L):
    """dt_proj inside the scan (ProjectedScanFn, bf16 autocast as C2 trains) against the unfused
    x_proj -> dt_proj -> scan chain and the fp64 oracle (reference model.py:519-528, 630-647):
    output and every parameter / input gradient.  768 is Mamba-130M's width (dt_rank 48)."""
    import mamba_clip_amd.model as M
    torch.manual_seed(d_model)
    m = M.MambaMixer(d_model, d_state=16).to(DEV)
    h = torch.randn(2, L, d_model, device=DEV)
    wts = torch.randn(2, L, d_model, device=DEV)
    taken = []
    real_ok = M.projected_scan_ok
    M.projected_scan_ok = lambda *a: taken.append(real_ok(*a)) or taken[-1]
    runs = []
    try:
        for fuse in (True, False):
            m.fuse_dt_proj = fuse
            m.zero_grad()
            hh = h.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = m(hh)
            (out.float() * wts).sum().backward()
            runs.append((out.detach().float(), hh.grad.clone(), {n: p.grad.clone() for n, p in m.named_parameters()}))
    finally:
        M.projected_scan_ok = real_ok
    assert taken == [True], "the fused path must run for this shape"
    (o_f, gh_f, gp_f), (o_u, gh_u, gp_u) = runs

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()

    assert rel(o_f, o_u) < 1e-2
    assert rel(gh_f, gh_u) < 2e-2
    for n in gp_u:
        assert rel(gp_f[n], gp_u[n]) < 3e-2, n
    ref = R.mamba_mixer_ref(m, h)   # fp64 on the GPU with the module's parameters
    assert rel(o_f, ref) < 2e-2


def test_weight_cast_scope_bitwise_and_model_identical():
    """ops.weight_cast_scope (mc_cast_f32_many: every Linear weight / bias of a model cast to bf16
    in one launch per forward) serves exactly torch's .to(bfloat16) bits, odd sizes included, and
    a bf16-autocast CLIP forward + backward is bitwise the same with and without it."""
    import mamba_clip_amd.ops as O
    from mamba_clip_amd.model import build_clip
    torch.manual_seed(0)
    lin = torch.nn.Sequential(torch.nn.Linear(37, 53), torch.nn.Linear(53, 16, bias=False),
                              torch.nn.Linear(4096, 8192)).to(DEV)   # 33.6M elements: several chunks
    with O.weight_cast_scope(lin, torch.bfloat16):
        for p in lin.parameters():
            got = O._wcast(p, torch.bfloat16)
            assert got.data_ptr() != p.data_ptr() and torch.equal(got, p.to(torch.bfloat16))
    assert O._WCAST is None
    model = build_clip("tiny-mamba-clip").to(DEV)
    images = torch.randn(4, 3, 32, 32, device=DEV)
    texts = torch.randint(1, 999, (4, 16), device=DEV)
    runs = []
    for use in (True, False):
        model.zero_grad()
        real = O.weight_cast_scope.__enter__
        if not use:
            O.weight_cast_scope.__enter__ = lambda self: self
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(images, texts)
            (out["image_features"].float().sum() + out["text_features"].float().square().sum()).backward()
        finally:
            O.weight_cast_scope.__enter__ = real
        runs.append([out["image_features"].detach().clone()] + [p.grad.clone() for p in model.parameters()
                                                                 if p.grad is not None])
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_weight_cast_scope_transposed_copies(dt):
    """mc_cast_transpose_f32_many (the scope's transposed copies for the "tn" input gradients) gives
    exactly w.to(dt).t() -- full 64 x 64 tiles, ragged edges and an odd leading dimension -- and a
    LinearSK input gradient served from them is bitwise the per-call transpose's."""
    import mamba_clip_amd.ops as O
    torch.manual_seed(1)
    ws = [torch.randn(r, c, device=DEV) for r, c in [(2304, 768), (768, 3072), (100, 70), (1, 5), (67, 129)]]
    plan = O._TransposePlan(ws, dt, DEV)
    for w, t in zip(ws, plan.run(ws)):
        assert t.shape == (w.shape[1], w.shape[0]) and torch.equal(t, w.to(dt).t())
    # the scope: the first forward registers, the next ones are served
    lin = torch.nn.Linear(768, 3072).to(DEV)
    x = torch.randn(8192 + 64, 768, device=DEV, dtype=dt)
    g = torch.randn(8192 + 64, 3072, device=DEV, dtype=dt)
    grads = []
    for _ in range(3):
        xx = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=dt), O.weight_cast_scope(lin, dt):
            y = O.LinearSK.apply(xx, lin.weight, lin.bias)
            served = O._WCAST_T is not None and id(lin.weight) in O._WCAST_T
        y.backward(g)
        grads.append((served, xx.grad.clone()))
    assert [s for s, _ in grads] == [False, True, True]
    assert torch.equal(grads[0][1], grads[1][1]) and torch.equal(grads[1][1], grads[2][1])


@pytest.mark.parametrize("M,N,K", [(50432, 2304, 768), (20480, 80, 1536), (20480, 1536, 48), (16384, 37, 5)])
def test_wgrad_split_k_slab_sum(M, N, K):
    """ops.wgrad (split-K strided-batched GEMM + mc_sum_slabs) against one fp32 GEMM of the same
    bf16 operands: only the summation order differs.  (37, 5): the scalar slab-sum path."""
    from mamba_clip_amd.ops import _split_factor, wgrad
    g = torch.Generator(device=DEV).manual_seed(M + N)
    G = torch.randn(N, M, device=DEV, generator=g).bfloat16()
    X = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    assert _split_factor(M, N, K) > 1
    got = wgrad(G, X)
    ref = G.double() @ X.double()
    assert got.dtype == torch.float32 and got.shape == (N, K)
    assert ((got.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5


@pytest.mark.parametrize("text_tower", ["mamba", "bert"])
def test_concurrent_towers_bitwise_identical(text_tower):
    """ClipModel runs the text tower on a second HIP stream beside the image tower -- beside a Mamba
    tower (C2) and beside a BERT tower (C3), whose library GEMMs now also run concurrently with the
    ViT's (data-parallel grids, mamba_clip_amd.GEMM_GRIDS_DATA_PARALLEL): features, loss and every
    gradient bitwise equal to the sequential forward / backward (same kernels, same order per tower;
    autograd joins the streams)."""
    import mamba_clip_amd
    from mamba_clip_amd.model import BertTextEncoder, ClipModel, VisionTransformer, init_model
    from mamba_clip_amd.loss import ClipLoss
    assert mamba_clip_amd.GEMM_GRIDS_DATA_PARALLEL
    torch.manual_seed(0)
    if text_tower == "mamba":
        model, _, _, _ = init_model("tiny-mamba-clip")
    else:
        model = ClipModel(VisionTransformer(img_size=32, patch=8, width=64, layers=2, heads=4, output_dim=32),
                          BertTextEncoder(vocab_size=1000, context_length=16, width=64, layers=2, heads=4,
                                          output_dim=32))
    model = model.to(DEV)
    img = torch.randn(8, 3, 32, 32, device=DEV)
    tok = torch.randint(1, 1000, (8, 16), device=DEV)
    runs = []
    for conc in (True, False):
        model.concurrent_towers = conc
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(img, tok)
            loss = ClipLoss()(**out)["contrastive_loss"]
        loss.backward()
        torch.cuda.synchronize()
        runs.append((out["text_features"].detach().clone(), loss.detach().clone(),
                     {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}))
        del out, loss   # no graph (and no AccumulateGrad node) survives into the next run
    (tf1, l1, g1), (tf0, l0, g0) = runs
    assert torch.equal(tf1, tf0) and torch.equal(l1, l0)
    assert g1.keys() == g0.keys() and len(g0) > 10
    for n in g0:
        assert torch.equal(g1[n], g0[n]), n


@pytest.mark.parametrize("conc", [False, True])
def test_grad_checkpointing_bitwise_gpu(conc):
    """Per-block / per-layer activation checkpointing on the HIP path (also with the text tower on its
    side stream, where the recompute runs during that stream's backward): gradients bitwise equal to
    the run that keeps the activations (deterministic kernels recompute identical values)."""
    from mamba_clip_amd.model import init_model
    from mamba_clip_amd.loss import ClipLoss
    torch.manual_seed(0)
    model, _, _, _ = init_model("tiny-mamba-clip")
    model = model.to(DEV)
    model.concurrent_towers = conc
    img = torch.randn(8, 3, 32, 32, device=DEV)
    tok = torch.randint(1, 1000, (8, 16), device=DEV)
    runs = []
    for ck in (False, True):
        model.set_grad_checkpointing(ck)
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(img, tok)
            loss = ClipLoss()(**out)["contrastive_loss"]
        loss.backward()
        torch.cuda.synchronize()
        runs.append((loss.detach().clone(), {n: p.grad.clone() for n, p in model.named_parameters()
                                             if p.grad is not None}))
        del out, loss
    (l0, g0), (l1, g1) = runs
    assert torch.equal(l0, l1)
    assert g0.keys() == g1.keys() and len(g0) > 10
    for n in g0:
        assert torch.equal(g1[n], g0[n]), n
