"""The Mamba mixer's fused projections (include/mc_ops.h mc_mixer_proj_fwd / _bwd, ops.MixerProjFn) vs
fp64 restatements of the library-GEMM chain they replace -- x_dbl = x_proj(x), delta = dt_proj.weight
@ dt_raw; d_dtraw = dt_proj.weight^T @ ddelta, dx = x_proj.weight^T @ [d_dtraw; dB; dC] + du -- with
the same roundings (each product stored once in the 16-bit dtype), and the whole mixer fused vs
unfused."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [(128, 64, 16), (1536, 2560, 48), (3072, 1024, 96), (256, 200, 32), (1536, 20480, 48)]


def _bound(ref, dtype):
    """|err| bound for a value stored once in `dtype` after an fp32 accumulation: one rounding of the
    value plus the accumulation-order difference (relative to the row's scale)."""
    u = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    return u * ref.abs() + 1e-3 * float(ref.abs().max()) + 1e-6


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_mixer_proj_fwd_bwd_matches_gemm_chain(shape, dtype):
    from mamba_clip_amd.ops import GradHandoff, mixer_proj
    D, T, R = shape
    P = R + 32
    g = torch.Generator().manual_seed(D + T + R)
    x = torch.randn(D, T, generator=g).to(dtype)
    wx = torch.randn(P, D, generator=g) * D ** -0.5
    wdt = torch.randn(D, R, generator=g) * R ** -0.5
    gxd = torch.randn(P, T, generator=g).to(dtype)
    gxd[:R] = 0                                   # dt_raw only feeds dt_proj inside the op
    gdl = torch.randn(D, T, generator=g).to(dtype)
    du = torch.randn(D, T, generator=g).to(dtype)
    # device run (weights as fp32 parameters, cast to the dtype like autocast)
    xg = x.to(DEV).requires_grad_(True)
    wxg, wdtg = wx.to(DEV).requires_grad_(True), wdt.to(DEV).requires_grad_(True)
    hand = GradHandoff()
    with torch.autocast("cuda", dtype=dtype):
        gb_rows, gc_rows, dl = mixer_proj(xg, wxg, wdtg, hand)
    assert dl.dtype == dtype and gb_rows.shape == (16, T) and gc_rows.shape == (16, T) and dl.shape == (D, T)
    xd = gb_rows._base                                     # the whole x_dbl (P, T) the rows view
    assert xd is not None and xd.shape == (P, T)
    hand.du = du.to(DEV).view(D, 1, T).transpose(0, 1)     # the scan parks du as (B, D, L): here B = 1
    torch.autograd.backward([gb_rows, gc_rows, dl], [gxd[R:R + 16].to(DEV), gxd[R + 16:].to(DEV), gdl.to(DEV)])
    assert hand.du is None
    # fp64 chain on the same 16-bit operands, each product rounded once to the dtype
    x64, wx64, wdt64 = x.double(), wx.to(dtype).double(), wdt.to(dtype).double()
    xd_exact = wx64 @ x64
    xd_got = xd.detach().cpu()
    assert ((xd_got.double() - xd_exact).abs() <= _bound(xd_exact, dtype)).all()
    dl_exact = wdt64 @ xd_got[:R].double()           # delta from the kernel's own (rounded) dt_raw
    assert ((dl.detach().cpu().double() - dl_exact).abs() <= _bound(dl_exact, dtype)).all()
    ddt = wdt64.t() @ gdl.double()
    dxd_exact = torch.cat([ddt, gxd[R:].double()])
    dxd_r = dxd_exact.to(dtype).double()
    dx_exact = wx64.t() @ dxd_r + du.double()
    assert ((xg.grad.cpu().double() - dx_exact).abs() <= _bound(dx_exact, dtype) + 2e-3 * float(dx_exact.abs().max())).all()
    # weight gradients: ops.wgrad, as in the library chain (fp32 split-K sums at T >= 8192; below that
    # one 16-bit GEMM, so one 16-bit rounding)
    dwx_exact = dxd_r @ x64.t()
    dwdt_exact = gdl.double() @ xd_got[:R].double().t()
    rt = 1e-3 if T >= 8192 else 2.0 ** -7
    torch.testing.assert_close(wxg.grad.cpu().double(), dwx_exact, rtol=2e-2, atol=2e-2 * float(dwx_exact.abs().max()))
    torch.testing.assert_close(wdtg.grad.cpu().double(), dwdt_exact, rtol=rt, atol=rt * float(dwdt_exact.abs().max()))


def test_mixer_proj_rejects_bad_shapes():
    from mamba_clip_amd.ops import mixer_proj, mixer_proj_ok
    x = torch.randn(100, 64, device=DEV, dtype=torch.bfloat16)
    assert not mixer_proj_ok(x, 48, 16)                         # D % 64
    assert not mixer_proj_ok(torch.randn(128, 64, device=DEV, dtype=torch.bfloat16), 8, 16)   # rank % 16
    assert not mixer_proj_ok(torch.randn(128, 64, device=DEV), 16, 16)                       # fp32 (no autocast)
    with pytest.raises(RuntimeError, match="proj_rows"):
        mixer_proj(torch.randn(128, 64, device=DEV, dtype=torch.bfloat16),
                   torch.randn(64, 128, device=DEV, dtype=torch.bfloat16),
                   torch.randn(128, 16, device=DEV, dtype=torch.bfloat16))   # P = 64 != R + 32


@pytest.mark.parametrize("d_model,L", [(768, 80), (1536, 64)])
def test_mamba_mixer_fused_projections_match_unfused(d_model, L):
    """The whole mixer under bf16 autocast: fused projections vs the library-GEMM chain (same model,
    same inputs) -- output, input gradient and every parameter gradient within bf16 rounding."""
    from mamba_clip_amd.model import MambaMixer
    torch.manual_seed(3)
    m = MambaMixer(d_model, d_state=16).to(DEV)
    assert m.dt_rank % 16 == 0
    h = torch.randn(4, L, d_model, device=DEV)
    gy = torch.randn(4, L, d_model, device=DEV)
    res = []
    for fused in (True, False):
        m.fuse_proj = fused
        m.zero_grad(set_to_none=True)
        hh = h.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(hh)
        (y.float() * gy).sum().backward()
        res.append((y.float().detach(), hh.grad.clone(), {n: p.grad.clone() for n, p in m.named_parameters()}))
    (y1, g1, p1), (y0, g0, p0) = res

    def rel(a, b):
        return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))
    assert rel(y1, y0) < 2e-2
    assert rel(g1, g0) < 3e-2
    for n in p0:
        assert rel(p1[n], p0[n]) < 3e-2, n
