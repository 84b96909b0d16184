"""GPU checks of the fused short-sequence attention (mc_attn_fwd / mc_attn_bwd, ops.PackedAttentionFn)
against an fp64 restatement of softmax(q k^T / sqrt(D)) v on the same 16-bit inputs, and of the
towers' Attention module (fused vs torch SDPA).  The reference reaches this op through timm /
open_clip / HF attention (model.py:1019-1064 builds the towers).

Tolerances: the kernel rounds P and dS to the input dtype before the P V / dS K products (as every
flash-style kernel does), so outputs are compared with a normalised error ||got - ref|| / ||ref||:
<= 8e-3 for o (bf16 output rounding alone is ~3e-3), <= 2e-2 for dq / dk / dv; lse to 1e-5."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(q, k, v, scale):
    """fp64 attention + lse; q, k, v (B, N, H, D)."""
    qd, kd, vd = (t.double() for t in (q, k, v))
    s = torch.einsum("bnhd,bmhd->bhnm", qd, kd) * scale
    lse = torch.logsumexp(s, -1)
    o = torch.einsum("bhnm,bmhd->bnhd", torch.softmax(s, -1), vd)
    return o, lse


def _nerr(a, b, floor=1e-30):
    """||a - b|| / max(||b||, floor): the floor covers gradients that vanish exactly (N = 1: dq = dk = 0)."""
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(floor)).item()


def _packed(B, N, H, D, dt, g):
    return (torch.randn(B, N, 3 * H * D, generator=g) * 1.5).to(dt).to(DEV)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N", [1, 7, 32, 50, 197, 224, 256])
def test_packed_attention_fwd_bwd_vs_fp64(N, dt):
    from mamba_clip_amd.ops import packed_attention
    g = torch.Generator().manual_seed(N)
    B, H, D = 2, 3, 64
    C = H * D
    qkv = _packed(B, N, H, D, dt, g).requires_grad_(True)
    o = packed_attention(qkv, H)
    go = torch.randn(B, N, C, generator=g).to(dt).to(DEV)
    o.backward(go)
    torch.cuda.synchronize()
    # fp64 reference on the same 16-bit inputs
    ref_in = qkv.detach().double().requires_grad_(True)
    q, k, v = ref_in.view(B, N, 3, H, D).unbind(2)
    ro, rlse = _ref(q, k, v, D ** -0.5)
    ro.reshape(B, N, C).backward(go.double())
    assert o.shape == (B, N, C) and o.dtype == dt
    assert _nerr(o, ro.reshape(B, N, C)) < 8e-3
    dq, dk, dv = qkv.grad.view(B, N, 3, H, D).unbind(2)
    rq, rk, rv = ref_in.grad.view(B, N, 3, H, D).unbind(2)
    floor = 1e-3 * ref_in.grad.norm().item()
    for name, a, b in (("dq", dq, rq), ("dk", dk, rk), ("dv", dv, rv)):
        assert _nerr(a, b, floor) < 2e-2, name


def test_packed_attention_lse_and_determinism():
    from mamba_clip_amd import _lib
    from mamba_clip_amd.ops import PackedAttentionFn
    g = torch.Generator().manual_seed(5)
    B, N, H, D = 3, 197, 12, 64
    qkv = _packed(B, N, H, D, torch.bfloat16, g).requires_grad_(True)
    o1 = PackedAttentionFn.apply(qkv, H)
    go = torch.randn_like(o1)
    (g1,) = torch.autograd.grad(o1, qkv, go)
    o2 = PackedAttentionFn.apply(qkv, H)
    (g2,) = torch.autograd.grad(o2, qkv, go)
    assert torch.equal(o1, o2) and torch.equal(g1, g2)   # no atomics: bitwise reproducible
    # lse straight from the C ABI
    lib = _lib.load()
    y = qkv.detach()
    o = torch.empty(B, N, H * D, device=DEV, dtype=y.dtype)
    lse = torch.empty(B, H, N, device=DEV)
    p = _lib.AttnFwdParams()
    p.batch, p.heads, p.seqlen, p.head_dim, p.dtype, p.scale = B, H, N, D, _lib.MC_DTYPE_BF16, 0.125
    es = y.element_size()
    p.q, p.k, p.v = y.data_ptr(), y.data_ptr() + H * D * es, y.data_ptr() + 2 * H * D * es
    p.q_bs, p.q_ns, p.q_hs = y.stride(0), y.stride(1), D
    p.o, p.o_bs, p.o_ns, p.o_hs, p.lse = o.data_ptr(), o.stride(0), o.stride(1), D, lse.data_ptr()
    _lib.check(lib.mc_attn_fwd(p, _lib.stream_handle()), "mc_attn_fwd")
    torch.cuda.synchronize()
    q, k, v = y.view(B, N, 3, H, D).unbind(2)
    _, rlse = _ref(q, k, v, 0.125)
    assert (lse.double() - rlse).abs().max().item() < 1e-5 * max(1.0, rlse.abs().max().item())
    assert torch.equal(o, o1.detach())


def test_packed_attention_rejects_unsupported():
    from mamba_clip_amd.ops import packed_attention
    with pytest.raises(RuntimeError, match="unsupported"):
        packed_attention(torch.zeros(1, 257, 3 * 64, device=DEV, dtype=torch.bfloat16), 1)
    with pytest.raises(RuntimeError, match="unsupported"):
        packed_attention(torch.zeros(1, 16, 3 * 128, device=DEV, dtype=torch.bfloat16), 1)
    with pytest.raises(RuntimeError, match="unsupported"):
        packed_attention(torch.zeros(1, 16, 3 * 64, device=DEV, dtype=torch.float32), 1)


@pytest.mark.parametrize("N", [197, 256])
def test_tower_attention_fused_matches_sdpa(N):
    """model.Attention under bf16 autocast (as C2 / C3 train): the fused path (packed qkv ->
    mc_attn -> proj) against the SDPA path with the same weights: output, input and every
    parameter gradient."""
    from mamba_clip_amd.model import Attention
    torch.manual_seed(N)
    m = Attention(768, 12).to(DEV)
    x = torch.randn(4, N, 768, device=DEV)
    gy = torch.randn(4, N, 768, device=DEV)
    runs = []
    for fused in (True, False):
        m.fused_attention = fused
        m.zero_grad()
        xx = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(xx)
        (y.float() * gy).sum().backward()
        runs.append((y.detach().float(), xx.grad.clone(), {n: p.grad.clone() for n, p in m.named_parameters()}))
    (yf, gxf, gpf), (yu, gxu, gpu) = runs
    assert _nerr(yf, yu) < 1e-2
    assert _nerr(gxf, gxu) < 2e-2
    for n in gpu:
        assert _nerr(gpf[n], gpu[n]) < 2e-2, n


@pytest.mark.parametrize("N", [64, 197])
def test_packed_attention_many_heads_persistent_backward(N):
    """More (batch, head) pairs than CUs: the persistent backward walks several heads per workgroup and
    streams the next head's q / dO / O into LDS during phase 2 -- every head must match the fp64
    reference (reference on the GPU in fp64, same 16-bit inputs)."""
    from mamba_clip_amd.ops import packed_attention
    g = torch.Generator().manual_seed(N + 1)
    B, H, D = 40, 12, 64            # 480 heads > 256 CUs
    C = H * D
    qkv = _packed(B, N, H, D, torch.bfloat16, g).requires_grad_(True)
    o = packed_attention(qkv, H)
    go = torch.randn(B, N, C, generator=g).to(torch.bfloat16).to(DEV)
    o.backward(go)
    ref_in = qkv.detach().double().requires_grad_(True)
    q, k, v = ref_in.view(B, N, 3, H, D).unbind(2)
    ro, _ = _ref(q, k, v, D ** -0.5)
    ro.reshape(B, N, C).backward(go.double())
    assert _nerr(o, ro.reshape(B, N, C)) < 8e-3
    got = qkv.grad.view(B, N, 3, H, D).double()
    want = ref_in.grad.view(B, N, 3, H, D)
    for bh in range(0, B * H, 37):     # per-head check on a spread of heads (any mix-up shows per head)
        b, h = divmod(bh, H)
        for s in range(3):
            assert _nerr(got[b, :, s, h], want[b, :, s, h], 1e-3 * want[b, :, s, h].norm().item() + 1e-12) < 3e-2, (b, h, s)
    assert _nerr(got, want) < 2e-2
