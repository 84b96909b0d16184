"""GPU parity of the contrastive-loss kernels (MFMA logits + fused CE) against
the reference loss.py golden vectors and the fp32 torch oracle."""
import pytest
import torch

from conftest import load_golden
from oracle.loss_ref import clip_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_gemm_nt_exact_fp32_and_bf16():
    from mamba_clip_amd.ops import gemm_nt
    g = torch.Generator().manual_seed(0)
    for (M, N, K) in [(1, 1, 8), (130, 257, 512), (256, 256, 512), (77, 300, 40), (512, 64, 768)]:
        A = torch.randn(M, K, generator=g)
        B = torch.randn(N, K, generator=g)
        ref = (A.double() @ B.double().T).float()
        C = gemm_nt(A.to(DEV), B.to(DEV), alpha=1.0).cpu()
        torch.testing.assert_close(C, ref, rtol=1e-5, atol=1e-4 * K ** 0.5)
        Ab, Bb = A.bfloat16(), B.bfloat16()
        refb = (Ab.double() @ Bb.double().T).float() * 2.5
        Cb = gemm_nt(Ab.to(DEV), Bb.to(DEV), alpha=2.5).cpu()
        torch.testing.assert_close(Cb, refb, rtol=1e-5, atol=1e-4 * K ** 0.5)
    # asymmetric operand check (catches a transposed C write)
    A = torch.eye(64)
    B = torch.arange(64 * 64, dtype=torch.float32).reshape(64, 64)
    torch.testing.assert_close(gemm_nt(A.to(DEV), B.to(DEV)).cpu(), B.T.contiguous())
    s = torch.tensor(3.0, device=DEV)
    torch.testing.assert_close(gemm_nt(A.to(DEV), B.to(DEV), alpha_dev=s).cpu(), 3 * B.T)


@pytest.mark.parametrize("fname", ["clip_loss_single_n8_e16.safetensors", "clip_loss_single_n64_e32.safetensors"])
def test_clip_loss_single_process_matches_reference(fname):
    from mamba_clip_amd.loss import ClipLoss
    g = load_golden(fname)
    img = g["img"].to(DEV).requires_grad_(True)
    txt = g["txt"].to(DEV).requires_grad_(True)
    s = g["scale"][0].to(DEV).requires_grad_(True)
    out = ClipLoss()(img, txt, s)
    loss = out["contrastive_loss"]
    loss.backward()
    torch.testing.assert_close(loss.detach().cpu().reshape(1), g["loss"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(img.grad.cpu(), g["grad_img"], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(txt.grad.cpu(), g["grad_txt"], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(s.grad.cpu().reshape(1), g["grad_scale"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("N,E", [(256, 512), (1000, 512), (8192, 512)])
def test_clip_loss_bf16_within_1e3(N, E):
    """bf16 features (autocast path): loss within 1e-3 rel of the fp32 oracle on the
    SAME bf16-rounded inputs (north_star tolerance); grads within 1e-2 rel."""
    from mamba_clip_amd.loss import ClipLoss
    g = torch.Generator().manual_seed(N)
    img = torch.nn.functional.normalize(torch.randn(N, E, generator=g), dim=-1).bfloat16()
    txt = torch.nn.functional.normalize(torch.randn(N, E, generator=g), dim=-1).bfloat16()
    ref_i = img.float().requires_grad_(True)
    ref_t = txt.float().requires_grad_(True)
    ref_s = torch.tensor(14.0, requires_grad=True)
    ref = clip_loss(ref_i, ref_t, ref_s)
    ref.backward()
    i_d = img.to(DEV).requires_grad_(True)
    t_d = txt.to(DEV).requires_grad_(True)
    s_d = torch.tensor(14.0, device=DEV, requires_grad=True)
    loss = ClipLoss()(i_d, t_d, s_d)["contrastive_loss"]
    loss.backward()
    assert abs(float(loss) - float(ref)) <= 1e-3 * abs(float(ref))
    for got, want in ((i_d.grad, ref_i.grad), (t_d.grad, ref_t.grad)):
        got = got.float().cpu()
        scale = float(want.abs().max())
        assert float((got - want).abs().max()) <= 1e-2 * scale
    assert abs(float(s_d.grad) - float(ref_s.grad)) <= 1e-3 * abs(float(ref_s.grad)) + 1e-4


def test_get_logits_matches_reference_semantics():
    from mamba_clip_amd.loss import ClipLoss
    g = torch.Generator().manual_seed(1)
    img = torch.randn(33, 64, generator=g)
    txt = torch.randn(33, 64, generator=g)
    li, lt = ClipLoss().get_logits(img.to(DEV), txt.to(DEV), torch.tensor(2.0, device=DEV))
    torch.testing.assert_close(li.cpu(), 2 * img @ txt.T, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(lt.cpu(), 2 * txt @ img.T, rtol=1e-5, atol=1e-4)


def _ce_oracle(X, Y, scale, row_off, coef_r, col_off=0, coef_c=0.0):
    """fp64 restatement of the dense part of ClipLoss (loss.py:102-145): rows i -> label i + row_off,
    columns j -> label j + col_off."""
    S = scale * X @ Y.T
    r = torch.arange(S.shape[0])
    loss = coef_r * (torch.logsumexp(S, 1) - S[r, r + row_off]).sum()
    if coef_c:
        c = torch.arange(S.shape[1])
        loss = loss + coef_c * (torch.logsumexp(S, 0) - S[c + col_off, c]).sum()
    return loss


@pytest.mark.parametrize("b,world,E", [(5, 3, 64), (64, 8, 512), (7, 2, 24), (130, 4, 512)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_scaled_logits_ce_local_loss_rectangular(b, world, E, dtype):
    """The local_loss path (loss.py:80-81, 101-103) on the HIP kernels: rectangular (b x N) logits,
    row labels offset by b*rank, no column term; loss, dX, dY and d(scale) vs fp64, every rank."""
    from mamba_clip_amd.ops import scaled_logits_ce
    N = b * world
    g = torch.Generator().manual_seed(b * 1000 + world)
    Yall = torch.nn.functional.normalize(torch.randn(N, E, generator=g), dim=-1).to(dtype)
    Xall = torch.nn.functional.normalize(torch.randn(N, E, generator=g), dim=-1).to(dtype)
    for rank in range(world):
        X = Xall[rank * b:(rank + 1) * b]
        xr = X.double().requires_grad_(True)
        yr = Yall.double().requires_grad_(True)
        sr = torch.tensor(12.5, dtype=torch.float64, requires_grad=True)
        ref = _ce_oracle(xr, yr, sr, b * rank, 0.5 / b)
        ref.backward()
        xd = X.to(DEV).requires_grad_(True)
        yd = Yall.to(DEV).requires_grad_(True)
        sd = torch.tensor(12.5, device=DEV, requires_grad=True)
        loss = scaled_logits_ce(xd, yd, sd, b * rank, 0.5 / b)
        loss.backward()
        tol = 1e-5 if dtype == torch.float32 else 1e-3
        assert abs(float(loss) - float(ref)) <= tol * abs(float(ref)) + 1e-6, (rank, float(loss), float(ref))
        for got, want in ((xd.grad, xr.grad), (yd.grad, yr.grad)):
            scale = float(want.abs().max())
            err = float((got.double().cpu() - want).abs().max())
            assert err <= (1e-5 if dtype == torch.float32 else 1e-2) * scale, (rank, err, scale)
        assert abs(float(sd.grad) - float(sr.grad)) <= tol * abs(float(sr.grad)) + 1e-5


@pytest.mark.parametrize("world", [2, 4])
def test_local_loss_matches_reference_gloo_golden(world):
    """Per rank, ClipLoss(local_loss=True)'s dense math on the HIP kernels (the feature gather done
    from the golden's global features) equals the reference's gloo results ll1_gg0 (loss.py as-is)."""
    from mamba_clip_amd.ops import scaled_logits_ce
    g = load_golden(f"clip_loss_gloo_w{world}.safetensors")
    b = g["img"].shape[0] // world
    all_i, all_t = g["img"].to(DEV), g["txt"].to(DEV)
    for rank in range(world):
        img = all_i[rank * b:(rank + 1) * b].clone().requires_grad_(True)
        txt = all_t[rank * b:(rank + 1) * b].clone().requires_grad_(True)
        s = torch.tensor(10.0, device=DEV, requires_grad=True)
        # loss.py:105-108 local branch; gathered copies carry no grad (gather_with_grad False)
        loss = (scaled_logits_ce(img, all_t, s, b * rank, 0.5 / b)
                + scaled_logits_ce(txt, all_i, s, b * rank, 0.5 / b))
        loss.backward()
        key = f"r{rank}.ll1_gg0"
        torch.testing.assert_close(loss.detach().cpu().reshape(1), g[f"{key}.loss"], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(img.grad.cpu(), g[f"{key}.grad_img"], rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(txt.grad.cpu(), g[f"{key}.grad_txt"], rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(s.grad.cpu().reshape(1), g[f"{key}.grad_scale"], rtol=1e-4, atol=1e-6)


# ---------------------------------------------------------------- fused logits + CE (mc_ce_fused_*)
@pytest.mark.parametrize("M,N,E,coef_c,dtype", [(1000, 1000, 64, 0.5 / 1000, torch.float32),
                                               (300, 1100, 96, 0.0, torch.float32),
                                               (640, 640, 128, 0.5 / 640, torch.bfloat16)])
def test_fused_ce_blocked_backward(monkeypatch, M, N, E, coef_c, dtype):
    """Force several G blocks per pass (row blocks for dX, column blocks for dY with the transposed
    problem) and check loss / dX / dY / d(scale) against fp64, with label offsets on both axes."""
    from mamba_clip_amd import ops
    monkeypatch.setattr(ops, "CE_GRAD_BLOCK_ELEMS", 128 * 256)
    g = torch.Generator().manual_seed(M + N)
    X = torch.nn.functional.normalize(torch.randn(M, E, generator=g), dim=-1).to(dtype)
    Y = torch.nn.functional.normalize(torch.randn(N, E, generator=g), dim=-1).to(dtype)
    roff = (N - M) // 2
    coff = 0
    xr, yr = X.double().requires_grad_(True), Y.double().requires_grad_(True)
    sr = torch.tensor(20.0, dtype=torch.float64, requires_grad=True)
    ref = _ce_oracle(xr, yr, sr, roff, 0.5 / M, coff, coef_c)
    ref.backward()
    xd, yd = X.to(DEV).requires_grad_(True), Y.to(DEV).requires_grad_(True)
    sd = torch.tensor(20.0, device=DEV, requires_grad=True)
    loss = ops.scaled_logits_ce(xd, yd, sd, roff, 0.5 / M, coff, coef_c)
    loss.backward()
    tol = 1e-5 if dtype == torch.float32 else 1e-3
    assert abs(float(loss) - float(ref)) <= tol * abs(float(ref)) + 1e-6
    for got, want in ((xd.grad, xr.grad), (yd.grad, yr.grad)):
        scale = float(want.abs().max())
        err = float((got.double().cpu() - want).abs().max())
        assert err <= (1e-5 if dtype == torch.float32 else 1e-2) * scale, (err, scale)
    assert abs(float(sd.grad) - float(sr.grad)) <= tol * abs(float(sr.grad)) + 1e-5


def test_fused_ce_no_n_by_n_allocation_c5_size():
    """N = 8192 (config 5's global batch), bf16: forward + backward never allocate an N x N buffer
    (peak growth stays below one bf16 N x N matrix), and the loss / lse agree with the unfused
    kernels over a materialised S."""
    from mamba_clip_amd.ops import ce_fused_fwd, ce_stats, gemm_nt, scaled_logits_ce
    N, E = 8192, 512
    g = torch.Generator().manual_seed(5)
    img = torch.nn.functional.normalize(torch.randn(N, E, generator=g), dim=-1).bfloat16().to(DEV)
    txt = torch.nn.functional.normalize(torch.randn(N, E, generator=g), dim=-1).bfloat16().to(DEV)
    s = torch.tensor(30.0, device=DEV, requires_grad=True)
    i_d, t_d = img.clone().requires_grad_(True), txt.clone().requires_grad_(True)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    loss = scaled_logits_ce(i_d, t_d, s, 0, 0.5 / N, 0, 0.5 / N)
    loss.backward()
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    assert peak < N * N * 2, f"peak {peak / 2**20:.1f} MiB >= one bf16 N x N"
    # unfused reference on the same device: S materialised once, row / column stats
    S = gemm_nt(img, txt, alpha_dev=s.detach())
    lr, l_r = ce_stats(S, 0, 0, 0.5 / N)
    lc, l_c = ce_stats(S, 1, 0, 0.5 / N)
    l2, lse_r, lse_c = ce_fused_fwd(img, txt, s.detach(), 0, 0.5 / N, 0, 0.5 / N)
    torch.testing.assert_close(lse_r, lr, rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(lse_c, lc, rtol=1e-6, atol=1e-5)
    assert abs(float(l2) - float(l_r + l_c)) <= 1e-5 * float(l_r + l_c)
    assert abs(float(loss) - float(l2)) <= 1e-6 * float(l2)
    assert torch.isfinite(i_d.grad).all() and torch.isfinite(t_d.grad).all()


def test_unfused_ce_kernels_match_fp64():
    """mc_ce_stats / mc_ce_grad over a materialised S (rows and columns, label offsets)."""
    from mamba_clip_amd.ops import ce_grad, ce_stats
    g = torch.Generator().manual_seed(3)
    S = (torch.randn(70, 300, generator=g) * 8).double()
    lr_ref = torch.logsumexp(S, 1)
    lc_ref = torch.logsumexp(S, 0)
    Sd = S.float().to(DEV)
    lr, loss_r = ce_stats(Sd, 0, 11, 0.25)
    lc, loss_c = ce_stats(Sd, 1, -5, 0.5)
    torch.testing.assert_close(lr.cpu().double(), lr_ref, rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(lc.cpu().double(), lc_ref, rtol=1e-6, atol=1e-5)
    r = torch.arange(70)
    c = torch.arange(300)
    want_r = 0.25 * (lr_ref - S[r, r + 11]).sum()
    ok = (c - 5 >= 0) & (c - 5 < 70)
    want_c = 0.5 * (lc_ref - torch.where(ok, S[(c - 5).clamp(0, 69), c], torch.zeros(300, dtype=S.dtype))).sum()
    assert abs(float(loss_r) - float(want_r)) <= 1e-5 * abs(float(want_r))
    assert abs(float(loss_c) - float(want_c)) <= 1e-5 * abs(float(want_c))
    sc = torch.tensor(2.0, device=DEV)
    G, ds = ce_grad(Sd, lr, 11, 0.25, lc, -5, 0.5, torch.tensor(1.5, device=DEV), torch.float32, sc)
    P_r = torch.softmax(S, 1)
    P_c = torch.softmax(S, 0)
    Gr = 0.25 * (P_r - torch.nn.functional.one_hot(r + 11, 300).double())
    oh_c = torch.zeros(70, 300, dtype=torch.float64)
    oh_c[(c - 5)[ok], c[ok]] = 1
    Gw = 1.5 * (Gr + 0.5 * (P_c - oh_c))
    torch.testing.assert_close(G.cpu().double(), Gw, rtol=1e-5, atol=1e-6)
    assert abs(float(ds) - float((Gw * S).sum() / 2.0)) <= 1e-4 * abs(float((Gw * S).sum() / 2.0)) + 1e-5


def test_fp32_ce_backward_products_stay_fp32_with_tf32_flag_on():
    """The fused CE backward's fp32 products (ops._mm_nt: dX = G @ Y, dY = G^T @ X) run the exact-fp32
    MFMA GEMM, so the process-wide allow_tf32 flag (set by init_device like the reference,
    utils/dist_utils.py:41-43) neither changes them nor is touched by them."""
    from mamba_clip_amd.ops import _mm_nt
    prev = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = True
    try:
        g = torch.Generator(device=DEV).manual_seed(3)
        a = torch.randn(512, 2048, device=DEV, generator=g)
        b = torch.randn(2048, 384, device=DEV, generator=g)
        out = torch.empty(768, 384, device=DEV)[100:612]         # a row block of a larger buffer
        _mm_nt(a, b.t().contiguous(), out)
        ref = a.double() @ b.double()
        err = float((out.double() - ref).abs().max() / ref.abs().max())
        assert err < 2e-5, err          # fp32 accumulation over K = 2048; tf32 would be ~1e-3
        assert torch.backends.cuda.matmul.allow_tf32 is True
    finally:
        torch.backends.cuda.matmul.allow_tf32 = prev
