"""mc_gemm_wgrad (csrc/gemm_wgrad.hip): the towers' long-reduction weight-gradient GEMM, dW = G^T X
(reference: the towers' Linear layers behind model.py:1011-1017), against an fp64 product of the same
16-bit operands, for every operand layout the towers produce (token-major rows of a Linear,
channel-major Mamba activations), ragged feature counts, split counts, and run-to-run bitwise
determinism.  Tolerance: fp32 accumulation of T products -> |err| <= 1e-5 * sum_t |a b| + 1e-6."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _operands(N, K, T, dt, a_fm, b_fm, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    # G (N, T): token-major = a (T, N) row-major buffer viewed transposed; feature-major = (N, T) rows
    Gb = torch.randn(N, T, device=DEV, generator=g).to(dt) if a_fm else \
        torch.randn(T, N, device=DEV, generator=g).to(dt).t()
    Xb = torch.randn(K, T, device=DEV, generator=g).to(dt).t() if b_fm else \
        torch.randn(T, K, device=DEV, generator=g).to(dt)
    return Gb, Xb


def _check(out, G, X):
    ref = G.double() @ X.double()
    bound = (G.double().abs() @ X.double().abs()) * 1e-5 + 1e-6
    err = (out.double() - ref).abs()
    assert bool((err <= bound).all()), f"max err {float(err.max()):.3e}, max bound ratio {float((err / bound).max()):.2f}"


CASES = [
    # N, K, T, a_fm, b_fm -- ViT shapes (token-major both), Mamba (channel-major both, and out_proj mixed)
    (768, 768, 4096, False, False),
    (2304, 768, 2048, False, False),
    (768, 3072, 1024, False, False),
    (3072, 768, 20480 // 8, True, True),
    (768, 1536, 2560, False, True),
    (80, 1536, 1280, True, True),       # x_proj: ragged M (one partial tile)
    (1536, 48, 1280, True, True),       # dt_proj: ragged N
    (264, 40, 512, False, False),       # ragged token-major feature counts (% 8 only)
]


@pytest.mark.parametrize("pipe", ["5", "4", "2"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"N{c[0]}K{c[1]}T{c[2]}{'F' if c[3] else 'T'}{'F' if c[4] else 'T'}")
def test_wgrad_matches_fp64(case, dt, pipe, monkeypatch):
    """Every main-loop variant (MC_WGRAD_PIPE: 5 staggered four-phase, 4 four-phase, 2 two-barrier)."""
    from mamba_clip_amd.ops import wgrad_hip
    monkeypatch.setenv("MC_WGRAD_PIPE", pipe)
    N, K, T, a_fm, b_fm = case
    G, X = _operands(N, K, T, dt, a_fm, b_fm, seed=N + K)
    out = wgrad_hip(G, X)
    assert out is not None and out.shape == (N, K) and out.dtype == torch.float32
    _check(out, G, X)


@pytest.mark.parametrize("splits", [1, 2, 5, 16])
def test_wgrad_split_counts_and_determinism(splits):
    from mamba_clip_amd.ops import wgrad_hip
    G, X = _operands(512, 768, 64 * 40, torch.bfloat16, False, False, seed=3)
    a = wgrad_hip(G, X, splits=splits)
    b = wgrad_hip(G, X, splits=splits)
    _check(a, G, X)
    assert torch.equal(a, b)


def test_wgrad_rejects_unsupported_and_falls_back():
    from mamba_clip_amd import ops
    G, X = _operands(256, 256, 100, torch.bfloat16, False, False)     # T % 64 != 0
    assert ops.wgrad_hip(G, X) is None
    G32, X32 = G.float(), X.float()
    assert ops.wgrad_hip(G32, X32) is None
    # the dispatcher falls back to the library path (a short reduction: one bf16-output GEMM)
    torch.testing.assert_close(ops.wgrad(G, X), (G.float() @ X.float()), rtol=1e-2, atol=1e-2)


def test_wgrad_c2_shape_and_linear_backward():
    """ViT fc1 weight gradient at the C2 token count (50,432 = 256 x 197) vs fp64, and LinearSK's
    backward with the HIP wgrad on equal to the library slabs within fp32 rounding."""
    from mamba_clip_amd import ops
    G, X = _operands(3072, 768, 50432, torch.bfloat16, False, False, seed=11)
    out = ops.wgrad_hip(G, X)
    _check(out, G, X)
    x = torch.randn(64, 197, 768, device=DEV, dtype=torch.bfloat16, requires_grad=True)   # 12,608 tokens (C3)
    w = torch.randn(3072, 768, device=DEV, requires_grad=True)
    gy = torch.randn(64, 197, 3072, device=DEV, dtype=torch.bfloat16)
    grads = {}
    prev = ops.WGRAD_HIP
    for on in (False, True):
        ops.WGRAD_HIP = on
        try:
            w.grad = None
            ops.linear_sk(x, w).backward(gy)
            grads[on] = w.grad.clone()
        finally:
            ops.WGRAD_HIP = prev
    ref = gy.reshape(-1, 3072).double().t() @ x.detach().reshape(-1, 768).double()
    for on in (False, True):
        assert float((grads[on].double() - ref).abs().max()) <= 1e-5 * float(ref.abs().max()) * 50
