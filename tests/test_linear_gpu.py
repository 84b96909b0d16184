"""mc_linear (csrc/gemm_wgrad.hip): the towers' Linear forward / input-gradient GEMM with fused
epilogues (reference: the ViT Linears and timm Mlp -- fc1 -> nn.GELU() exact erf -> fc2 -- behind
model.py:1011-1017), and ops.MlpFn built on it.

Tolerances: the GEMM accumulates in fp32 and rounds once to the 16-bit dtype, so against an fp64
product of the same operands |err| <= 1e-5 * sum_k |x w| + half an ulp of the result (2^-8 relative
for bf16, 2^-11 for f16), plus the bias's own rounding.  GELU / GELU' are evaluated in fp32 on the
ROUNDED h / ga as torch's F.gelu / gelu_backward on the stored tensors, in torch's form
0.5 (1 + erf(x / sqrt2)) -- with erf from an erfc fit (fractional error 1.2e-7) instead of the library
erff.  Checked against torch applied to OUR rounded h / ga: within one ulp of the output dtype plus
the fp32 granularity of erf near +-1 (torch's own cancellation in 1 + erf for x << 0: 2^-23 |x|
absolute), and bitwise equal on > 99 % of the elements."""
import pytest
import torch

from mamba_clip_amd import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
ULP = {torch.bfloat16: 2.0 ** -7, torch.float16: 2.0 ** -10}


def _rand(shape, dt, g, scale=1.0):
    return ((torch.rand(*shape, device=DEV, generator=g) * 2 - 1) * scale).to(dt)


def _gemm_check(y, x, w, b=None):
    ref = x.double() @ w.double().t()
    mag = x.double().abs() @ w.double().abs().t()
    if b is not None:
        ref = ref + b.double()
        mag = mag + b.double().abs()
    bound = mag * 1e-5 + ref.abs() * ULP[y.dtype] / 2 + 1e-6
    err = (y.double() - ref).abs()
    assert bool((err <= bound).all()), f"max err {float(err.max()):.3e} ratio {float((err / bound).max()):.2f}"


def _ulp_close(a, b, dt, x):
    err = (a.double() - b.double()).abs()
    bound = b.double().abs() * ULP[dt] + 2.0 ** -22 * x.double().abs() + (1e-6 if dt == torch.float16 else 1e-30)
    frac_exact = float((a == b).float().mean())
    assert bool((err <= bound).all()), f"max err {float(err.max()):.3e} ratio {float((err / bound).max()):.2f}"
    return frac_exact


SHAPES = [
    # rows (tokens), cols (out features), K
    (4096, 768, 768),      # ViT proj
    (1576, 3072, 768),     # ViT fc1 at batch 8 (ragged token tile: 1576 = 6 x 256 + 40)
    (1000, 768, 3072),     # ViT fc2 (ragged)
    (512, 2304, 768),      # ViT qkv
    (300, 264, 128),       # ragged features (% 8 only) and a short K
]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("rows,cols,K", SHAPES)
def test_linear_none_and_bias(rows, cols, K, dt):
    g = torch.Generator(device=DEV).manual_seed(rows + cols + K)
    x, w, b = _rand((rows, K), dt, g), _rand((cols, K), dt, g, 0.05), _rand((cols,), dt, g)
    assert ops.linear_hip_ok(x, w)
    y = ops.linear_hip(x, w)
    assert y.dtype == dt and y.shape == (rows, cols)
    _gemm_check(y, x, w)
    yb = ops.linear_hip(x, w, b)
    _gemm_check(yb, x, w, b)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("rows,cols,K", SHAPES[:3])
def test_linear_bias_gelu(rows, cols, K, dt):
    g = torch.Generator(device=DEV).manual_seed(7 + rows)
    x, w, b = _rand((rows, K), dt, g), _rand((cols, K), dt, g, 0.08), _rand((cols,), dt, g)
    h, a = ops.linear_hip(x, w, b, _lib.MC_LINEAR_EPI_BIAS_GELU)
    _gemm_check(h, x, w, b)
    ref_a = torch.nn.functional.gelu(h.float()).to(dt)       # torch's GELU of the stored h
    frac = _ulp_close(a, ref_a, dt, h)
    assert frac > 0.99, f"only {frac:.4f} of gelu(h) bitwise equal to torch's"


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("rows,cols,K", [(1576, 3072, 768), (1000, 768, 3072), (300, 264, 128)])
def test_linear_gelu_grad_and_colsum(rows, cols, K, dt):
    g = torch.Generator(device=DEV).manual_seed(11 + cols)
    gy, wt, h = _rand((rows, K), dt, g), _rand((cols, K), dt, g, 0.05), _rand((rows, cols), dt, g, 3.0)
    gh, cs = ops.linear_hip(gy, wt, None, _lib.MC_LINEAR_EPI_GELU_GRAD, h=h, want_colsum=True)
    ga = ops.linear_hip(gy, wt)                                # the stored fc2 input gradient, same rounding
    _gemm_check(ga, gy, wt)
    ref = torch.ops.aten.gelu_backward(ga.float(), h.float()).to(dt)
    frac = _ulp_close(gh, ref, dt, h * ga)
    assert frac > 0.99, f"only {frac:.4f} of gh bitwise equal to torch's gelu_backward"
    ref_cs = gh.double().sum(0)
    err = (cs.double() - ref_cs).abs()
    bound = gh.double().abs().sum(0) * 1e-6 + 1e-6
    assert bool((err <= bound).all()), f"colsum max err {float(err.max()):.3e}"
    # no colsum requested: same gh, bitwise
    gh2, none = ops.linear_hip(gy, wt, None, _lib.MC_LINEAR_EPI_GELU_GRAD, h=h)
    assert none is None and torch.equal(gh, gh2)


def test_linear_deterministic_and_strided():
    g = torch.Generator(device=DEV).manual_seed(3)
    dt = torch.bfloat16
    xb = _rand((2048, 1024), dt, g)
    x = xb[:, :768]                                           # row stride 1024
    w, b = _rand((768, 768), dt, g, 0.05), _rand((768,), dt, g)
    y1 = ops.linear_hip(x, w, b)
    y2 = ops.linear_hip(x.contiguous(), w, b)
    assert torch.equal(y1, y2)
    _gemm_check(y1, x, w, b)


def test_linear_rejects_bad_shapes():
    lib = _lib.load()
    p = _lib.LinearParams()
    x = torch.zeros(64, 96, device=DEV, dtype=torch.bfloat16)   # K = 96: not % 64
    w = torch.zeros(64, 96, device=DEV, dtype=torch.bfloat16)
    y = torch.zeros(64, 64, device=DEV, dtype=torch.bfloat16)
    p.rows, p.cols, p.K, p.dtype, p.epilogue = 64, 64, 96, _lib.dtype_code(x.dtype), 0
    p.X, p.ldx, p.W, p.ldw, p.Y, p.ldy = x.data_ptr(), 96, w.data_ptr(), 96, y.data_ptr(), 64
    assert lib.mc_linear(p, None) != 0
    p.K, p.epilogue = 64, _lib.MC_LINEAR_EPI_BIAS              # bias epilogue without a bias
    assert lib.mc_linear(p, None) != 0
    assert not ops.linear_hip_ok(x, w)


@pytest.fixture
def mlp_all_hip(monkeypatch):
    for flag in ("MLP_HIP_FC1", "MLP_HIP_FC2", "MLP_HIP_BWD"):
        monkeypatch.setattr(ops, flag, True)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_mlp_fn_matches_unfused_chain(dt, mlp_all_hip):
    """MlpFn (mc_linear forward / backward epilogues) vs the unfused chain fc1_gelu + linear_sk (library
    GEMMs + mc_gelu_bwd), same weights and output gradient, under autocast as the towers run."""
    torch.manual_seed(0)
    fc1, fc2 = torch.nn.Linear(768, 3072).to(DEV), torch.nn.Linear(3072, 768).to(DEV)
    x0 = torch.randn(8, 197, 768, device=DEV)
    gy = torch.randn(8, 197, 768, device=DEV).to(dt)
    outs = []
    for fused in (True, False):
        for p in (*fc1.parameters(), *fc2.parameters()):
            p.grad = None
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=dt):
            if fused:
                assert ops.mlp_hip_ok(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias)
                y = ops.MlpFn.apply(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias)
            else:
                y = ops.linear_sk(ops.fc1_gelu(x, fc1.weight, fc1.bias), fc2.weight, fc2.bias)
        y.backward(gy)
        outs.append([y.detach().float(), x.grad.float()] + [p.grad.float() for p in (*fc1.parameters(), *fc2.parameters())])
    names = ["y", "dx", "dw1", "db1", "dw2", "db2"]
    for n, a, b in zip(names, *outs):
        rel = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        assert rel < (2e-2 if dt == torch.bfloat16 else 4e-3), f"{n}: max rel diff {rel:.3e}"


def test_mlp_fn_bitwise_repeatable(mlp_all_hip):
    torch.manual_seed(1)
    fc1, fc2 = torch.nn.Linear(768, 3072).to(DEV), torch.nn.Linear(3072, 768).to(DEV)
    x0 = torch.randn(4, 197, 768, device=DEV)
    gy = torch.randn(4, 197, 768, device=DEV).bfloat16()
    runs = []
    for _ in range(2):
        for p in (*fc1.parameters(), *fc2.parameters()):
            p.grad = None
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = ops.MlpFn.apply(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias)
        y.backward(gy)
        runs.append([y.detach(), x.grad] + [p.grad.clone() for p in (*fc1.parameters(), *fc2.parameters())])
    assert all(torch.equal(a, b) for a, b in zip(*runs))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,K,T", [(1536, 48, 20480), (1536, 48, 640), (3072, 64, 2056), (100, 16, 256), (48, 32, 8)])
def test_gemm_small_k(M, K, T, dt):
    """mc_gemm_small_k (the mixer's dt_proj forward) vs an fp64 product of the same operands; X a row view
    of a wider buffer (the x_dbl slab's dt rows), ragged M and T."""
    g = torch.Generator(device=DEV).manual_seed(M + K + T)
    w = _rand((M, K), dt, g, 0.2)
    xb = _rand((K + 32, T), dt, g)
    x = xb[:K]                                                 # dt rows of a (R + 2N, T) slab
    assert ops.small_k_ok(w, x)
    y = ops.gemm_small_k(w, x)
    ref = w.double() @ x.double()
    bound = (w.double().abs() @ x.double().abs()) * 1e-5 + ref.abs() * ULP[dt] / 2 + 1e-6
    err = (y.double() - ref).abs()
    assert bool((err <= bound).all()), f"max err {float(err.max()):.3e}"
    assert torch.equal(y, ops.gemm_small_k(w, x))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,K,T", [(80, 1536, 20480), (80, 1536, 640), (96, 3072, 2056), (20, 256, 8), (17, 512, 136)])
def test_gemm_skinny_m(M, K, T, dt, monkeypatch):
    """mc_gemm_skinny_m (the mixer's x_proj forward; off by default) vs an fp64 product of the same
    operands; X a row view of a wider buffer, ragged M and T; bitwise repeatable (fixed-order sum of the
    waves' K quarters)."""
    monkeypatch.setattr(ops, "SKINNY_M_HIP", True)
    g = torch.Generator(device=DEV).manual_seed(M + K + T)
    w = _rand((M, K), dt, g, 0.05)
    xb = _rand((K, T + 24), dt, g)
    x = xb[:, :T]                                              # row stride T + 24
    assert ops.skinny_m_ok(w, x)
    y = ops.gemm_skinny_m(w, x)
    ref = w.double() @ x.double()
    bound = (w.double().abs() @ x.double().abs()) * 1e-5 + ref.abs() * ULP[dt] / 2 + 1e-6
    err = (y.double() - ref).abs()
    assert bool((err <= bound).all()), f"max err {float(err.max()):.3e}"
    assert torch.equal(y, ops.gemm_skinny_m(w, x))
