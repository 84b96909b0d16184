"""Pin the CPU oracle against the golden vectors generated from the reference
(tests/golden/make_golden.py).  CPU only."""
import glob
import os

import pytest
import torch

from conftest import GOLDEN, golden_meta, load_golden
from oracle.scan_ref import selective_scan_ref, selective_scan_ref_grads
from oracle.loss_ref import clip_loss

SCAN_FILES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "scan_*.safetensors")))


def _scan_inputs(g):
    return {k[3:]: v for k, v in g.items() if k.startswith("in.")}


@pytest.mark.parametrize("fname", SCAN_FILES)
def test_scan_oracle_forward_matches_reference_text(fname):
    g = load_golden(fname)
    meta = golden_meta(fname)
    sp = meta["softplus"] == "1"
    last = meta["last"] == "1"
    x = _scan_inputs(g)
    res = selective_scan_ref(**x, delta_softplus=sp, return_last_state=last)
    out, ls = (res if last else (res, None))
    assert out.dtype == g["out"].dtype and out.shape == g["out"].shape
    # fp32 restatement vs fp32 reference text: same math, different summation order
    torch.testing.assert_close(out.float(), g["out"].float(), rtol=1e-5, atol=1e-5) if out.dtype == torch.float32 \
        else torch.testing.assert_close(out.float(), g["out"].float(), rtol=1e-2, atol=1e-2)
    if last:
        torch.testing.assert_close(ls, g["last_state"], rtol=1e-5, atol=1e-5)
    # fp64 oracle against the fp32 reference output (pre-cast)
    out64 = selective_scan_ref(**{k: (v.double() if v.is_floating_point() else v) for k, v in x.items()},
                               delta_softplus=sp, compute_dtype=torch.float64)
    scale = float(g["out_f32"].abs().max().clamp_min(1.0))
    torch.testing.assert_close(out64.float(), g["out_f32"], rtol=1e-4, atol=1e-4 * scale)


@pytest.mark.parametrize("fname", SCAN_FILES)
def test_scan_oracle_backward_matches_reference_text(fname):
    g = load_golden(fname)
    sp = golden_meta(fname)["softplus"] == "1"
    x = {k: v.float() for k, v in _scan_inputs(g).items()}
    grads = selective_scan_ref_grads(**x, delta_softplus=sp, dout=g["dout"])
    for k, v in grads.items():
        ref = g[f"grad.{k}"]
        scale = ref.abs().max().clamp_min(1.0)
        assert torch.allclose(v.float(), ref, rtol=1e-3, atol=1e-4 * float(scale)), k


def test_scan_oracle_rejects_off_path_shapes():
    u = torch.randn(1, 4, 3)
    with pytest.raises(NotImplementedError):
        selective_scan_ref(u, u, torch.randn(4, 2), torch.randn(4, 2), torch.randn(4, 2))


@pytest.mark.parametrize("fname", ["clip_loss_single_n8_e16.safetensors", "clip_loss_single_n64_e32.safetensors"])
def test_loss_oracle_single_process(fname):
    g = load_golden(fname)
    img = g["img"].clone().requires_grad_(True)
    txt = g["txt"].clone().requires_grad_(True)
    s = g["scale"][0].clone().requires_grad_(True)
    loss = clip_loss(img, txt, s)
    loss.backward()
    torch.testing.assert_close(loss.detach().reshape(1), g["loss"], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(img.grad, g["grad_img"], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(txt.grad, g["grad_txt"], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(s.grad.reshape(1), g["grad_scale"], rtol=1e-5, atol=1e-7)


def test_quant_rows_fp8_ref_properties():
    """fp8 oracle (config 5): padding, zero rows, scale and the e4m3 round-trip bound."""
    from oracle.loss_ref import quant_rows_fp8_ref, similarity_fp8_ref
    g = torch.Generator().manual_seed(0)
    X = torch.randn(9, 40, generator=g) * 5
    X[3] = 0
    q, inv = quant_rows_fp8_ref(X)
    assert q.shape == (9, 48) and q.dtype == torch.uint8
    assert (q[:, 40:] == 0).all() and (q[3] == 0).all() and inv[3] == 1.0
    deq = q[:, :40].view(torch.float8_e4m3fn).float() * inv[:, None]
    assert ((deq - X).abs() <= X.abs() * 2 ** -4 + inv[:, None] * 2 ** -9).all()
    # every nonzero row uses the full range: its largest element maps to 448 exactly
    full = q[:, :40].view(torch.float8_e4m3fn).float().abs().amax(dim=1)
    assert torch.equal(full[torch.arange(9) != 3], torch.full((8,), 448.0))
    S = similarity_fp8_ref(X, X, 1.0)
    assert torch.allclose(S, S.T)
