"""fp32 torch-CPU restatements of the encoder pieces (TEST INFRASTRUCTURE ONLY).

Functional versions of the build's modules, fed the SAME parameters, used to
check the HIP-backed modules: RMSNorm, residual-add + LayerNorm (timm pre-LN Block), depthwise causal conv1d, the Mamba
mixer (conv -> x_proj/dt_proj -> selective scan -> gate -> out_proj; the
reference's analogue is SS2D.forward, model.py:630-647, with the 1-D Mamba
layout of mamba_ssm's Mamba), patch im2col (Conv2d k = s = P, model.py:189-191).
The reference's own encoders are open_clip / HF towers unavailable offline:
"parity unpinned" beyond these restatements.
"""
import torch
import torch.nn.functional as F

from .scan_ref import selective_scan_ref


def rmsnorm_ref(x, res, w, eps=1e-5):
    h = x.double() + (res.double() if res is not None else 0)
    y = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps) * w.double()
    return y, h


def add_layernorm_ref(x, res, w, b, eps=1e-6, h_dtype=None):
    """(LayerNorm(x + res), x + res) in fp64; h rounded to h_dtype first (the activation-dtype residual add)."""
    h = x.double() + (res.double() if res is not None else 0)
    if h_dtype is not None:
        h = h.to(h_dtype).double()
    mu = h.mean(-1, keepdim=True)
    var = (h - mu).pow(2).mean(-1, keepdim=True)
    y = (h - mu) * torch.rsqrt(var + eps) * w.double() + (b.double() if b is not None else 0)
    return y, h


def causal_conv1d_ref(x, w, b, silu=True):
    D, K = w.shape[0], w.shape[-1]
    y = F.conv1d(x.double(), w.double().reshape(D, 1, K), b.double() if b is not None else None,
                 padding=K - 1, groups=D)[..., : x.shape[-1]]
    return F.silu(y) if silu else y


def mamba_mixer_ref(m, hidden):
    """mixer math in fp64 with the module's parameters (m: MambaMixer), on hidden's device (the same
    torch code on the host or, for full-size checks, evaluated on the GPU in fp64)."""
    p = {k: v.detach().to(hidden.device, torch.float64) for k, v in m.state_dict().items()}
    h = hidden.double()
    xz = torch.einsum("ed,bld->bel", p["in_proj.weight"], h)
    x, z = xz[:, : m.d_inner], xz[:, m.d_inner:]
    x = causal_conv1d_ref(x, p["conv1d.weight"], p["conv1d.bias"], True)
    x_dbl = torch.einsum("cd,bdl->bcl", p["x_proj.weight"], x)
    dt_raw, Bm, Cm = torch.split(x_dbl, [m.dt_rank, m.d_state, m.d_state], dim=1)
    delta = torch.einsum("dr,brl->bdl", p["dt_proj.weight"], dt_raw)
    y = selective_scan_ref(x, delta, -torch.exp(p["A_log"]), Bm, Cm, p["D"], z=z, delta_bias=p["dt_proj.bias"],
                           delta_softplus=True, compute_dtype=torch.float64)
    return torch.einsum("md,bdl->blm", p["out_proj.weight"], y)


def im2col_ref(img, P):
    B, C, H, W = img.shape
    cols = F.unfold(img, P, stride=P)            # (B, C*P*P, L)
    return cols.transpose(1, 2).reshape(B * (H // P) * (W // P), C * P * P)
