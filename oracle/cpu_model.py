"""CPU restatement of the stage-1 training step (TEST / BASELINE INFRASTRUCTURE ONLY).

Used by bench.py's `cpu_baseline` leg and by tests: the SAME module classes
as the product (mamba_clip_amd.model), with their HIP entry points
swapped for the fp32 CPU restatements of this directory while the context is
active, and the loss computed by oracle/loss_ref.clip_loss (loss.py:89-147).
This is the "reference's CPU path" of SURVEY.md 8(d): fp32 PyTorch-CPU eager,
scan by the model.py:83-169 semantics.  The product path never imports this.
"""
import time
from contextlib import contextmanager

import torch
import torch.nn.functional as F

from .loss_ref import clip_loss
from .scan_ref import selective_scan_ref


def _add_rmsnorm_f32(x, res, w, eps=1e-5):
    h = x.float() + (res.float() if res is not None else 0)
    y = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype), h


def _causal_conv1d_f32(x, w, b=None, silu=True, dx_slab=None):
    D, K = w.shape[0], w.shape[-1]
    y = F.conv1d(x, w.reshape(D, 1, K).to(x.dtype), b.to(x.dtype) if b is not None else None,
                 padding=K - 1, groups=D)[..., : x.shape[-1]]
    return F.silu(y) if silu else y


def _add_layernorm_f32(x, res, w, b, eps=1e-6):
    h = x if res is None else (x + res.to(x.dtype))
    y = F.layer_norm(h.float(), (h.shape[-1],), w.float(), b.float() if b is not None else None, eps)
    return y.to(x.dtype), h


IMAGE_MEAN = (0.48145466, 0.4578275, 0.40821073)   # open_clip OPENAI_DATASET_MEAN / _STD (data.py:47-53)
IMAGE_STD = (0.26862954, 0.26130258, 0.27577711)


def to_tensor_normalize(img_u8, mean=IMAGE_MEAN, std=IMAGE_STD):
    """The reference's ToTensor + Normalize (data.py:102-106) on a (B, H, W, C) uint8 batch -> NCHW fp32."""
    C = img_u8.shape[-1]
    x = img_u8.permute(0, 3, 1, 2).double() / 255.0
    m = torch.tensor(mean[:C], dtype=torch.float64).view(1, C, 1, 1)
    s = torch.tensor(std[:C], dtype=torch.float64).view(1, C, 1, 1)
    return ((x - m) / s).float()


def _im2col(img, P, out_dtype=None, mean=None, std=None):
    if img.dtype == torch.uint8:
        img = to_tensor_normalize(img, mean or IMAGE_MEAN, std or IMAGE_STD)
    B, C, H, W = img.shape
    cols = F.unfold(img, P, stride=P).transpose(1, 2).reshape(B * (H // P) * (W // P), C * P * P)
    return cols.to(out_dtype) if out_dtype is not None else cols


def grouped_scan_ref(u, delta, A, B, C, D=None, delta_bias=None, delta_softplus=False, reverse_groups=0,
                     u_groups=1):
    """Restatement of the grouped-direction scan with EXPLICIT copies, the way the reference builds
    SS2D's cross-scan (model.py:510-517: stack, flip) and merges it (553-565: flip back): group g
    scans u block g % u_groups, flipped along L when bit g of reverse_groups is set, and its output
    is flipped back."""
    Bsz, dim, L = delta.shape
    G = B.shape[1]
    d = dim // G
    ub = u.view(Bsz, u_groups, d, L)
    rev = [bool((reverse_groups >> g) & 1) for g in range(G)]
    fl = lambda t, g: t.flip(-1) if rev[g] else t  # noqa: E731
    xs = torch.stack([fl(ub[:, g % u_groups], g) for g in range(G)], 1).reshape(Bsz, dim, L)
    dl = torch.stack([fl(delta.view(Bsz, G, d, L)[:, g], g) for g in range(G)], 1).reshape(Bsz, dim, L)
    Bs = torch.stack([fl(B[:, g], g) for g in range(G)], 1)
    Cs = torch.stack([fl(C[:, g], g) for g in range(G)], 1)
    out = selective_scan_ref(xs, dl, A, Bs, Cs, D, delta_bias=delta_bias, delta_softplus=delta_softplus)
    out = out.view(Bsz, G, d, L)
    return torch.stack([fl(out[:, g], g) for g in range(G)], 1).reshape(Bsz, dim, L)


def ss2d_conv_stack_ref(x, weight, bias):
    """SS2D's conv front and cross-scan input the way the reference builds it (model.py:636-637:
    permute + depthwise conv2d + SiLU; 510-517: stack [x, x^T]; 531-537: fp32): (B, 2, C, H*W)."""
    xc = x.permute(0, 3, 1, 2)
    k = weight.shape[-1]
    y = F.silu(F.conv2d(xc, weight.to(x.dtype), bias.to(x.dtype) if bias is not None else None, padding=k // 2,
                        groups=xc.shape[1]))
    Bsz, C, H, W = y.shape
    return torch.stack([y.reshape(Bsz, C, H * W), y.transpose(2, 3).reshape(Bsz, C, H * W)], dim=1).float()


def ss2d_merge_ln_gate_ref(out, z, ln_weight, ln_bias, eps):
    """The reference merge (model.py:553-565: directions 1 / 3 transposed back; 640-643: y1 + y2 + y3 +
    y4, transpose, out_norm, * silu(z)) on the grouped scan's (B, 4C, H*W) output."""
    Bsz, H, W, C = z.shape
    o = out.view(Bsz, 4, C, H * W)
    back = lambda t: t.reshape(Bsz, C, W, H).transpose(2, 3).reshape(Bsz, C, H * W)  # noqa: E731
    y = o[:, 0] + o[:, 2] + back(o[:, 1]) + back(o[:, 3])
    y = y.transpose(1, 2).reshape(Bsz, H, W, C)
    return F.layer_norm(y, (C,), ln_weight, ln_bias, eps) * F.silu(z)


def _mixer_scan(x, delta, A, Bm, Cm, D, z, delta_bias, dz_slab, du_handoff=None, dbc_slab=None):
    return selective_scan_ref(x, delta, A, Bm, Cm, D, z=z, delta_bias=delta_bias, delta_softplus=True)


_OPS = {"selective_scan_fn": selective_scan_ref, "mixer_scan": _mixer_scan, "grouped_scan_fn": grouped_scan_ref, "add_rmsnorm": _add_rmsnorm_f32,
        "causal_conv1d": _causal_conv1d_f32, "patch_im2col": _im2col, "add_layernorm": _add_layernorm_f32,
        "ss2d_conv_stack": ss2d_conv_stack_ref, "ss2d_merge_ln_gate": ss2d_merge_ln_gate_ref}


@contextmanager
def oracle_ops():
    """Temporarily route mamba_clip_amd.model's op references to the CPU restatements."""
    import mamba_clip_amd.model as M
    saved = {k: getattr(M, k) for k in _OPS}
    try:
        for k, f in _OPS.items():
            setattr(M, k, f)
        yield
    finally:
        for k, f in saved.items():
            setattr(M, k, f)


def oracle_clip_loss(image_features, text_features, logit_scale, output_dict=True, target=None, **_):
    loss = clip_loss(image_features, text_features, logit_scale)
    return {"contrastive_loss": loss} if output_dict else loss


def cpu_train_pairs_per_sec(model_name="vit_b16-mamba130m", batch=8, steps=5, warmup=1, threads=None, seed=0):
    """fp32 CPU fwd+bwd+AdamW steps of the same architecture; returns (pairs/s from the MEDIAN step
    time, seconds timed in total) -- the median of `steps` timed steps, as BASELINE.md plans."""
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.model import build_clip
    if threads:
        torch.set_num_threads(threads)
    torch.manual_seed(seed)
    model = build_clip(model_name)
    text = model.text
    images, texts, _ = synthetic_batch(batch, 224 if model_name != "tiny-mamba-clip" else 32,
                                       text.context_length, text.vocab_size, seed=1000)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-5)
    with oracle_ops():
        def step():
            opt.zero_grad(set_to_none=True)
            out = model(images, texts)
            oracle_clip_loss(**out)["contrastive_loss"].backward()
            opt.step()
            with torch.no_grad():
                model.logit_scale.clamp_(0, 4.605170185988092)
        for _ in range(warmup):
            step()
        times = []
        for _ in range(steps):
            t0 = time.perf_counter()
            step()
            times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2] if len(times) % 2 else 0.5 * (times[len(times) // 2 - 1] + times[len(times) // 2])
    return batch / med, sum(times)


def cpu_scan_gbps(batch=1, dim=3072, seqlen=4096, dstate=16, threads=None, seed=0):
    """Oracle selective-scan forward at C4 channel/length shape, bf16 I/O semantics; returns (GB/s, seconds)."""
    if threads:
        torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(seed)
    u = torch.randn(batch, dim, seqlen, generator=g).bfloat16()
    dl = (torch.randn(batch, dim, seqlen, generator=g) * 0.5).bfloat16()
    z = torch.randn(batch, dim, seqlen, generator=g).bfloat16()
    A = -torch.exp(torch.log(torch.arange(1, dstate + 1).float()).repeat(dim, 1))
    B = torch.randn(batch, dstate, seqlen, generator=g).bfloat16()
    C = torch.randn(batch, dstate, seqlen, generator=g).bfloat16()
    Dv = torch.ones(dim)
    bias = torch.full((dim,), -3.0)
    t0 = time.perf_counter()
    with torch.no_grad():
        selective_scan_ref(u, dl, A, B, C, Dv, z=z, delta_bias=bias, delta_softplus=True)
    dt = time.perf_counter() - t0
    nbytes = batch * dim * seqlen * 8 + 2 * batch * dstate * seqlen * 2 + (dim * dstate + 2 * dim) * 4
    return nbytes / dt / 1e9, dt
