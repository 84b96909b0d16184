"""Model-stage-1 / model-stage-2 module API on MI355X.

Mirrors /root/reference/src/mamba_clip/model.py's public surface:
  ClipModel (model.py:998-1112)      forward(image, text) -> {"image_features", "text_features",
                                     "logit_scale" (=exp), ["logit_bias"]}; encode_image/encode_text;
                                     get_logits; lock_text_tower; set_grad_checkpointing
  ClipClassifier (model.py:1115-1205) frozen stage-1 CLIP + MLP head; classify
  SS2D / SS_Conv_SSM / VSSLayer / VSSM (model.py:297-995): the MedMamba
                                     cross-scan vision backbone ("medmamba")
  init_model (model.py:1257-1289)    factory returning (model, preprocess_train, preprocess_val, tokenizer)

Towers the reference obtains from open_clip / HF hub (not available offline,
SURVEY.md 8c) are defined here and random-initialised:
  VisionTransformer  ViT-B/16 (timm vit_base_patch16_224 shape: 12 pre-LN
                     blocks, 768 wide, cls pooling, proj -> embed_dim)
  MambaTextEncoder   Mamba LM text tower (Mamba-130M: 24 x d_model 768,
                     d_inner 1536, d_state 16, RMSNorm, fp32 residual stream)
  BertTextEncoder    PubMedBERT-base shape (12 x 768, ctx 256) for BiomedCLIP
Hot ops run on the HIP library: selective scan, causal conv1d, fused
add+RMSNorm / add+LayerNorm, patch im2col, short-sequence attention
(attention.hip), contrastive loss; dense projections are plain library GEMMs
(hipBLASLt through torch, launched data-parallel: see __init__.py).
"""
import contextlib
import math
import os
from functools import partial

import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.utils.checkpoint

from . import GEMM_GRIDS_DATA_PARALLEL
from .ops import (GradHandoff, GradSlab, _compute_dtype, add_layernorm, add_pos, add_rmsnorm, attn_supported,
                  causal_conv1d, l2_normalize, linear_sk, mixer_proj, mixer_proj_ok, mlp, neg_exp_many,
                  packed_attention, patch_im2col, qkv_proj, split_rows, split_rows_n, ss2d_conv_stack,
                  ss2d_merge_ln_gate, ss2d_proj, ss2d_proj_ok, token_embed, weight_cast_scope, wleft_mm)
from .selective_scan_interface import (SS2D_REVERSE_GROUPS, SS2D_U_GROUPS, ProjectedScanFn, SelectiveScanFn,
                                       fine_state_scope,
                                       grouped_scan_fn, projected_scan_ok, selective_scan_fn)


# ============================================================================ Mamba text tower
def _dt_bias_init(d_inner, dt_min=0.001, dt_max=0.1, dt_init_floor=1e-4):
    """softplus^-1 of dt ~ logU[dt_min, dt_max] (model.py:459-468 semantics)."""
    dt = torch.exp(torch.rand(d_inner) * (math.log(dt_max) - math.log(dt_min)) + math.log(dt_min))
    dt = dt.clamp(min=dt_init_floor)
    return dt + torch.log(-torch.expm1(-dt))


XPROJ_GRAD_SLAB = os.environ.get("MAMBA_CLIP_AMD_XPROJ_GRAD_SLAB", "1") != "0"   # A/B toggle


def mixer_scan(x, delta, A, Bm, Cm, D, z, delta_bias, dz_slab, du_handoff=None, dbc_slab=None):
    """The mixer's scan call (selective_scan_fn semantics, softplus on) with dz written into
    the in_proj gradient slab, dB / dC into the x_proj gradient slab and du handed to x_proj's
    backward (ops.GradHandoff)."""
    return SelectiveScanFn.apply(x, delta, A, Bm, Cm, D, z, delta_bias, True, False, dz_slab, du_handoff, dbc_slab)


class MambaMixer(nn.Module):
    """One Mamba mixer: in_proj -> causal conv1d+SiLU -> x_proj/dt_proj -> selective scan (z-gated) -> out_proj.

    Channel-major activations: every projection is ONE 2-D GEMM on the
    (channels, batch*seqlen) matrix, and the conv / scan see it as a
    (batch, channels, seqlen) view with strides (seqlen, batch*seqlen, 1) --
    unit stride along the sequence, no transposes or copies between the GEMMs
    (the HIP kernels take batch/channel strides and write outputs and
    gradients in the same layout).
    """

    def __init__(self, d_model, d_state=16, d_conv=4, expand=2, dt_rank="auto"):
        super().__init__()
        self.d_model, self.d_state, self.d_conv = d_model, d_state, d_conv
        self.d_inner = int(expand * d_model)
        self.dt_rank = math.ceil(d_model / 16) if dt_rank == "auto" else dt_rank
        self.in_proj = nn.Linear(d_model, 2 * self.d_inner, bias=False)
        self.conv1d = nn.Conv1d(self.d_inner, self.d_inner, d_conv, groups=self.d_inner, padding=d_conv - 1)
        self.x_proj = nn.Linear(self.d_inner, self.dt_rank + 2 * d_state, bias=False)
        self.dt_proj = nn.Linear(self.dt_rank, self.d_inner, bias=True)
        std = self.dt_rank ** -0.5
        nn.init.uniform_(self.dt_proj.weight, -std, std)
        with torch.no_grad():
            self.dt_proj.bias.copy_(_dt_bias_init(self.d_inner))
        A = torch.arange(1, d_state + 1, dtype=torch.float32).repeat(self.d_inner, 1)
        self.A_log = nn.Parameter(torch.log(A))
        self.A_log._no_weight_decay = True
        self.D = nn.Parameter(torch.ones(self.d_inner))
        self.D._no_weight_decay = True
        self.out_proj = nn.Linear(self.d_inner, d_model, bias=False)
        # dt_proj inside the scan (ProjectedScanFn) where the shapes allow.  Off by default: the scan
        # kernels are VALU-bound, so forming delta on their MFMAs costs more than the delta stream it
        # saves (C2 step 88.4 vs 86.5 ms on one box, profiles/r03/c2_ab_fuse_dt_proj.txt)
        self.fuse_dt_proj = os.environ.get("MAMBA_CLIP_AMD_FUSE_DT_PROJ", "0") == "1"   # A/B toggle
        self.du_handoff = True   # scan du -> x_proj's dX epilogue (ops.GradHandoff)
        # x_proj + dt_proj as one HIP pass each way (ops.MixerProjFn); A/B toggle
        self.fuse_proj = os.environ.get("MAMBA_CLIP_AMD_FUSE_MIXER_PROJ", "0") == "1"

    def forward(self, hidden, A=None):  # (B, L, d_model) contiguous; A: -exp(A_log) when the tower formed it
        Bsz, L, dm = hidden.shape
        dt_in = hidden.dtype
        di, R, N = self.d_inner, self.dt_rank, self.d_state
        H = hidden.reshape(Bsz * L, dm)
        # projections: weight-left GEMMs with split-K weight gradients (ops.wleft_mm / linear_sk)
        xz = wleft_mm(self.in_proj.weight, H.t())                             # (2*di, B*L)
        # the conv / scan backward kernels write dx / dz into one (2*di, B*L) slab: the split's
        # gradient is that slab, no concatenation (ops.GradSlab)
        slab = GradSlab(2 * di, Bsz * L, xz.dtype, xz.device) if xz.requires_grad else None
        x, z = split_rows(xz, di, slab)
        x = x.view(di, Bsz, L).transpose(0, 1)                                # (B, di, L) channel-major
        z = z.view(di, Bsz, L).transpose(0, 1)
        x = causal_conv1d(x, self.conv1d.weight, self.conv1d.bias, silu=True, dx_slab=slab)
        x_cm = x.transpose(0, 1).reshape(di, Bsz * L)                          # view
        if A is None:
            A = -torch.exp(self.A_log.float())
        dz = (slab, di) if slab is not None else None
        if self.fuse_dt_proj and projected_scan_ok(x, R, N):
            # dt_proj inside the scan (ProjectedScanFn): x_proj's dt rows come out token-major,
            # (B*L, R), the scan kernel forms delta per chunk on MFMA; B / C stay channel-major
            dt_raw = linear_sk(x_cm.t(), self.x_proj.weight[:R])              # (B*L, R)
            BC = wleft_mm(self.x_proj.weight[R:], x_cm)                       # (2N, B*L)
            Bm = BC[:N].view(N, Bsz, L).transpose(0, 1)
            Cm = BC[N:].view(N, Bsz, L).transpose(0, 1)
            y = ProjectedScanFn.apply(x, dt_raw, self.dt_proj.weight, A, Bm, Cm, self.D.float(), z,
                                      self.dt_proj.bias.float(), True, dz)
        elif self.fuse_proj and mixer_proj_ok(x_cm, R, N):
            # x_proj and dt_proj in one pass over x (and one backward pass over ddelta that also adds
            # the scan's du into dx: ops.GradHandoff)
            hand = GradHandoff() if (self.du_handoff and x.requires_grad) else None
            Brows, Crows, delta = mixer_proj(x_cm, self.x_proj.weight, self.dt_proj.weight, hand)
            Bm = Brows.view(N, Bsz, L).transpose(0, 1)                         # (B, N, L)
            Cm = Crows.view(N, Bsz, L).transpose(0, 1)
            delta = delta.view(di, Bsz, L).transpose(0, 1)
            y = mixer_scan(x, delta, A, Bm, Cm, self.D.float(), z, self.dt_proj.bias.float(), dz, hand)
        else:
            # x's gradient: the scan's du is handed to x_proj's backward, which adds its dX in the
            # GEMM epilogue (ops.GradHandoff) instead of autograd summing the two producers
            hand = GradHandoff() if (self.du_handoff and x.is_cuda and x.requires_grad) else None
            x_dbl = wleft_mm(self.x_proj.weight, x_cm, hand)                   # (R+2N, B*L)
            # dt_proj's backward writes d(dt_raw) and the scan's writes dB / dC straight into one
            # (R+2N, B*L) gradient slab: no transpose copies of dB / dC, no concatenation
            pslab = GradSlab(R + 2 * N, Bsz * L, x_dbl.dtype, x_dbl.device) if (x_dbl.requires_grad and
                                                                                 XPROJ_GRAD_SLAB) else None
            dt_raw, Bm, Cm = split_rows_n(x_dbl, (R, N, N), pslab)
            delta = wleft_mm(self.dt_proj.weight, dt_raw, out_slab=(pslab, 0) if pslab is not None else None)
            delta = delta.view(di, Bsz, L).transpose(0, 1)
            Bm = Bm.view(N, Bsz, L).transpose(0, 1)                           # (B, N, L)
            Cm = Cm.view(N, Bsz, L).transpose(0, 1)
            y = mixer_scan(x, delta, A, Bm, Cm, self.D.float(), z, self.dt_proj.bias.float(), dz, hand,
                           (pslab, R, R + N) if pslab is not None else None)
        y2 = y.transpose(0, 1).reshape(di, Bsz * L)                            # view: y keeps x's layout
        out = linear_sk(y2.t(), self.out_proj.weight)                          # (B*L, d_model)
        return out.view(Bsz, L, dm)


class MambaLayer(nn.Module):
    """Pre-norm block: (hidden, residual) -> add+RMSNorm -> mixer (mamba_ssm Block semantics)."""

    def __init__(self, d_model, d_state=16, eps=1e-5):
        super().__init__()
        self.mixer = MambaMixer(d_model, d_state=d_state)
        self.norm_weight = nn.Parameter(torch.ones(d_model))
        self.eps = eps

    def forward(self, hidden, residual, A=None):
        normed, residual = add_rmsnorm(hidden, residual, self.norm_weight, self.eps)
        return self.mixer(normed, A), residual


class MambaTextEncoder(nn.Module):
    """Mamba LM text tower for CLIP: tokens (B, T) int64 -> (B, output_dim).

    Pools the hidden state at the end-of-text position (the last position, as
    the synthetic tokens put EOT there: SURVEY 8d).  The sequence is padded to
    a multiple of 8 positions after the real tokens (causal: padding never
    reaches earlier positions) so every activation row is 16-B aligned.
    """

    def __init__(self, vocab_size=50280, context_length=77, d_model=768, n_layer=24, d_state=16,
                 output_dim=512):
        super().__init__()
        self.vocab_size, self.context_length, self.d_model = vocab_size, context_length, d_model
        self.output_dim = output_dim
        self.embedding = nn.Embedding(vocab_size, d_model)
        nn.init.normal_(self.embedding.weight, std=0.02)
        self.layers = nn.ModuleList([MambaLayer(d_model, d_state) for _ in range(n_layer)])
        self.norm_f = nn.Parameter(torch.ones(d_model))
        self.proj = nn.Linear(d_model, output_dim, bias=False)
        nn.init.normal_(self.proj.weight, std=d_model ** -0.5)

    def lock_units(self):
        """(embeddings, [layer, ...], final norm) as lists of (name, parameter) for lock_text_tower."""
        return ([("embedding.weight", self.embedding.weight)],
                [list(l.named_parameters(prefix=f"layers.{i}")) for i, l in enumerate(self.layers)],
                [("norm_f", self.norm_f)])

    def forward(self, tokens):
        Bsz, T = tokens.shape
        Lp = (T + 7) // 8 * 8
        if Lp != T:
            tokens = F.pad(tokens, (0, Lp - T))
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else torch.float32
        hidden = self.embedding(tokens).to(dt)
        residual = None
        # every mixer's A = -exp(A_log) in one launch (ops.NegExpManyFn)
        As = (neg_exp_many([l.mixer.A_log for l in self.layers]) if hidden.is_cuda
              else [None] * len(self.layers))
        ckpt = self.grad_checkpointing and torch.is_grad_enabled()
        n = len(self.layers)

        def run(layer, hidden, residual, A):
            # each layer's scan may keep fine saved states within budget / n_layer (a static choice: the
            # same in the checkpoint recompute, which runs on the autograd thread)
            with fine_state_scope(n):
                return layer(hidden, residual, A)
        for layer, A in zip(self.layers, As):
            if ckpt:   # recompute the layer in backward instead of keeping its activations
                hidden, residual = torch.utils.checkpoint.checkpoint(run, layer, hidden, residual, A, use_reentrant=False)
            else:
                hidden, residual = run(layer, hidden, residual, A)
        normed, _ = add_rmsnorm(hidden, residual, self.norm_f)
        pooled = normed[:, T - 1]                                   # EOT position
        return self.proj(pooled)

    grad_checkpointing = False

    def set_grad_checkpointing(self, enable=True):
        """Activation checkpointing per Mamba layer (torch.utils.checkpoint, non-reentrant): the reference's
        ClipModel.set_grad_checkpointing (model.py:1099-1102) turns it on in open_clip's towers."""
        self.grad_checkpointing = bool(enable)


def _run_blocks(blocks, m, h, ckpt):
    for blk in blocks:
        m, h = torch.utils.checkpoint.checkpoint(blk, m, h, use_reentrant=False) if ckpt else blk(m, h)
    return m, h


# ============================================================================ ViT-B/16 visual tower
class PatchEmbed(nn.Module):
    """Conv2d(k = s = patch) as im2col (HIP) + one GEMM."""

    def __init__(self, img_size=224, patch=16, in_chans=3, dim=768, bias=True):
        super().__init__()
        self.patch, self.grid = patch, img_size // patch
        self.proj = nn.Conv2d(in_chans, dim, patch, patch, bias=bias)

    def forward(self, x):  # (B, C, H, W) float, or (B, H, W, C) uint8 raw images -> (B, H/P * W/P, dim)
        Bsz = x.shape[0]
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else (
            torch.float32 if x.dtype == torch.uint8 else x.dtype)
        # the input cast (and for raw images ToTensor + Normalize) happens inside the patch kernel
        cols = patch_im2col(x, self.patch, dt)
        w = self.proj.weight.reshape(self.proj.weight.shape[0], -1)
        if cols.is_cuda:   # split-K weight gradient (ops.wgrad): 188 -> 85 us at C2
            out = linear_sk(cols, w, self.proj.bias)
        else:
            out = F.linear(cols, w.to(dt), self.proj.bias.to(dt) if self.proj.bias is not None else None)
        return out.reshape(Bsz, -1, w.shape[0])


def _gpu_sdpa_backends():
    """Backend priority for the towers' attention on MI355X: the memory-efficient
    kernel first (measured at C2, 197 tokens x 12 heads x 64: attention block
    fwd+bwd 2.36 ms vs 2.51 ms for the default choice), then flash, then math."""
    from torch.nn.attention import SDPBackend, sdpa_kernel
    order = [SDPBackend.EFFICIENT_ATTENTION, SDPBackend.FLASH_ATTENTION, SDPBackend.MATH]
    try:
        return sdpa_kernel(order, set_priority=True)
    except TypeError:  # older torch: no priority argument
        return sdpa_kernel(order)


class Attention(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.heads = heads
        self.qkv = nn.Linear(dim, 3 * dim, bias=True)
        self.proj = nn.Linear(dim, dim)
        self.fused_attention = True   # mc_attn_fwd/bwd where supported (bf16/f16, head_dim 64, N <= 256)

    def forward(self, x):
        Bsz, N, C = x.shape
        if self.fused_attention and x.is_cuda and attn_supported(N, C // self.heads, _compute_dtype(x)):
            # packed qkv projection -> fused attention kernel (ops.PackedAttentionFn: the whole
            # sequence of a head in LDS) -> output projection; o is already (B, N, C) and the
            # backward writes dq / dk / dv into the packed projection gradient
            qkv = linear_sk(x, self.qkv.weight, self.qkv.bias)
            return linear_sk(packed_attention(qkv, self.heads), self.proj.weight, self.proj.bias)
        # unbind (not index) the q/k/v slices: its backward stacks the three
        # gradients in one write instead of zero-filling and accumulating a
        # (3, B, H, N, D) buffer three times and copying it contiguous again
        # q, k, v: (B, H, N, D) views of the packed qkv output; the backward packs dq / dk / dv and
        # the qkv bias gradient in one pass (ops.QKVProjFn)
        q, k, v = qkv_proj(x, self.qkv.weight, self.qkv.bias, self.heads)
        if x.is_cuda:
            with _gpu_sdpa_backends():
                o = F.scaled_dot_product_attention(q, k, v)
        else:
            o = F.scaled_dot_product_attention(q, k, v)
        return linear_sk(o.transpose(1, 2).reshape(Bsz, N, C), self.proj.weight, self.proj.bias)


class ViTBlock(nn.Module):
    """Pre-LN transformer block (timm Block parameters: norm1, attn, norm2, fc1/fc2 MLP).

    forward(m, h) takes the previous block's branch output m and residual
    stream h (x = h + m) and returns its own (m', h'): each residual add is
    fused into the following LayerNorm (mc_add_layernorm), the way the Mamba
    blocks fuse add + RMSNorm.  Same math as x = x + attn(norm1(x));
    x = x + mlp(norm2(x)).
    """

    def __init__(self, dim, heads, mlp_ratio=4.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, heads)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.fc1 = nn.Linear(dim, int(dim * mlp_ratio))
        self.fc2 = nn.Linear(int(dim * mlp_ratio), dim)

    def forward(self, m, h=None):
        y, h = add_layernorm(m, h, self.norm1.weight, self.norm1.bias, self.norm1.eps)
        a = self.attn(y)
        y, h = add_layernorm(a, h, self.norm2.weight, self.norm2.bias, self.norm2.eps)
        return mlp(y, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias), h


class VisionTransformer(nn.Module):
    """ViT-B/16 image tower: (B, 3, 224, 224) -> (B, output_dim)."""

    def __init__(self, img_size=224, patch=16, width=768, layers=12, heads=12, output_dim=512):
        super().__init__()
        self.output_dim = output_dim
        self.patch_embed = PatchEmbed(img_size, patch, 3, width)
        n = (img_size // patch) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, width))
        self.pos_embed = nn.Parameter(torch.randn(1, n + 1, width) * 0.02)
        self.blocks = nn.ModuleList([ViTBlock(width, heads) for _ in range(layers)])
        self.norm = nn.LayerNorm(width, eps=1e-6)
        self.head = nn.Linear(width, output_dim, bias=False)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.patch_embed(x)
        # cat([cls, x]) + pos with a deterministic backward (ops.TokenEmbedFn)
        m, h = token_embed(self.cls_token, x, self.pos_embed), None
        m, h = _run_blocks(self.blocks, m, h, self.grad_checkpointing and torch.is_grad_enabled())
        # final norm on the pooled (cls) rows only: same values as norm(x)[:, 0]
        y, _ = add_layernorm(m[:, 0], h[:, 0], self.norm.weight, self.norm.bias, self.norm.eps)
        return self.head(y)

    def lock(self, unlocked_groups=0, freeze_bn_stats=False):
        for p in self.parameters():
            p.requires_grad = False

    grad_checkpointing = False

    def set_grad_checkpointing(self, enable=True):
        """Activation checkpointing per transformer block (timm / open_clip semantics)."""
        self.grad_checkpointing = bool(enable)


# ============================================================================ BERT text tower (BiomedCLIP shape)
class BertTextEncoder(nn.Module):
    """PubMedBERT-base-shaped encoder (12 x 768, ctx 256), CLS pooling + MLP projection."""

    def __init__(self, vocab_size=30522, context_length=256, width=768, layers=12, heads=12, output_dim=512):
        super().__init__()
        self.vocab_size, self.context_length, self.output_dim = vocab_size, context_length, output_dim
        self.tok = nn.Embedding(vocab_size, width)
        self.pos = nn.Parameter(torch.randn(1, context_length, width) * 0.02)
        self.ln = nn.LayerNorm(width, eps=1e-12)
        self.blocks = nn.ModuleList([ViTBlock(width, heads) for _ in range(layers)])
        self.proj = nn.Sequential(nn.Linear(width, (width + output_dim) // 2, bias=False), nn.GELU(),
                                  nn.Linear((width + output_dim) // 2, output_dim, bias=False))

    def lock_units(self):
        """(embeddings incl. their LayerNorm, [block, ...], nothing after) for lock_text_tower."""
        return ([("tok.weight", self.tok.weight), ("pos", self.pos), ("ln.weight", self.ln.weight),
                 ("ln.bias", self.ln.bias)],
                [list(b.named_parameters(prefix=f"blocks.{i}")) for i, b in enumerate(self.blocks)], [])

    grad_checkpointing = False

    def set_grad_checkpointing(self, enable=True):
        """Activation checkpointing per encoder layer (HF gradient_checkpointing semantics)."""
        self.grad_checkpointing = bool(enable)

    def forward(self, tokens):
        m, h = self.ln(add_pos(self.tok(tokens), self.pos)), None
        m, h = _run_blocks(self.blocks, m, h, self.grad_checkpointing and torch.is_grad_enabled())
        return self.proj(m[:, 0] + h[:, 0])


# ============================================================================ CLIP wrapper (model.py:998-1112)
def _is_norm_param(name):
    """Parameters of the modules the reference's lock_text_tower keeps under `freeze_layer_norm`:
    those under a module literally named "LayerNorm" (model.py:1076, 1094-1096), i.e. HF BERT's
    embedding / attention-output / output LayerNorms = our BERT tower's ln / norm1 / norm2.  The
    Mamba LM's RMSNorms (HF names norm / norm_f) match no "LayerNorm" and are frozen with the rest."""
    return any(part in ("ln", "norm1", "norm2") for part in name.split("."))


class ClipModel(nn.Module):
    """ClipModel(model) as the reference (model.py:1001-1009): wraps a CLIP-like model and SHARES its
    visual / text towers and its logit_scale / logit_bias parameters.  ClipModel(visual, text) builds
    one from two towers with fresh logit_scale = log(1/0.07) (and optional logit_bias)."""
    output_dict = True

    def __init__(self, model, text=None, init_logit_scale=math.log(1 / 0.07), init_logit_bias=None):
        super().__init__()
        self.output_dict = True
        if text is None:                      # reference form: a model with .visual / .text / .logit_scale
            self.visual = model.visual
            self.text = model.text
            self.logit_scale = model.logit_scale
            self.logit_bias = getattr(model, "logit_bias", None)
        else:
            self.visual = model
            self.text = text
            self.logit_scale = nn.Parameter(torch.ones([]) * init_logit_scale)
            self.logit_bias = nn.Parameter(torch.ones([]) * init_logit_bias) if init_logit_bias is not None else None
        self.context_length = getattr(self.text, "context_length", None)
        self.vocab_size = getattr(self.text, "vocab_size", None)

    # image and text towers on two HIP streams (ClipModel.forward).  Under a multi-process group only
    # when train.wrap_ddp joined the streams in its comm hook (ddp_streams_joined): DDP launches a
    # gradient bucket's all-reduce behind one stream, and a bucket may hold gradients of both towers.
    concurrent_towers = os.environ.get("MAMBA_CLIP_AMD_CONCURRENT_TOWERS", "1") != "0"
    ddp_streams_joined = False
    last_main_stream = None
    _side_streams = {}

    @property
    def side_priority(self):
        """HIP priority of the text-tower stream (-1 high, 0 normal, 1 low where the device has it):
        high beside the BERT tower (C3 25.3 -> 25.0 ms per step), normal beside the Mamba tower
        (C2 69.9 -> 70.8 ms at high); profiles/r04/stream_priority/.  MAMBA_CLIP_AMD_SIDE_PRIORITY
        overrides (A/B)."""
        env = os.environ.get("MAMBA_CLIP_AMD_SIDE_PRIORITY")
        if env is not None:
            return int(env)
        return -1 if isinstance(self.text, BertTextEncoder) else 0

    @property
    def side_tower(self):
        """Which tower runs on the side stream: the text tower, for every text tower.  Round 4 put the
        image tower there beside the Mamba text tower (C2 -0.3 ms, profiles/r04/stream_priority/); in
        round 5 that arrangement was not run-to-run reproducible (the scan backward's packed op_sel
        broadcast, found and removed in round 6) and the two measured the same on one box
        (3683 vs 3684 pairs/s), so the text tower stays on the side stream.  MAMBA_CLIP_AMD_SIDE_TOWER=
        image restores the other arrangement for A/B."""
        env = os.environ.get("MAMBA_CLIP_AMD_SIDE_TOWER")
        if env in ("text", "image"):
            return env
        return "text"

    def side_tower_module(self):
        return self.visual if self.side_tower == "image" else self.text

    def side_stream_for(self, device):
        device = torch.device(device)
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        key = (device, int(self.side_priority))
        if key not in ClipModel._side_streams:
            ClipModel._side_streams[key] = torch.cuda.Stream(device=device, priority=key[1])
        return ClipModel._side_streams[key]

    def _side_stream(self, image, text):
        # Only when no kernel of either tower waits on another workgroup of its launch: our HIP kernels
        # never do, and the library GEMMs do not when hipBLASLt launches them data-parallel (one
        # workgroup per output tile, GEMM_GRIDS_DATA_PARALLEL).  Its default stream-K
        # grids split tiles over workgroups that wait on each other's partial sums, so two of them on
        # two streams can each hold part of the CUs and wait forever (the round-3 C3 hang); the C2
        # Mamba tower ran such split launches too (tools/sk_probe.sh).
        if not (self.concurrent_towers and GEMM_GRIDS_DATA_PARALLEL and image is not None
                and text is not None and image.is_cuda and torch.is_grad_enabled()):
            return None
        if torch.distributed.is_available() and torch.distributed.is_initialized() \
                and torch.distributed.get_world_size() > 1 and not self.ddp_streams_joined:
            return None
        return self.side_stream_for(image.device)

    def _towers_two_streams(self, image, text, side, main, dt=None):
        """(image_features, text_features) with the side tower on `side`.  With dt, each tower runs in its own
        weight-cast scope entered on its own stream; without (shared_weight_casts), the caller's scope
        serves both."""
        def scope(module):
            return weight_cast_scope(module, dt) if dt is not None else contextlib.nullcontext()
        if self.side_tower == "image":
            image.record_stream(side)
            with torch.cuda.stream(side), scope(self.visual):
                image_features = self.encode_image(image, normalize=True)
            with scope(self.text):
                text_features = self.encode_text(text, normalize=True)
            main.wait_stream(side)
            image_features.record_stream(main)
        else:
            text.record_stream(side)
            with torch.cuda.stream(side), scope(self.text):
                text_features = self.encode_text(text, normalize=True)
            with scope(self.visual):
                image_features = self.encode_image(image, normalize=True)
            main.wait_stream(side)
            text_features.record_stream(main)
        return image_features, text_features

    def encode_image(self, image, normalize: bool = False):
        f = self.visual(image)
        return l2_normalize(f) if normalize else f

    def encode_text(self, text, normalize: bool = False):
        f = self.text(text)
        return l2_normalize(f) if normalize else f

    # A/B switch (round 4 behaviour): one weight-cast buffer for both towers, made on the main stream and
    # handed to the side stream with record_stream.  Off: each tower casts its own weights on its own stream
    # (DESIGN 4.9), so no buffer crosses the streams in either direction.
    shared_weight_casts = os.environ.get("MAMBA_CLIP_AMD_SHARED_WEIGHT_CASTS", "0") == "1"

    def forward(self, image, text, secondary_text=None):
        # under CUDA autocast: the towers' Linear weights cast to 16 bits in one launch per tower and forward
        # (ops.weight_cast_scope) instead of one cast per weight and use
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else None
        side = self._side_stream(image, text)
        secondary = None
        if side is None:
            with weight_cast_scope(self, dt):
                image_features = self.encode_image(image, normalize=True) if image is not None else None
                text_features = self.encode_text(text, normalize=True) if text is not None else None
                if secondary_text is not None:
                    secondary = self.encode_text(secondary_text, normalize=True)
        elif self.shared_weight_casts:
            with weight_cast_scope(self, dt) as casts:
                main = torch.cuda.current_stream()
                self.last_main_stream = main
                side.wait_stream(main)
                casts.record_stream(side)
                image_features, text_features = self._towers_two_streams(image, text, side, main)
                if secondary_text is not None:
                    secondary = self.encode_text(secondary_text, normalize=True)
        else:
            # the towers are independent until the loss: one of them runs on a second HIP stream (its
            # backward follows it there: autograd runs each backward op on its forward op's stream and joins
            # the streams at the end of backward).  Each tower's weight casts are made on the stream that
            # uses them, so nothing allocated on one stream is read on the other except the inputs (recorded)
            # and the side tower's features (recorded for the loss on the main stream).
            main = torch.cuda.current_stream()
            self.last_main_stream = main                 # train._join_streams_allreduce joins it
            side.wait_stream(main)                       # the inputs, the parameters the optimizer updated
            image_features, text_features = self._towers_two_streams(image, text, side, main, dt)
            if secondary_text is not None:
                with weight_cast_scope(self.text, dt):
                    secondary = self.encode_text(secondary_text, normalize=True)
        if self.output_dict:
            out = {"image_features": image_features, "text_features": text_features,
                   "logit_scale": self.logit_scale.exp()}
            if secondary is not None:
                out["secondary_text_features"] = secondary
            if self.logit_bias is not None:
                out["logit_bias"] = self.logit_bias
            return out
        out = (image_features, text_features, self.logit_scale.exp())
        if secondary is not None:
            out += (secondary,)
        if self.logit_bias is not None:
            out += (self.logit_bias,)
        return out

    def lock_image_tower(self, unlocked_groups=0, freeze_bn_stats=False):
        self.visual.lock(unlocked_groups=unlocked_groups, freeze_bn_stats=freeze_bn_stats)

    def lock_text_tower(self, unlocked_layers: int = 0, freeze_layer_norm: bool = True):
        """model.py:1072-1097: freeze the text transformer -- embeddings, every layer (and the final
        norm) -- or, with unlocked_layers = k, [embeddings, *layers][:-k]; norm parameters follow
        `not freeze_layer_norm`.  The output projection stays trainable (it is not part of the
        HF transformer the reference freezes)."""
        emb, layers, final = self.text.lock_units()
        units = [emb, *layers, final] if not unlocked_layers else [emb, *layers][:-unlocked_layers]
        for unit in units:
            for n, p in unit:
                p.requires_grad = (not freeze_layer_norm) if _is_norm_param(n) else False

    def set_grad_checkpointing(self, enable=True):
        """model.py:1099-1102: both towers recompute their blocks / layers in backward."""
        for t in (self.visual, self.text):
            if hasattr(t, "set_grad_checkpointing"):
                t.set_grad_checkpointing(enable)

    def get_logits(self, image, text, precision=None):
        """(logits_per_image, logits_per_text) = scale * I @ T.T (model.py:1104-1112).

        precision="fp8": the similarity matmul runs on the fp8 MFMA path with
        row-wise e4m3fn quantisation of the normalised features (config 5).
        """
        from .ops import gemm_nt, similarity_fp8
        i = self.encode_image(image, normalize=True)
        t = self.encode_text(text, normalize=True)
        scale = self.logit_scale.exp().float().reshape(())
        if precision == "fp8":
            image_logits = similarity_fp8(i, t, scale)
        else:
            dt = i.dtype if i.dtype == torch.bfloat16 else torch.float32
            image_logits = gemm_nt(i.to(dt), t.to(dt), alpha_dev=scale)
        if self.logit_bias is not None:
            image_logits = image_logits + self.logit_bias
        return image_logits, image_logits.T


# ============================================================================ stage-2 head (model.py:1115-1205)
def unwrap_model(m):
    return m.module if hasattr(m, "module") else m


class ClipClassifier(nn.Module):
    def __init__(self, clip_model, feature_dim=None, num_classes: int = 2, use_visual_only=False,
                 use_text_only=False, use_inner_prod=False):
        super().__init__()
        self.clip_model = unwrap_model(clip_model)
        self.num_classes = num_classes
        for p in self.clip_model.parameters():
            p.requires_grad = False
        if feature_dim is None:
            i_dim = getattr(self.clip_model.visual, "output_dim", None)
            t_dim = getattr(self.clip_model.text, "output_dim", None)
            if i_dim is None or t_dim is None:
                raise ValueError("Could not find image and text feature dimensions in the model")
            feature_dim = i_dim + t_dim
        self.use_visual_only, self.use_text_only, self.use_inner_prod = use_visual_only, use_text_only, use_inner_prod
        out_dim = feature_dim if (use_visual_only or use_text_only or use_inner_prod) else feature_dim // 2
        self.fc = nn.Sequential(nn.Linear(feature_dim, out_dim), nn.ReLU(), nn.Linear(out_dim, num_classes))

    def forward(self, image, text):
        with torch.no_grad():
            out = self.clip_model(image, text)
        i, t = out["image_features"], out["text_features"]
        if self.use_visual_only:
            return self.fc(i.float())
        if self.use_text_only:
            return self.fc(t.float())
        if self.use_inner_prod:
            return self.fc((i * t).float())
        return self.fc(torch.cat((i, t), dim=1).float())

    def get_logits(self, image_features, text_features):
        # the reference's clup_model typo (Appendix A.6) is not reproduced
        logits = image_features * text_features
        if self.clip_model.logit_bias is not None:
            logits = logits + self.clip_model.logit_bias
        return logits

    def classify(self, image, text):
        probabilities = F.softmax(self.forward(image, text), dim=1)
        return torch.argmax(probabilities, dim=1), probabilities


# ============================================================================ MedMamba / VSSM (model.py:174-995)
class PatchEmbed2D(nn.Module):
    """Conv2d k = s = patch (model.py:174-201) as im2col + GEMM, channels-last output."""

    def __init__(self, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None, **kwargs):
        super().__init__()
        self.patch = patch_size if isinstance(patch_size, int) else patch_size[0]
        self.proj = nn.Conv2d(in_chans, embed_dim, self.patch, self.patch)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):  # (B, C, H, W) float, or (B, H, W, C) uint8 raw images
        Bsz, H, W = (x.shape[0], x.shape[1], x.shape[2]) if x.dtype == torch.uint8 else (x.shape[0], x.shape[2], x.shape[3])
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else (
            torch.float32 if x.dtype == torch.uint8 else x.dtype)
        cols = patch_im2col(x, self.patch, dt)
        w = self.proj.weight.reshape(self.proj.weight.shape[0], -1).to(cols.dtype)
        y = F.linear(cols, w, self.proj.bias.to(cols.dtype)).reshape(Bsz, H // self.patch, W // self.patch, -1)
        return self.norm(y) if self.norm is not None else y


class PatchMerging2D(nn.Module):
    """2x2 neighbourhood concat -> LN -> Linear(4C, 2C) (model.py:204-246)."""

    def __init__(self, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = norm_layer(4 * dim)

    def forward(self, x):
        Bsz, H, W, C = x.shape
        h2, w2 = H // 2, W // 2
        parts = [x[:, 0::2, 0::2], x[:, 1::2, 0::2], x[:, 0::2, 1::2], x[:, 1::2, 1::2]]
        x = torch.cat([p[:, :h2, :w2] for p in parts], -1)
        return self.reduction(self.norm(x))


class SS2D(nn.Module):
    """2-D selective scan over four directions (model.py:297-647), scan on the HIP kernel.

    Parameter names/shapes match the reference so its state dicts load as-is.
    """

    def __init__(self, d_model, d_state=16, d_conv=3, expand=2, dt_rank="auto", dt_min=0.001, dt_max=0.1,
                 dt_init="random", dt_scale=1.0, dt_init_floor=1e-4, dropout=0.0, conv_bias=True, bias=False,
                 **kwargs):
        super().__init__()
        self.d_model, self.d_state, self.d_conv, self.expand = d_model, d_state, d_conv, expand
        self.d_inner = int(expand * d_model)
        self.dt_rank = math.ceil(d_model / 16) if dt_rank == "auto" else dt_rank
        K, di, R, N = 4, self.d_inner, self.dt_rank, d_state
        self.in_proj = nn.Linear(d_model, 2 * di, bias=bias)
        self.conv2d = nn.Conv2d(di, di, d_conv, groups=di, bias=conv_bias, padding=(d_conv - 1) // 2)
        self.act = nn.SiLU()
        xw = torch.empty(K, R + 2 * N, di)
        for k in range(K):
            nn.init.kaiming_uniform_(xw[k], a=math.sqrt(5))
        self.x_proj_weight = nn.Parameter(xw)
        std = R ** -0.5 * dt_scale
        dtw = torch.empty(K, di, R)
        if dt_init == "constant":
            nn.init.constant_(dtw, std)
        elif dt_init == "random":
            nn.init.uniform_(dtw, -std, std)
        else:
            raise NotImplementedError
        self.dt_projs_weight = nn.Parameter(dtw)
        self.dt_projs_bias = nn.Parameter(torch.stack([_dt_bias_init(di, dt_min, dt_max, dt_init_floor)
                                                       for _ in range(K)]))
        A = torch.arange(1, N + 1, dtype=torch.float32).repeat(K * di, 1)
        self.A_logs = nn.Parameter(torch.log(A))
        self.A_logs._no_weight_decay = True
        self.Ds = nn.Parameter(torch.ones(K * di))
        self.Ds._no_weight_decay = True
        self.out_norm = nn.LayerNorm(di)
        self.out_proj = nn.Linear(di, d_model, bias=bias)
        self.dropout = nn.Dropout(dropout) if dropout > 0.0 else None

    def _scan_u(self, u):  # u = [x, x^T] (B, 2, d, L) fp32 -> (B, 4 d, L), directions in their own frames
        """model.py:503-565 with the cross-scan inside the kernels: u holds x and x^T once (the
        reference stacks [x, x^T, flip x, flip x^T]); the per-direction projections read it in place;
        directions 2 / 3 walk u blocks 0 / 1 backwards (grouped_scan_fn), so their outputs come back
        un-flipped.  Blocks 1 / 3 stay in the transposed (W, H) frame: the merge reads them there."""
        Bsz, _, d, L = u.shape
        K = 4
        wx, wdt = self.x_proj_weight.to(u.dtype), self.dt_projs_weight.to(u.dtype)
        if ss2d_proj_ok(u, wx, wdt):
            # both projections on mc_ss2d_group_proj, no permuted operand copies (ops.SS2DProjFn)
            dts, Bs, Cs = ss2d_proj(u, wx, wdt, self.dt_rank, self.d_state)
        else:
            x_dbl = torch.einsum("bjdl,ijcd->bijcl", u, wx.view(2, 2, -1, d)).reshape(Bsz, K, -1, L)   # k = 2 i + j
            dts, Bs, Cs = torch.split(x_dbl, [self.dt_rank, self.d_state, self.d_state], dim=2)
            dts = torch.einsum("bkrl,kdr->bkdl", dts, wdt)
        return grouped_scan_fn(u.float().reshape(Bsz, 2 * d, L), dts.float().reshape(Bsz, K * d, L),
                               -torch.exp(self.A_logs.float()), Bs.float(), Cs.float(), self.Ds.float(),
                               self.dt_projs_bias.float().reshape(-1), delta_softplus=True,
                               reverse_groups=SS2D_REVERSE_GROUPS, u_groups=SS2D_U_GROUPS)

    def forward_core(self, x):  # (B, d, H, W) -> four (B, d, L) maps, fp32, reference order
        """The reference's forward_corev0 contract (model.py:503-565) on a conv output: y1 .. y4 back in
        the (H, W) frame.  Not on the forward path (forward fuses the stack and the merge)."""
        Bsz, d, H, W = x.shape
        L = H * W
        u = torch.stack([x.reshape(Bsz, d, L), x.transpose(2, 3).reshape(Bsz, d, L)], dim=1).float()
        out = self._scan_u(u).view(Bsz, 4, d, L)
        back = lambda t: t.reshape(Bsz, d, W, H).transpose(2, 3).reshape(Bsz, d, L)  # noqa: E731
        return out[:, 0], out[:, 2], back(out[:, 1]), back(out[:, 3])

    def forward(self, x, **kwargs):  # (B, H, W, C)
        # model.py:630-647.  x / z stay channels-last halves of in_proj's output (no permute copy);
        # ss2d_conv_stack writes silu(conv2d(x)) straight into the scan input u = [x, x^T] (fp32), and
        # ss2d_merge_ln_gate sums the four directions (the two column-major ones read transposed),
        # applies out_norm and the silu(z) gate, channels-last for out_proj (mc_ss2d.h)
        x, z = self.in_proj(x).chunk(2, dim=-1)
        u = ss2d_conv_stack(x, self.conv2d.weight, self.conv2d.bias)
        y = ss2d_merge_ln_gate(self._scan_u(u), z, self.out_norm.weight, self.out_norm.bias, self.out_norm.eps)
        out = self.out_proj(y)
        return self.dropout(out) if self.dropout is not None else out

def channel_shuffle(x, groups):
    Bsz, H, W, C = x.shape
    return x.view(Bsz, H, W, groups, C // groups).transpose(3, 4).reshape(Bsz, H, W, C)


class SS_Conv_SSM(nn.Module):
    """Half the channels through a conv stack, half through SS2D; shuffle; residual (model.py:666-723)."""

    def __init__(self, hidden_dim=0, drop_path=0.0, norm_layer=partial(nn.LayerNorm, eps=1e-6), attn_drop_rate=0.0,
                 d_state=16, **kwargs):
        super().__init__()
        h = hidden_dim // 2
        self.ln_1 = norm_layer(h)
        self.self_attention = SS2D(d_model=h, dropout=attn_drop_rate, d_state=d_state, **kwargs)
        self.drop_path = nn.Identity() if drop_path == 0 else _DropPath(drop_path)
        self.conv33conv33conv11 = nn.Sequential(
            nn.BatchNorm2d(h), nn.Conv2d(h, h, 3, 1, 1), nn.BatchNorm2d(h), nn.ReLU(),
            nn.Conv2d(h, h, 3, 1, 1), nn.BatchNorm2d(h), nn.ReLU(), nn.Conv2d(h, h, 1, 1), nn.ReLU())

    def forward(self, inp):
        left, right = inp.chunk(2, dim=-1)
        x = self.drop_path(self.self_attention(self.ln_1(right)))
        left = self.conv33conv33conv11(left.permute(0, 3, 1, 2).contiguous()).permute(0, 2, 3, 1).contiguous()
        return channel_shuffle(torch.cat((left, x), dim=-1), groups=2) + inp


class _DropPath(nn.Module):
    def __init__(self, p):
        super().__init__()
        self.p = p

    def forward(self, x):
        if not self.training or self.p == 0.0:
            return x
        keep = x.new_empty((x.shape[0],) + (1,) * (x.dim() - 1)).bernoulli_(1 - self.p)
        return x * keep / (1 - self.p)


class VSSLayer(nn.Module):
    def __init__(self, dim, depth, attn_drop=0.0, drop_path=0.0, norm_layer=nn.LayerNorm, downsample=None,
                 use_checkpoint=False, d_state=16, **kwargs):
        super().__init__()
        self.dim, self.use_checkpoint = dim, use_checkpoint
        self.blocks = nn.ModuleList([
            SS_Conv_SSM(hidden_dim=dim, drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                        norm_layer=norm_layer, attn_drop_rate=attn_drop, d_state=d_state)
            for i in range(depth)])
        self.downsample = downsample(dim=dim, norm_layer=norm_layer) if downsample is not None else None

    def forward(self, x):
        for blk in self.blocks:
            x = torch.utils.checkpoint.checkpoint(blk, x, use_reentrant=False) if self.use_checkpoint else blk(x)
        return self.downsample(x) if self.downsample is not None else x


class VSSM(nn.Module):
    """MedMamba backbone + head (model.py:868-995); "medmamba" = depths [2,2,8,2], dims [64,128,256,512]."""

    def __init__(self, patch_size=4, in_chans=3, num_classes=1000, depths=(2, 2, 4, 2), dims=(96, 192, 384, 768),
                 d_state=16, drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.1, norm_layer=nn.LayerNorm,
                 patch_norm=True, use_checkpoint=False, **kwargs):
        super().__init__()
        depths, dims = list(depths), list(dims)
        self.num_classes, self.num_layers = num_classes, len(depths)
        self.embed_dim, self.num_features, self.dims = dims[0], dims[-1], dims
        self.patch_embed = PatchEmbed2D(patch_size, in_chans, dims[0], norm_layer if patch_norm else None)
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [v.item() for v in torch.linspace(0, drop_path_rate, sum(depths))]
        self.layers = nn.ModuleList([
            VSSLayer(dims[i], depths[i], d_state=math.ceil(dims[0] / 6) if d_state is None else d_state,
                     attn_drop=attn_drop_rate, drop_path=dpr[sum(depths[:i]): sum(depths[: i + 1])],
                     norm_layer=norm_layer, downsample=PatchMerging2D if i < self.num_layers - 1 else None,
                     use_checkpoint=use_checkpoint)
            for i in range(self.num_layers)])
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.head = nn.Linear(self.num_features, num_classes) if num_classes > 0 else nn.Identity()
        self.output_dim = num_classes if num_classes > 0 else self.num_features
        self.apply(self._init_weights)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    @staticmethod
    def _init_weights(m):
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def forward_backbone(self, x):
        x = self.pos_drop(self.patch_embed(x))
        for layer in self.layers:
            x = layer(x)
        return x

    def forward(self, x):
        x = self.forward_backbone(x).permute(0, 3, 1, 2)
        return self.head(torch.flatten(self.avgpool(x), 1))


# ============================================================================ factory (model.py:1257-1289)
MODEL_CONFIGS = {
    # C1: tiny plumbing config (BASELINE configs[0]): Mamba text d_model 128, L = 256, d_state 16, 32-dim output
    "tiny-mamba-clip": dict(vision=dict(img_size=32, patch=8, width=64, layers=2, heads=4, output_dim=32),
                            text=dict(vocab_size=1000, context_length=256, d_model=128, n_layer=2, output_dim=32)),
    # C2: ViT-B/16 + Mamba-130M text (BASELINE configs[1])
    "vit_b16-mamba130m": dict(vision=dict(), text=dict(vocab_size=50280, context_length=77, d_model=768,
                                                        n_layer=24, output_dim=512)),
    # C4 text tower (BASELINE configs[3])
    "mamba790m-text": dict(vision=dict(), text=dict(vocab_size=50280, context_length=4096, d_model=1536,
                                                     n_layer=48, output_dim=512)),
    # C3: BiomedCLIP-shaped (ViT-B/16 + PubMedBERT-256), random init (BASELINE configs[2])
    "biomedclip-vit_b16-pubmedbert256": dict(vision=dict(), bert=dict()),
}


def build_clip(name):
    cfg = MODEL_CONFIGS[name]
    visual = VisionTransformer(**cfg["vision"])
    text = BertTextEncoder(**cfg["bert"]) if "bert" in cfg else MambaTextEncoder(**cfg["text"])
    return ClipModel(visual, text)


def init_model(model, tokenizer=None, aug_cfg=None, is_clip=False, use_tokenizer=False):
    """Returns (model, preprocess_train, preprocess_val, tokenizer) like model.py:1257-1289.

    "medmamba" -> VSSM(depths=[2,2,8,2], dims=[64,128,256,512], num_classes=2);
    a MODEL_CONFIGS name -> a random-init ClipModel (no hub access offline);
    a callable -> model().  Preprocessing is identity on synthetic tensors.
    """
    if model == "medmamba":
        model = VSSM(depths=[2, 2, 8, 2], dims=[64, 128, 256, 512], num_classes=2)
    elif isinstance(model, str):
        if model not in MODEL_CONFIGS:
            raise ValueError(f"unknown model {model!r}: offline build knows {sorted(MODEL_CONFIGS)}")
        model = build_clip(model)
    elif callable(model):
        model = model()
    if is_clip and not isinstance(model, ClipModel):
        model = ClipModel(model)          # shares the towers AND logit_scale / logit_bias (model.py:1274-1275)
    if use_tokenizer and tokenizer is not None and callable(tokenizer):
        tokenizer = tokenizer()
    identity = (lambda x: x)
    return model, identity, identity, tokenizer
