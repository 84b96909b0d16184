"""CPU checks of the module API (construction, shapes, parameter counts) and of the module wiring via the CPU restatement ops; no HIP kernels run."""
import torch

from mamba_clip_amd.model import MODEL_CONFIGS, ClipClassifier, build_clip, init_model


def _count(m):
    return sum(p.numel() for p in m.parameters())


def test_configs_build_and_sizes():
    m = build_clip("vit_b16-mamba130m")
    vis, txt = _count(m.visual), _count(m.text)
    assert 85e6 < vis < 90e6, vis                 # ViT-B/16 (+ 768x512 proj)
    assert 125e6 < txt < 135e6, txt               # Mamba-130M (+ proj)
    assert m.context_length == 77 and m.vocab_size == 50280
    assert set(MODEL_CONFIGS) >= {"tiny-mamba-clip", "vit_b16-mamba130m", "biomedclip-vit_b16-pubmedbert256"}


def test_medmamba_param_count_matches_reference():
    m, pre_t, pre_v, tok = init_model("medmamba")
    assert _count(m) == 8529666                   # measured on the reference


def test_classifier_head_shapes():
    clip = build_clip("tiny-mamba-clip")
    head = ClipClassifier(clip, feature_dim=None, num_classes=2)
    assert head.fc[0].in_features == 64 and head.fc[0].out_features == 32
    assert all(not p.requires_grad for p in head.clip_model.parameters())
    assert ClipClassifier(clip, num_classes=3, use_inner_prod=True, feature_dim=32).fc[0].out_features == 32


def test_fused_vit_blocks_equal_unfused_math_cpu():
    """The (m, h) fused-residual ViT (CPU restatement ops) equals the textbook pre-LN recurrence."""
    import torch.nn.functional as F
    from mamba_clip_amd.model import VisionTransformer
    from oracle.cpu_model import oracle_ops
    torch.manual_seed(0)
    vit = VisionTransformer(img_size=32, patch=8, width=64, layers=2, heads=4, output_dim=16)
    img = torch.randn(3, 3, 32, 32)
    with oracle_ops(), torch.no_grad():
        out = vit(img)
        x = vit.patch_embed.proj(img).flatten(2).transpose(1, 2)
        x = torch.cat([vit.cls_token.expand(3, -1, -1), x], 1) + vit.pos_embed
        for blk in vit.blocks:
            x = x + blk.attn(blk.norm1(x))
            x = x + blk.fc2(F.gelu(blk.fc1(blk.norm2(x))))
        ref = vit.head(vit.norm(x)[:, 0])
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-6)


def test_cpu_restatement_train_step_runs():
    from oracle.cpu_model import cpu_train_pairs_per_sec
    pps, secs = cpu_train_pairs_per_sec("tiny-mamba-clip", batch=4, steps=1, warmup=1)
    assert pps > 0 and secs > 0


def test_cli_parser_hot_path_flags():
    from mamba_clip_amd.cli import build_parser
    a = build_parser().parse_args(["--synthetic", "--batch-size", "8", "--local-loss", "--gather-with-grad",
                                   "--lr-scheduler", "const", "--stage", "2", "--use-inner-prod", "--accum-freq", "2"])
    assert a.synthetic and a.local_loss and a.gather_with_grad and a.stage == 2 and a.use_inner_prod
    assert a.precision == "amp_bf16" and a.accum_freq == 2 and a.model == "vit_b16-mamba130m"


def test_cli_requires_synthetic():
    import pytest
    from mamba_clip_amd.cli import main
    with pytest.raises(SystemExit):
        main(["--batch-size", "4"])


def test_schedulers_match_reference_formulas():
    import math
    from mamba_clip_amd.scheduler import const_lr, const_lr_cooldown, cosine_lr

    class Opt:
        param_groups = [{"lr": 0.0}]
    o = Opt()
    f = cosine_lr(o, 1.0, 10, 110)
    assert abs(f(0) - 0.1) < 1e-12 and abs(f(9) - 1.0) < 1e-12
    assert abs(f(60) - 0.5 * (1 + math.cos(math.pi * 50 / 100))) < 1e-12
    g = const_lr(o, 2.0, 4, 100)
    assert g(1) == 1.0 and g(50) == 2.0
    h = const_lr_cooldown(o, 1.0, 0, 100, 20, cooldown_power=1.0, cooldown_end_lr=0.0)
    assert h(79) == 1.0 and abs(h(90) - 0.5) < 1e-12 and o.param_groups[0]["lr"] == h(90)


def test_split_k_projection_autograd_cpu():
    """linear_sk / wleft_mm (split-K weight-gradient projections) against autograd, incl. transposed-view inputs."""
    import torch
    from mamba_clip_amd.ops import linear_sk, wleft_mm
    torch.manual_seed(0)
    x = torch.randn(64, 16, dtype=torch.float64, requires_grad=True)
    w = torch.randn(8, 16, dtype=torch.float64, requires_grad=True)
    b = torch.randn(8, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(lambda x, w, b: linear_sk(x, w, b), (x, w, b))
    xt = torch.randn(16, 64, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(lambda xt, w: linear_sk(xt.t(), w, None), (xt, w))
    X = torch.randn(16, 64, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(lambda w, X: wleft_mm(w, X), (w, X))
    H = torch.randn(64, 16, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(lambda w, H: wleft_mm(w, H.t()), (w, H))


# ---------------------------------------------------------------- boundary fidelity (model.py:998-1112, 1257-1289)
def test_clip_model_reference_constructor_shares_logit_params():
    """ClipModel(model) shares the towers and logit_scale / logit_bias (model.py:1001-1009), and
    init_model(..., is_clip=True) keeps a learned temperature (model.py:1274-1275)."""
    import math
    import torch.nn as nn
    from mamba_clip_amd.model import ClipModel

    base = build_clip("tiny-mamba-clip")
    with torch.no_grad():
        base.logit_scale.fill_(3.3)
    base.logit_bias = nn.Parameter(torch.tensor(-2.0))
    wrapped = ClipModel(base)
    assert wrapped.visual is base.visual and wrapped.text is base.text
    assert wrapped.logit_scale is base.logit_scale and wrapped.logit_bias is base.logit_bias
    assert wrapped.context_length == 256 and wrapped.vocab_size == 1000

    class Raw(nn.Module):                   # an open_clip-like CLIP that is not a ClipModel
        def __init__(self):
            super().__init__()
            self.visual, self.text = base.visual, base.text
            self.logit_scale = nn.Parameter(torch.tensor(2.5))
            self.logit_bias = None
    m, _, _, _ = init_model(Raw, is_clip=True)
    assert isinstance(m, ClipModel) and float(m.logit_scale) == 2.5 and m.logit_bias is None
    fresh = ClipModel(base.visual, base.text)
    assert abs(float(fresh.logit_scale) - math.log(1 / 0.07)) < 1e-6 and fresh.logit_bias is None


def test_lock_text_tower_freezes_embeddings_and_layers():
    """model.py:1072-1097: full lock freezes embeddings + every layer (norms follow freeze_layer_norm);
    unlocked_layers=k freezes [embeddings, *layers][:-k]; the projection stays trainable."""
    def trainable(m):
        return {n for n, p in m.text.named_parameters() if p.requires_grad}

    m = build_clip("tiny-mamba-clip")                          # Mamba text: 2 layers
    m.lock_text_tower()
    assert trainable(m) == {"proj.weight"}
    m = build_clip("tiny-mamba-clip")
    # the Mamba RMSNorms (HF norm / norm_f) are not "LayerNorm" modules: frozen either way (model.py:1076)
    m.lock_text_tower(freeze_layer_norm=False)
    assert trainable(m) == {"proj.weight"}
    m = build_clip("tiny-mamba-clip")
    m.lock_text_tower(unlocked_layers=1)
    t = trainable(m)
    assert "embedding.weight" not in t and not any(n.startswith("layers.0.") for n in t)
    assert any(n.startswith("layers.1.") for n in t) and "norm_f" in t and "proj.weight" in t
    from mamba_clip_amd.model import BertTextEncoder, ClipModel, VisionTransformer
    bm = ClipModel(VisionTransformer(img_size=32, patch=8, width=64, layers=1, heads=4, output_dim=16),
                   BertTextEncoder(vocab_size=100, context_length=8, width=64, layers=2, heads=4, output_dim=16))
    bm.lock_text_tower(unlocked_layers=1)
    t = trainable(bm)
    assert not {"tok.weight", "pos", "ln.weight"} & t and not any(n.startswith("blocks.0.") for n in t)
    assert any(n.startswith("blocks.1.") for n in t) and any(n.startswith("proj.") for n in t)
    # BERT's LayerNorms (embeddings + both per block) follow `not freeze_layer_norm`
    bm.lock_text_tower(freeze_layer_norm=False)
    t = trainable(bm)
    assert {"ln.weight", "ln.bias", "blocks.0.norm1.weight", "blocks.1.norm2.bias"} <= t
    assert not any(("attn" in n or "fc" in n) for n in t) and "tok.weight" not in t


def test_ss2d_parameter_inits_follow_reference_statistics():
    """model.py:437-501: dt_proj weight ~ U(+-dt_rank^-0.5), softplus(dt bias) ~ logU[1e-3, 1e-1]
    (floored 1e-4), A_logs = log(1..N) per channel (S4D-real), Ds = 1, x_proj kaiming-uniform."""
    import math
    import torch.nn.functional as F
    from mamba_clip_amd.model import SS2D
    torch.manual_seed(0)
    m = SS2D(d_model=128)
    R, di, N = m.dt_rank, m.d_inner, m.d_state
    assert (R, di, N) == (8, 256, 16)
    w = m.dt_projs_weight
    assert w.shape == (4, di, R) and float(w.abs().max()) <= R ** -0.5 + 1e-7
    assert abs(float(w.std()) - R ** -0.5 / math.sqrt(3)) < 0.02 * R ** -0.5
    dt = F.softplus(m.dt_projs_bias)
    assert dt.shape == (4, di) and float(dt.min()) >= 1e-4 * 0.999 and float(dt.max()) <= 0.1 * 1.001
    # log-uniform: log dt is uniform on [log 1e-3, log 1e-1] -> mean at the midpoint, std (range)/sqrt(12)
    lg = dt.log()
    mid, rng = (math.log(1e-3) + math.log(1e-1)) / 2, math.log(1e-1) - math.log(1e-3)
    assert abs(float(lg.mean()) - mid) < 0.05 * rng and abs(float(lg.std()) - rng / math.sqrt(12)) < 0.05 * rng
    torch.testing.assert_close(m.A_logs, torch.log(torch.arange(1, N + 1).float()).repeat(4 * di, 1))
    assert torch.equal(m.Ds, torch.ones(4 * di))
    bound = 1 / math.sqrt(di)                       # kaiming_uniform(a=sqrt(5)) on fan_in = d_inner
    assert m.x_proj_weight.shape == (4, R + 2 * N, di) and float(m.x_proj_weight.abs().max()) <= bound + 1e-7


def test_ss2d_c1_shape_cpu_restatement_matches_reference_golden():
    """Our SS2D module wiring at C1's exact shape (d_model 128, 8x16x16) with the CPU restatement ops,
    against the reference SS2D golden -- the GPU test runs the same fixture on the HIP path."""
    from conftest import load_golden
    from mamba_clip_amd.model import SS2D
    from oracle.cpu_model import oracle_ops
    g = load_golden("ss2d_c1_d128_h16w16.safetensors")
    gen = torch.Generator().manual_seed(2025)
    x = torch.randn(8, 16, 16, 128, generator=gen)
    gy = torch.randn(8, 16, 16, 128, generator=gen)
    chk = torch.stack([x.double().sum(), x.double().abs().sum(), gy.double().sum()])
    torch.testing.assert_close(chk, g["x_checksum"], rtol=0, atol=0)
    m = SS2D(d_model=128).eval()
    m.load_state_dict({k[3:]: v for k, v in g.items() if k.startswith("sd.")})
    xg = x.requires_grad_(True)
    with oracle_ops():
        y = m(xg)
        y.backward(gy)
    torch.testing.assert_close(y.detach(), g["y"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(xg.grad, g["gx"], rtol=1e-3, atol=1e-5)
    for n, p in m.named_parameters():
        ref = g[f"grad.{n}"]
        torch.testing.assert_close(p.grad, ref, rtol=1e-3, atol=1e-4 * float(ref.abs().max()), msg=n)


def test_vssm_tiny_cpu_restatement_matches_reference_golden():
    """Our VSSM wiring (PatchEmbed2D im2col incl. its inverse-permutation backward, PatchMerging2D,
    SS_Conv_SSM stages, avgpool head) with the CPU restatement ops vs the reference VSSM golden."""
    from conftest import load_golden
    from mamba_clip_amd.model import VSSM
    from mamba_clip_amd.ops import PatchIm2colFn
    from oracle.cpu_model import oracle_ops
    g = load_golden("vssm_tiny_d16.safetensors")
    m = VSSM(patch_size=4, in_chans=3, num_classes=2, depths=[1, 1, 2, 1], dims=[16, 32, 64, 128]).eval()
    m.load_state_dict({k[3:]: v for k, v in g.items() if k.startswith("sd.")})
    x = g["x"].clone().requires_grad_(True)
    with oracle_ops():
        y = m(x)
        y.backward(g["gy"])
    torch.testing.assert_close(y.detach(), g["y"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(x.grad, g["gx"], rtol=1e-3, atol=1e-6)
    torch.testing.assert_close(m.head.weight.grad, g["grad.head.weight"], rtol=1e-3, atol=1e-6)
    # the product im2col's backward is the exact inverse permutation of the unfold layout
    img = torch.randn(2, 3, 8, 12, dtype=torch.float64)
    cols = torch.nn.functional.unfold(img, 4, stride=4).transpose(1, 2).reshape(-1, 48)
    back = PatchIm2colFn.backward(type("C", (), {"meta": (2, 3, 8, 12, 4, torch.float64)})(), cols)[0]
    assert torch.equal(back, img)


def test_gemm_grids_data_parallel_gate():
    """Importing the package asks hipBLASLt for data-parallel GEMM grids; the two-stream
    towers are gated on it: with the variable preset to anything but 1 the gate is off and ClipModel
    keeps both towers on one stream."""
    import os
    import subprocess
    import sys
    import mamba_clip_amd
    assert os.environ["TENSILE_STREAMK_DATA_PARALLEL"] == "1"
    assert mamba_clip_amd.GEMM_GRIDS_DATA_PARALLEL
    code = ("import mamba_clip_amd, mamba_clip_amd.model as m; "
            "print(mamba_clip_amd.GEMM_GRIDS_DATA_PARALLEL, m.GEMM_GRIDS_DATA_PARALLEL)")
    env = dict(os.environ, TENSILE_STREAMK_DATA_PARALLEL="0")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = os.path.join(root, "mamba-clip_amd") + os.pathsep + env.get("PYTHONPATH", "")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["False", "False"]


def test_grad_checkpointing_recomputes_same_gradients_cpu():
    """ClipModel.set_grad_checkpointing (reference model.py:1099-1102) recomputes every ViT block and
    Mamba layer in backward: same loss and gradients as without it (CPU restatement ops)."""
    from oracle.cpu_model import oracle_clip_loss, oracle_ops
    torch.manual_seed(0)
    model, _, _, _ = init_model("tiny-mamba-clip")
    img = torch.randn(4, 3, 32, 32)
    tok = torch.randint(1, 1000, (4, 16))
    res = []
    for ck in (False, True):
        model.set_grad_checkpointing(ck)
        assert model.visual.grad_checkpointing == ck and model.text.grad_checkpointing == ck
        model.zero_grad(set_to_none=True)
        with oracle_ops():
            loss = oracle_clip_loss(**model(img, tok))["contrastive_loss"]
            loss.backward()
        res.append((loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}))
    (l0, g0), (l1, g1) = res
    torch.testing.assert_close(l1, l0, rtol=0, atol=0)
    assert g0.keys() == g1.keys() and len(g0) > 10
    for n in g0:
        torch.testing.assert_close(g1[n], g0[n], rtol=1e-6, atol=1e-7, msg=n)
