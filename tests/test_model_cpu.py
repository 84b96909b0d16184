"""CPU checks of the module API (construction, shapes, parameter counts); no kernels run."""
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
