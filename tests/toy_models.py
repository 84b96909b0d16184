"""Toy models for the train-step fixtures (tests/golden/make_golden.py `gen_train`).

Tiny modules with the reference's model contracts, so the REFERENCE's own
train_one_epoch / prepare_params (train.py:92-385, pipeline.py:205-408) can run
them on the CPU here, and ours can run the very same weights:

* ToyClip       -- ClipModel's dict contract (model.py:1019-1064): normalised
                   image/text features + exp(logit_scale).  Parameter names
                   include "ln" and "bias" so the AdamW grouping
                   (pipeline.py:280-298) has members on both sides.
* ToyClassifier -- a stage-2 style head (model.py:1174-1192): logits (b, C)
                   from (image, text); trained with cross_entropy_loss on the
                   balanced-mixup soft targets (loss.py:47-53).
* ToyData       -- the data["train"] object train_one_epoch reads: set_epoch,
                   dataloader.num_batches / num_samples, and ComboLoader-shaped
                   batches ((img, txt, tgt), (bal_img, bal_txt, bal_tgt)).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

IMG = (3, 8, 8)
VOCAB, CTX, WIDTH = 64, 6, 16


class ToyClip(nn.Module):
    def __init__(self):
        super().__init__()
        self.visual = nn.Sequential(nn.Flatten(), nn.Linear(math.prod(IMG), WIDTH))
        self.visual_ln = nn.LayerNorm(WIDTH)
        self.text = nn.Embedding(VOCAB, WIDTH)
        self.text_proj = nn.Linear(WIDTH, WIDTH, bias=False)
        self.logit_scale = nn.Parameter(torch.ones([]) * math.log(1 / 0.07))

    def forward(self, image, text):
        i = F.normalize(self.visual_ln(self.visual(image)), dim=-1)
        t = F.normalize(self.text_proj(self.text(text).mean(1)), dim=-1)
        return {"image_features": i, "text_features": t, "logit_scale": self.logit_scale.exp()}


class ToyClassifier(nn.Module):
    def __init__(self, num_classes=2):
        super().__init__()
        self.visual = nn.Sequential(nn.Flatten(), nn.Linear(math.prod(IMG), WIDTH))
        self.text = nn.Embedding(VOCAB, WIDTH)
        self.fc = nn.Sequential(nn.Linear(2 * WIDTH, WIDTH), nn.ReLU(), nn.Linear(WIDTH, num_classes))

    def forward(self, image, text):
        return self.fc(torch.cat([self.visual(image), self.text(text).mean(1)], dim=1))


def toy_batches(n_batches, b, seed, num_classes=2):
    """ComboLoader-shaped batches: ((img, txt, tgt), (bal_img, bal_txt, bal_tgt))."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n_batches):
        pair = []
        for _ in range(2):
            img = torch.randn((b,) + IMG, generator=g)
            txt = torch.randint(1, VOCAB, (b, CTX), generator=g)
            tgt = torch.randint(0, num_classes, (b,), generator=g)
            pair.append((img, txt, tgt))
        out.append(tuple(pair))
    return out


class _Loader(list):
    def __init__(self, batches, b):
        super().__init__(batches)
        self.num_batches = len(batches)
        self.num_samples = len(batches) * b


class ToyData:
    def __init__(self, batches, b):
        self.dataloader = _Loader(batches, b)
        self.epochs = []

    def set_epoch(self, epoch):
        self.epochs.append(epoch)
