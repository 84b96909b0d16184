#!/usr/bin/env python3
"""One C2 training step (forward, ClipLoss, backward, AdamW) after two warm-up steps, for kernel traces."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
import argparse
import torch
ap = argparse.ArgumentParser()
ap.add_argument("--model", default="vit_b16-mamba130m")
ap.add_argument("--batch", type=int, default=256)
args = ap.parse_args()
from types import SimpleNamespace
from mamba_clip_amd import train
from mamba_clip_amd.data import synthetic_batch
from mamba_clip_amd.loss import ClipLoss
from mamba_clip_amd.model import build_clip
from mamba_clip_amd.tuning import load_gemm_tuning
from mamba_clip_amd.utils.amp_utils import get_autocast
dev = torch.device("cuda", 0)
load_gemm_tuning(model=args.model)
targs = SimpleNamespace(precision="amp_bf16", lr=5e-4, wd=0.2, beta1=0.9, beta2=0.98, eps=1e-6, grad_clip_norm=None, accum_freq=1)
model = build_clip(args.model).to(dev)
images, texts, _ = synthetic_batch(args.batch, 224, model.text.context_length, model.text.vocab_size, device=dev, seed=1000)
opt = train.create_optimizer(model, targs)
loss_fn = ClipLoss()
autocast = get_autocast(targs.precision)
for s in range(3):
    opt.zero_grad(set_to_none=True)
    with autocast():
        out = model(images, texts)
        total = loss_fn(**out)["contrastive_loss"]
    total.backward()
    train.optimizer_step(model, opt, None, targs)
    torch.cuda.synchronize()
print("ok")
