"""Dev tool: torch.profiler table of the C2 train step (op-level attribution of GPU time, input shapes).

usage: python tools/torch_prof.py [--batch 256] [--rows 60]
"""
import argparse
import os
import sys
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
from mamba_clip_amd.data import synthetic_batch  # noqa: E402
from mamba_clip_amd.loss import ClipLoss  # noqa: E402
from mamba_clip_amd.model import build_clip  # noqa: E402
from mamba_clip_amd.train import create_optimizer, train_step  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--rows", type=int, default=60)
ap.add_argument("--model", default="vit_b16-mamba130m")
args = ap.parse_args()
dev = torch.device("cuda")
targs = SimpleNamespace(precision="amp_bf16", lr=5e-4, wd=0.2, beta1=0.9, beta2=0.98, eps=1e-6, grad_clip_norm=None)
torch.manual_seed(0)
model = build_clip(args.model).to(dev)
opt = create_optimizer(model, targs)
loss = ClipLoss()
img, txt, tgt = synthetic_batch(args.batch, 224, model.text.context_length, model.text.vocab_size, device=dev)
for _ in range(3):
    train_step(model, img, txt, tgt, loss, opt, None, targs)
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
    for _ in range(2):
        train_step(model, img, txt, tgt, loss, opt, None, targs)
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=args.rows,
                                                           max_name_column_width=40, max_shapes_column_width=70))
