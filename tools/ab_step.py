"""Dev tool: interleaved same-box A/B of the C2 training step with a model toggle (not the bench contract).

usage: python tools/ab_step.py --toggle fuse_dt_proj [--model vit_b16-mamba130m --batch 256 --steps 10 --reps 3]
The toggle is an attribute set on every module that has it (True = variant A, False = variant B), or
`ops.NAME` / `train.NAME` for a module-level flag of mamba_clip_amd.ops / .train.
"""
import argparse
import os
import sys
import time
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
from mamba_clip_amd.data import synthetic_batch  # noqa: E402
from mamba_clip_amd.loss import ClipLoss  # noqa: E402
from mamba_clip_amd.model import build_clip  # noqa: E402
from mamba_clip_amd.train import create_optimizer, train_step  # noqa: E402
from mamba_clip_amd.tuning import load_gemm_tuning  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="vit_b16-mamba130m")
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--toggle", default="fuse_dt_proj")
ap.add_argument("--watchdog", type=float, default=0, help="dump every thread's stack and exit after S seconds")
args = ap.parse_args()
if args.watchdog:
    import faulthandler
    faulthandler.dump_traceback_later(args.watchdog, exit=True)

targs = SimpleNamespace(precision="amp_bf16", lr=5e-4, wd=0.2, beta1=0.9, beta2=0.98, eps=1e-6,
                        grad_clip_norm=None, accum_freq=1, rank=0, world_size=1, distributed=False)
load_gemm_tuning()
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = build_clip(args.model).to(dev)
opt = create_optimizer(model, targs)
loss = ClipLoss()
images, texts, targets = synthetic_batch(args.batch, 224, model.text.context_length, model.text.vocab_size,
                                         device=dev, seed=1000)
if args.toggle.startswith(("ops.", "train.")):
    import importlib
    modname, attr = args.toggle.split(".", 1)
    holder = importlib.import_module(f"mamba_clip_amd.{modname}")
    mods, tog = [holder], attr
else:
    mods = [m for m in model.modules() if hasattr(m, args.toggle)]
    tog = args.toggle
print(f"{len(mods)} holders carry {args.toggle}")


def run(flag, steps):
    for m in mods:
        setattr(m, tog, flag)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        train_step(model, images, texts, targets, loss, opt, None, targs)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps * 1e3


print("warmup A", flush=True)
run(True, 3)
print("warmup B", flush=True)
run(False, 3)
for r in range(args.reps):
    a = run(True, args.steps)
    b = run(False, args.steps)
    print(f"rep {r}: {args.toggle}=True {a:.2f} ms/step   {args.toggle}=False {b:.2f} ms/step", flush=True)
