"""Dev tool: which library GEMM kernels does one training step dispatch, for which shapes, towers
and streams, and with how many workgroups (stream-K vs data-parallel grids).

Run under rocprofv3 --kernel-trace (tools/sk_probe.sh); this script logs every aten GEMM of ONE
training step in dispatch order (TorchDispatchMode also sees the autograd backward), brackets the
step with torch.cuda._sleep markers (spin kernels), and writes the log as JSON.
tools/sk_probe_report.py joins the log with the kernel trace.

By default the towers run on one stream (concurrent_towers off) and the kernel <-> call map is by
order; with --concurrent the text tower runs on its side stream and the report matches kernels to
calls per stream (HIP queue <-> logged stream, in order within each).
"""
import argparse
import json
import os
import sys
from types import SimpleNamespace

import torch
from torch.utils._python_dispatch import TorchDispatchMode

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
ap.add_argument("--out", default="gpurun_out/sk_probe_calls.json")
ap.add_argument("--no-tuning", action="store_true")
ap.add_argument("--concurrent", action="store_true", help="text tower on the side stream (ClipModel default)")
args = ap.parse_args()

GEMM_OPS = {"mm", "addmm", "bmm", "baddbmm", "addmm_", "_scaled_mm", "mm.out", "bmm.out", "addmm.out",
            "_addmm_activation", "linear"}


class GemmLog(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.calls = []

    def __torch_dispatch__(self, func, types, args_=(), kwargs=None):
        name = func.overloadpacket.__name__
        if name in GEMM_OPS or name.rstrip("_") in GEMM_OPS:
            ts = [a for a in args_ if isinstance(a, torch.Tensor)]
            self.calls.append({"op": str(func.__name__),
                               "shapes": [list(t.shape) for t in ts],
                               "strides": [list(t.stride()) for t in ts],
                               "dtypes": [str(t.dtype) for t in ts],
                               "kwargs": {k: str(v) for k, v in (kwargs or {}).items()},
                               "stream": torch.cuda.current_stream().cuda_stream})
        return func(*args_, **(kwargs or {}))


targs = SimpleNamespace(precision="amp_bf16", lr=5e-4, wd=0.2, beta1=0.9, beta2=0.98, eps=1e-6,
                        grad_clip_norm=None, accum_freq=1, rank=0, world_size=1, distributed=False)
tuned = False if args.no_tuning else load_gemm_tuning()
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = build_clip(args.model).to(dev)
model.concurrent_towers = args.concurrent
opt = create_optimizer(model, targs)
loss = ClipLoss()
images, texts, targets = synthetic_batch(args.batch, 224, model.text.context_length, model.text.vocab_size,
                                         device=dev, seed=1000)
for _ in range(2):
    train_step(model, images, texts, targets, loss, opt, None, targs)
torch.cuda.synchronize()
log = GemmLog()
torch.cuda._sleep(100000)          # marker: step start
with log:
    train_step(model, images, texts, targets, loss, opt, None, targs)
torch.cuda._sleep(100000)          # marker: step end
torch.cuda.synchronize()
os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
json.dump({"model": args.model, "batch": args.batch, "tuned": tuned, "concurrent": args.concurrent,
           "env": {k: v for k, v in os.environ.items() if k.startswith(("TENSILE", "HIPBLASLT", "ROCBLAS"))},
           "calls": log.calls}, open(args.out, "w"), indent=1)
print(f"{len(log.calls)} GEMM calls logged -> {args.out}", flush=True)
