#!/usr/bin/env python3
"""Every aten reduction (sum / mean / norm / ...) one C2 training step runs, with its shape and the
mamba_clip_amd frames that issued it (torch's cross-workgroup reductions go wrong beside
concurrent kernels; each of these is a candidate)."""
import os, sys, json, traceback
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
import torch
from torch.utils._python_dispatch import TorchDispatchMode
model_name = sys.argv[1] if len(sys.argv) > 1 else "vit_b16-mamba130m"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 256
from mamba_clip_amd.data import synthetic_batch
from mamba_clip_amd.loss import ClipLoss
from mamba_clip_amd.model import build_clip
dev = torch.device("cuda", 0)
model = build_clip(model_name).to(dev)
images, texts, _ = synthetic_batch(batch, 224, model.text.context_length, model.text.vocab_size, device=dev, seed=1000)
RED = ("sum", "mean", "norm", "linalg_vector_norm", "amax", "amin", "max", "min", "prod", "var", "std", "all", "any",
       "cumsum", "embedding_dense_backward", "_embedding_bag_backward", "index_add", "index_put", "scatter_add", "sort",
       "unique", "nonzero", "_foreach_norm")
seen = {}
class M(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, a=(), kw=None):
        name = func.__name__.split(".")[0]
        if name in RED or name.startswith("_foreach_norm"):
            node = torch._C._current_autograd_node()
            fr = [f"{os.path.basename(f.filename)}:{f.lineno}" for f in traceback.extract_stack() if "mamba_clip_amd" in f.filename or "torch/nn" in f.filename][-3:]
            shp = [tuple(t.shape) for t in a if isinstance(t, torch.Tensor)][:2]
            k = (str(func), str(shp), node.name() if node is not None else "fwd", tuple(fr))
            seen[k] = seen.get(k, 0) + 1
        return func(*a, **(kw or {}))
for s in range(2):
    model.zero_grad(set_to_none=True)
    ctx = M() if s == 1 else None
    if ctx: ctx.__enter__()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = model(images, texts)
        loss = ClipLoss()(**out)["contrastive_loss"]
    loss.backward()
    if ctx: ctx.__exit__(None, None, None)
    torch.cuda.synchronize()
for k, v in seen.items():
    print(v, json.dumps(k))
