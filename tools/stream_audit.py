#!/usr/bin/env python3
"""Which tensors does an op read or write on a stream other than the one whose pool their memory
came from?  (the two-stream C2 step is run-to-run nondeterministic, and with
PYTORCH_NO_CUDA_MEMORY_CACHING=1 it is not -- an allocator-reuse hazard, a block used on a second
stream without record_stream.)

A TorchDispatchMode sees every aten op of one training step (forward, ClipLoss, backward; the
autograd engine carries the mode into its device thread).  For each tensor argument and output it
looks up the caching-allocator segment holding the data pointer (torch.cuda.memory._snapshot();
a segment belongs to one stream's pool) and reports the uses whose current stream differs from the
segment's stream: op, argument, shape, both streams, the autograd node running (backward) and the
innermost mamba_clip_amd frames.  Legitimate cross-stream uses (the inputs and the side tower's
features, which model.py hands over with record_stream) show up too and are listed as such."""
import argparse
import collections
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402
from torch.utils._pytree import tree_flatten  # noqa: E402


class Segments:
    def __init__(self):
        self.segs = []

    def refresh(self):
        self.segs = sorted((s["address"], s["address"] + s["total_size"], s["stream"])
                           for s in torch.cuda.memory._snapshot()["segments"])

    def stream_of(self, ptr, refresh=True):
        for _ in range(2 if refresh else 1):
            lo, hi = 0, len(self.segs)
            while lo < hi:
                mid = (lo + hi) // 2
                if self.segs[mid][1] <= ptr:
                    lo = mid + 1
                else:
                    hi = mid
            if lo < len(self.segs) and self.segs[lo][0] <= ptr < self.segs[lo][1]:
                return self.segs[lo][2]
            if refresh:
                self.refresh()
        return None


def _ints(v, depth=0):
    """Integer values (candidate device pointers) in a ctypes argument: plain ints, c_void_p, and the
    fields of parameter structs passed by pointer or byref."""
    import ctypes
    if depth > 3 or v is None:
        return
    if isinstance(v, int):
        yield v
    elif isinstance(v, ctypes._SimpleCData):
        if isinstance(v.value, int):
            yield v.value
    elif isinstance(v, ctypes.Structure):
        for f in v._fields_:
            yield from _ints(getattr(v, f[0]), depth + 1)
    elif isinstance(v, ctypes.Array):
        for x in v:
            yield from _ints(x, depth + 1)
    elif hasattr(v, "_obj"):                       # byref(...)
        yield from _ints(v._obj, depth + 1)
    elif isinstance(v, ctypes._Pointer):
        try:
            yield from _ints(v.contents, depth + 1)
        except ValueError:
            pass


class LibProxy:
    """Stands in for the loaded CDLL: every mc_* call is checked like an aten op (its pointers'
    segments against the current stream) before it runs."""

    def __init__(self, lib, audit):
        self._lib, self._audit = lib, audit

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        if not callable(fn) or not name.startswith("mc_") or name.endswith("_bytes") or name == "mc_last_error":
            return fn
        audit = self._audit

        def call(*args):
            if audit.active:
                cur = torch.cuda.current_stream().cuda_stream
                for i, a in enumerate(args):
                    for v in _ints(a):
                        if v > (1 << 32):
                            audit.check_ptr(name, i, v, cur)
            return fn(*args)
        return call


class Audit(TorchDispatchMode):
    def __init__(self, segs, names):
        super().__init__()
        self.segs, self.names = segs, names
        self.hits = collections.OrderedDict()
        self.active = False

    def __enter__(self):
        self.active = True
        return super().__enter__()

    def __exit__(self, *a):
        self.active = False
        return super().__exit__(*a)

    def check_ptr(self, name, i, ptr, cur):
        s = self.segs.stream_of(ptr, refresh=False)
        if s is None or s == cur:
            return
        node = torch._C._current_autograd_node()
        frames = [f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in traceback.extract_stack()
                  if "mamba_clip_amd" in f.filename][-3:]
        key = (name, "ptr", i, node.name() if node is not None else "fwd", tuple(frames))
        e = self.hits.get(key)
        if e is None:
            self.hits[key] = {"op": name, "kind": "hip-arg", "arg": i, "seg_stream": self.names.get(s, hex(s)),
                              "cur_stream": self.names.get(cur, hex(cur)), "node": key[3], "frames": list(frames),
                              "count": 1}
        else:
            e["count"] += 1

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        cur = torch.cuda.current_stream().cuda_stream
        self._check(func, "in", tree_flatten((args, kwargs))[0], cur)
        out = func(*args, **kwargs)
        self._check(func, "out", tree_flatten(out)[0], cur)
        return out

    def _check(self, func, kind, flat, cur):
        for i, t in enumerate(flat):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.numel()):
                continue
            s = self.segs.stream_of(t.untyped_storage().data_ptr())
            if s is None or s == cur:
                continue
            node = torch._C._current_autograd_node()
            frames = [f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in traceback.extract_stack()
                      if "mamba_clip_amd" in f.filename][-3:]
            key = (str(func), kind, i, tuple(t.shape), node.name() if node is not None else "fwd", tuple(frames))
            e = self.hits.get(key)
            if e is None:
                self.hits[key] = {"op": str(func), "kind": kind, "arg": i, "shape": list(t.shape),
                                  "dtype": str(t.dtype), "seg_stream": self.names.get(s, hex(s)),
                                  "cur_stream": self.names.get(cur, hex(cur)),
                                  "node": key[4], "frames": list(frames), "count": 1}
            else:
                e["count"] += 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vit_b16-mamba130m")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--side-tower", default=None, choices=[None, "image", "text"])
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if args.side_tower:
        os.environ["MAMBA_CLIP_AMD_SIDE_TOWER"] = args.side_tower
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.loss import ClipLoss
    from mamba_clip_amd.model import build_clip

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = build_clip(args.model).to(dev)
    images, texts, _ = synthetic_batch(args.batch, 224, model.text.context_length, model.text.vocab_size,
                                       device=dev, seed=1000)
    loss_fn = ClipLoss()
    side = model.side_stream_for(dev)
    names = {torch.cuda.current_stream().cuda_stream: "main", side.cuda_stream: "side"}

    def step():
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(images, texts)
            loss = loss_fn(**out)["contrastive_loss"]
        loss.backward()

    step()       # warm-up: plans, transposed-copy registration, library handles
    torch.cuda.synchronize()
    segs = Segments()
    segs.refresh()
    audit = Audit(segs, names)
    from mamba_clip_amd import _lib
    _lib._lib = LibProxy(_lib.load(), audit)
    with audit:
        step()
    torch.cuda.synchronize()
    hits = list(audit.hits.values())
    for h in hits:
        print(json.dumps(h), flush=True)
    print(json.dumps({"distinct_cross_stream_uses": len(hits), "side_tower": model.side_tower}), flush=True)
    if args.out:
        json.dump(hits, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
