#!/usr/bin/env python3
"""Does any kernel of the training step read LDS it never wrote?  

One stream, deterministic.  The C2 model steps twice from identical state (forward, ClipLoss,
backward):
  run A: as is;
  run B: before every aten op and every mc_* library call, tools/liblds_poison.so fills the LDS of
         every CU with 0xFFFFFFFF (NaN in fp32 / bf16 / fp16) on the current stream.
A TorchDispatchMode checksums (fp64 sum, abs-sum) every floating-point input and output of every aten
op in both runs.  A kernel that consumes LDS left over by an earlier kernel reads NaN in run B; the
first entry whose checksum differs between A and B names the op that saw it (for an input: the
library call logged just before it wrote the tensor).  Two-stream runs are nondeterministic exactly
when such leftovers depend on which kernel of the other stream ran on the CU before."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402
from torch.utils._pytree import tree_flatten  # noqa: E402

POISON = ctypes.CDLL(os.path.join(ROOT, "tools", "liblds_poison.so"))
POISON.lds_poison.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
POISON.lds_poison.restype = ctypes.c_int


def poison():
    rc = POISON.lds_poison(0xFFFFFFFF, 2048, torch.cuda.current_stream().cuda_stream)
    if rc:
        raise RuntimeError(f"lds_poison failed ({rc})")


class Trace(TorchDispatchMode):
    def __init__(self, do_poison):
        super().__init__()
        self.do_poison = do_poison
        self.rec = []
        self.last_lib = None

    def _sum(self, func, kind, flat):
        node = torch._C._current_autograd_node()
        for i, t in enumerate(flat):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.is_floating_point() and t.numel()):
                continue
            with torch.no_grad():
                v = t.detach().double()
                s = torch.stack([v.sum(), v.abs().sum()])
            self.rec.append((str(func).replace("aten.", ""), node.name() if node is not None else "fwd", kind, i,
                             tuple(t.shape), self.last_lib, s))

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = str(func)
        if "empty" in name or "view" in name or "detach" in name or "record_stream" in name or "slice" in name \
                or "transpose" in name or name.endswith(".t.default") or "as_strided" in name or "split" in name \
                or "unsqueeze" in name or "squeeze" in name or "expand" in name or "permute" in name \
                or "select" in name or "alias" in name or "_reshape" in name:
            return func(*args, **kwargs)
        self._sum(func, "in", tree_flatten((args, kwargs))[0])
        if self.do_poison:
            poison()
        out = func(*args, **kwargs)
        self._sum(func, "out", tree_flatten(out)[0])
        return out


class LibProxy:
    def __init__(self, lib, holder):
        self._lib, self._holder = lib, holder

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        if not callable(fn) or not name.startswith("mc_") or name.endswith("_bytes") or name == "mc_last_error":
            return fn
        holder = self._holder

        def call(*args):
            t = holder.get("trace")
            if t is not None:
                t.last_lib = name
                if t.do_poison:
                    poison()
            return fn(*args)
        return call


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vit_b16-mamba130m")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--show", type=int, default=12)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from mamba_clip_amd import _lib
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.loss import ClipLoss
    from mamba_clip_amd.model import build_clip

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = build_clip(args.model).to(dev)
    model.concurrent_towers = False
    images, texts, _ = synthetic_batch(args.batch, 224, model.text.context_length, model.text.vocab_size,
                                       device=dev, seed=1000)
    loss_fn = ClipLoss()
    holder = {}
    _lib._lib = LibProxy(_lib.load(), holder)

    def run(trace):
        model.zero_grad(set_to_none=True)
        holder["trace"] = trace
        with trace:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(images, texts)
                loss = loss_fn(**out)["contrastive_loss"]
            loss.backward()
        holder["trace"] = None
        torch.cuda.synchronize()
        return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}

    run(Trace(False))                       # warm-up (plans, registrations)
    ta, tb, tc = Trace(False), Trace(True), Trace(False)
    ga, gb, gc = run(ta), run(tb), run(tc)
    names = [n for n, _ in model.named_parameters()]
    rep = {"entries": [len(ta.rec), len(tb.rec), len(tc.rec)],
           "grads_differ_poisoned": [n for n in names if n in ga and not torch.equal(ga[n], gb[n])][:20],
           "grads_nonfinite_poisoned": [n for n in names if n in gb and not bool(torch.isfinite(gb[n]).all())][:20],
           "grads_differ_repeat": [n for n in names if n in ga and not torch.equal(ga[n], gc[n])][:20]}

    def diffs(x, y):
        out = []
        for j, (ra, rb) in enumerate(zip(x.rec, y.rec)):
            if ra[:5] != rb[:5]:
                out.append({"idx": j, "structure": [list(map(str, ra[:6])), list(map(str, rb[:6]))]})
                break
            if not torch.equal(ra[6].cpu(), rb[6].cpu()):
                out.append({"idx": j, "op": ra[0], "node": ra[1], "kind": ra[2], "arg": ra[3], "shape": list(ra[4]),
                            "last_lib_call": ra[5], "ref": [float(v) for v in ra[6]], "got": [float(v) for v in rb[6]]})
                if len(out) >= args.show:
                    break
        return out
    rep["first_diffs_poisoned"] = diffs(ta, tb)
    rep["first_diffs_repeat"] = diffs(ta, tc)
    print(json.dumps(rep, indent=1), flush=True)
    if args.out:
        json.dump(rep, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
