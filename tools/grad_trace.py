#!/usr/bin/env python3
"""Where does a two-stream backward first diverge from run to run?  

Runs forward + ClipLoss + backward of the C2 model --repeats times from identical state with the
towers on two streams.  During backward a TorchDispatchMode enqueues, right before and right after
every aten op, a checksum (fp64 sum and abs-sum) of each tensor argument and output on the op's own
stream -- so each checksum sees the tensor exactly as that op read or wrote it.  The dispatch order
of the single-threaded autograd engine is the same in every run; the report lists, per run, the
first entries whose checksum differs from run 0: op, autograd node, stream, in/out, shape.  An
input that differs while the op that wrote it matched means the memory changed in between (a
cross-stream hazard); an output that differs with identical inputs means a nondeterministic op."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402
from torch.utils._pytree import tree_flatten  # noqa: E402


class Trace(TorchDispatchMode):
    def __init__(self, names, skip_small):
        super().__init__()
        self.names, self.skip_small = names, skip_small
        self.rec = []

    def _sum(self, func, kind, flat, cur):
        node = torch._C._current_autograd_node()
        for i, t in enumerate(flat):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.numel() >= self.skip_small
                    and (t.is_floating_point())):
                continue
            with torch.no_grad():
                v = t.detach().double()
                s = torch.stack([v.sum(), v.abs().sum()])
            self.rec.append((str(func).replace("aten.", ""), node.name() if node is not None else "-",
                             self.names.get(cur, hex(cur)), kind, i, tuple(t.shape), s))

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in (torch.ops.aten.record_stream.default,) or "view" in str(func) or "detach" in str(func):
            return func(*args, **kwargs)
        cur = torch.cuda.current_stream().cuda_stream
        self._sum(func, "in", tree_flatten((args, kwargs))[0], cur)
        out = func(*args, **kwargs)
        self._sum(func, "out", tree_flatten(out)[0], cur)
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vit_b16-mamba130m")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--repeats", type=int, default=6)
    ap.add_argument("--side-tower", default=None, choices=[None, "image", "text"])
    ap.add_argument("--show", type=int, default=8)
    ap.add_argument("--skip-small", type=int, default=1)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if args.side_tower:
        os.environ["MAMBA_CLIP_AMD_SIDE_TOWER"] = args.side_tower
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.loss import ClipLoss
    from mamba_clip_amd.model import build_clip
    from mamba_clip_amd.tuning import load_gemm_tuning

    dev = torch.device("cuda", 0)
    load_gemm_tuning(model=args.model)
    torch.manual_seed(0)
    model = build_clip(args.model).to(dev)
    images, texts, _ = synthetic_batch(args.batch, 224, model.text.context_length, model.text.vocab_size,
                                       device=dev, seed=1000)
    loss_fn = ClipLoss()
    side = model.side_stream_for(dev)
    names = {torch.cuda.current_stream().cuda_stream: "main", side.cuda_stream: "side"}
    pnames = [n for n, _ in model.named_parameters()]

    def run(trace):
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(images, texts)
            loss = loss_fn(**out)["contrastive_loss"]
        if trace is not None:
            with trace:
                loss.backward()
        else:
            loss.backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
        return grads

    run(None)     # warm-up (plans, transposed-copy registration)
    ref_t = Trace(names, args.skip_small)
    ref_g = run(ref_t)
    ref = [(r[:6], r[6].cpu()) for r in ref_t.rec]
    report = {"side_tower": model.side_tower, "n_entries": len(ref), "runs": []}
    print(json.dumps({"side_tower": model.side_tower, "entries": len(ref)}), flush=True)
    for rep in range(1, args.repeats):
        t = Trace(names, args.skip_small)
        g = run(t)
        cur = [(r[:6], r[6].cpu()) for r in t.rec]
        line = {"repeat": rep, "entries": len(cur),
                "grads_differ": [n for n in pnames if n in ref_g and not torch.equal(ref_g[n], g[n])][:6]}
        diffs = []
        if len(cur) == len(ref):
            for j, ((ka, sa), (kb, sb)) in enumerate(zip(ref, cur)):
                if ka != kb:
                    diffs.append({"idx": j, "structure_differs": [list(map(str, ka)), list(map(str, kb))]})
                    break
                if not torch.equal(sa, sb):
                    diffs.append({"idx": j, "op": ka[0], "node": ka[1], "stream": ka[2], "kind": ka[3], "arg": ka[4],
                                  "shape": list(ka[5]), "ref": [float(x) for x in sa], "got": [float(x) for x in sb]})
                    if len(diffs) >= args.show:
                        break
        line["first_diffs"] = diffs
        if diffs and "idx" in diffs[0]:
            j0 = diffs[0]["idx"]
            line["context_before"] = [{"idx": k, "op": ref[k][0][0], "node": ref[k][0][1], "stream": ref[k][0][2],
                                       "kind": ref[k][0][3], "shape": list(ref[k][0][5])}
                                      for k in range(max(0, j0 - 6), j0)]
        report["runs"].append(line)
        print(json.dumps(line), flush=True)
    if args.out:
        json.dump(report, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
