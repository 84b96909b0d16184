#!/usr/bin/env python3
"""Locate run-to-run differences of the two-stream training step down to one kernel call.

Wraps the scan wrappers (selective_scan_interface.scan_fwd / scan_bwd) and records, per call, every
input and output; runs the C2 step (forward + ClipLoss + backward, no optimizer) --repeats times on
identical state and reports, for each run after the first, the first scan call whose INPUTS differ
and the first whose OUTPUTS differ while its inputs are identical (a nondeterministic kernel), plus
the same for the towers' features and parameter gradients.

  --side-load gemm: instead of the image tower, a stream of unrelated library GEMMs runs on a side
  stream while the text tower steps alone on the main stream (is the text tower sensitive to
  concurrency by itself?)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--repeats", type=int, default=4)
    ap.add_argument("--concurrent", type=int, default=1)
    ap.add_argument("--side-load", choices=["none", "gemm"], default="none")
    ap.add_argument("--out", default=None)
    ap.add_argument("--light", action="store_true",
                    help="per scan_bwd call record only fp64 checksums of the inputs (enqueued before the call) "
                         "and the dA / dD / dbias outputs: little extra work, so the timing stays close to the step's")
    ap.add_argument("--watch", action="store_true",
                    help="snapshot every scan_bwd input again right after the call; when one "
                         "changed during the call, report which, and the allocator history of its address range")
    args = ap.parse_args()
    if args.watch:
        torch.cuda.memory._record_memory_history(enabled="all", context="all", stacks="python", max_entries=400000)

    from mamba_clip_amd import selective_scan_interface as ssi
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.loss import ClipLoss
    from mamba_clip_amd.model import build_clip
    from mamba_clip_amd.tuning import load_gemm_tuning

    dev = torch.device("cuda", 0)
    load_gemm_tuning(model="vit_b16-mamba130m")
    torch.manual_seed(0)
    model = build_clip("vit_b16-mamba130m").to(dev)
    model.concurrent_towers = bool(args.concurrent)
    images, texts, _ = synthetic_batch(args.batch, 224, model.text.context_length, model.text.vocab_size,
                                       device=dev, seed=1000)
    gfix = torch.randn(args.batch, 512, device=dev, generator=torch.Generator(device=dev).manual_seed(7))

    calls = []
    real_fwd, real_bwd = ssi.scan_fwd, ssi.scan_bwd

    def snap(x):
        if isinstance(x, torch.Tensor):
            return x.detach().clone()
        if isinstance(x, (tuple, list)):
            return type(x)(snap(v) for v in x)
        return x

    def fwd(*a, **k):
        if args.light:
            return real_fwd(*a, **k)
        out = real_fwd(*a, **k)
        calls.append(("fwd", snap(a), snap(out)))
        return out

    changed = []

    def csum(x):
        if isinstance(x, torch.Tensor) and x.is_floating_point() and x.is_cuda:
            v = x.detach().double()
            return torch.stack([v.sum(), v.abs().sum()])
        return None

    def bwd(*a, **k):
        if args.light:
            ins = tuple(csum(x) for x in a)
            wss = []
            real_empty = torch.empty

            def empty(*sz, **kw):       # catch the workspace (the one uint8 allocation of scan_bwd)
                t = real_empty(*sz, **kw)
                if kw.get("dtype") is torch.uint8:
                    wss.append(t)
                return t
            torch.empty = empty
            try:
                out = real_bwd(*a, **k)
            finally:
                torch.empty = real_empty
            # pair-path workspace (scan_bwd.hip bwd_ws_layout): [bq][slab_bc][slab_a][slab_d][slab_bias], 256-B aligned
            u_, delta_ = a[0], a[1]
            bsz, dim, L = delta_.shape
            al = lambda x: (x + 255) // 256 * 256
            nblk = (dim + 63) // 64
            o_bc = al(bsz * L * 8 * 16)
            o_a = o_bc + al(bsz * nblk * 16 * 2 * L * 4)
            o_d = o_a + al(bsz * dim * 16 * 4)
            o_b = o_d + al(bsz * dim * 4)
            ws = wss[0] if wss else None
            slabs = (ws[o_d:o_d + bsz * dim * 4].clone(), ws[o_b:o_b + bsz * dim * 4].clone()) if ws is not None else ()
            outs = tuple(csum(x) for x in out) + slabs
            calls.append(("bwd", ins, outs + (out[2].clone(), out[7].clone() if out[7] is not None else None)))
            return out
        ins = snap(a)          # the inputs as the kernel will read them (same stream: ordered)
        out = real_bwd(*a, **k)
        calls.append(("bwd", ins, snap(out)))
        if args.watch:
            post = snap(a)     # enqueued right behind the call on the same stream (timing kept)
            for j, (x, y) in enumerate(zip(ins, post)):
                if isinstance(x, torch.Tensor) and not torch.equal(x, y):
                    t = a[j]
                    lo = t.data_ptr()
                    hi = lo + (t.untyped_storage().nbytes() if t.numel() else 0)
                    changed.append({"call": len(calls) - 1, "arg": j, "ptr": lo, "end": hi,
                                    "n_changed": int((x != y).sum()), "shape": list(t.shape)})
        return out

    ssi.scan_fwd, ssi.scan_bwd = fwd, bwd
    side = torch.cuda.Stream()
    ga = torch.randn(8192, 8192, device=dev).bfloat16()

    def run():
        calls.clear()
        model.zero_grad(set_to_none=True)
        stop = None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if args.side_load == "gemm":
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    for _ in range(40):
                        ga @ ga
                f = model.text(texts)
                loss = (f.float() * gfix).sum()
            else:
                out = model(images, texts)
                loss = ClipLoss()(**out)["contrastive_loss"]
        loss.backward()
        torch.cuda.synchronize()
        feats = {"loss": loss.detach().clone()}
        if args.side_load == "none":
            feats["img"], feats["txt"] = out["image_features"].detach().clone(), out["text_features"].detach().clone()
        grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
        return feats, grads, list(calls)

    def eq(a, b):
        if isinstance(a, torch.Tensor):
            return isinstance(b, torch.Tensor) and a.shape == b.shape and torch.equal(a, b)
        if isinstance(a, (tuple, list)):
            return len(a) == len(b) and all(eq(x, y) for x, y in zip(a, b))
        return a == b

    def first_diff_idx(a, b):
        if isinstance(a, (tuple, list)):
            return [i for i, (x, y) in enumerate(zip(a, b)) if not eq(x, y)]
        return None

    def history(lo, hi, keep=25):
        """Allocator events (alloc / free) whose block overlaps [lo, hi): stream, size, top Python frames."""
        snap_ = torch.cuda.memory._snapshot()
        evs = []
        for dev_tr in snap_.get("device_traces", []):
            for e in dev_tr:
                a0, sz = e.get("addr", 0), e.get("size", 0)
                if a0 < hi and a0 + sz > lo:
                    fr = [f"{f.get('filename', '').split('/')[-1]}:{f.get('line')}:{f.get('name')}"
                          for f in (e.get("frames") or [])[:8] if "mamba_clip_amd" in f.get("filename", "")
                          or "race_probe" in f.get("filename", "")]
                    evs.append({"action": e.get("action"), "addr": a0, "size": sz, "stream": e.get("stream"),
                                "frames": fr[:4]})
        return evs[-keep:]

    ref = run()
    changed.clear()
    lines = []
    for r in range(1, args.repeats):
        cur = run()
        d = {"repeat": r, "features_equal": {k: eq(ref[0][k], cur[0][k]) for k in ref[0]},
             "grads_differ": sum(1 for n in ref[1] if not eq(ref[1][n], cur[1][n]))}
        first_in, first_out = None, None
        for i, ((kind, ia, oa), (_, ib, ob)) in enumerate(zip(ref[2], cur[2])):
            ins_eq, outs_eq = eq(ia, ib), eq(oa, ob)
            if not ins_eq and first_in is None:
                first_in = {"call": i, "kind": kind, "input_args_differ": first_diff_idx(ia, ib)}
            if ins_eq and not outs_eq and first_out is None:
                od = first_diff_idx(oa, ob)
                first_out = {"call": i, "kind": kind, "outputs_differ": od,
                             "max_abs": [float((oa[j].float() - ob[j].float()).abs().max()) for j in od
                                         if isinstance(oa[j], torch.Tensor)],
                             "n_elems_differ": [int((oa[j] != ob[j]).sum()) for j in od if isinstance(oa[j], torch.Tensor)]}
        d["first_call_inputs_differ"] = first_in
        d["first_call_outputs_differ_same_inputs"] = first_out
        d["n_calls"] = len(cur[2])
        if args.watch:
            d["inputs_changed_during_call"] = list(changed)
            if changed:
                d["history"] = history(changed[0]["ptr"], changed[0]["end"])
            changed.clear()
        lines.append(d)
        print(json.dumps(d), flush=True)
    if args.out:
        json.dump(lines, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
