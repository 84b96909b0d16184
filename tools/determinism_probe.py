#!/usr/bin/env python3
"""Run-to-run determinism of the training step, variant by variant.

One process builds the C2 model once, then for each variant and repeat restores the initial
parameters, builds a fresh optimizer and runs --steps optimizer steps on the same resident batch.
Repeat 0 of the first variant is the reference; every later run reports, bitwise:
  - step-1 image / text features and loss,
  - step-1 gradients (first differing parameter names per tower),
  - final parameters.
Variants (comma list, --variants):
  conc      towers on two streams (the default path)
  seq       one stream
  conc_sync two streams, device synchronize after forward and after backward
  conc_fsync two streams, device synchronize after forward only
  conc_torchadam  two streams, torch's fused AdamW instead of HipAdamW
  conc_text two streams, text tower on the side stream
  conc_nowt two streams, no transposed weight copies (ops.WCAST_T off)
Run once as is and once with PYTORCH_NO_CUDA_MEMORY_CACHING=1 to separate allocator-reuse hazards
(a missing record_stream) from ordering hazards (a missing wait)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vit_b16-mamba130m")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--variants", default="conc,seq,conc_sync,conc_torchadam,conc_text,conc_nowt")
    ap.add_argument("--out", default=None)
    ap.add_argument("--compare", choices=["first", "prev"], default="first",
                    help="compare each run with the first run overall, or with the previous run of its variant")
    ap.add_argument("--summary", action="store_true",
                    help="compare every run with one seq run: per variant, how many of --repeats runs differ "
                         "(step-1 grads, final params, losses) and their first differing grads in backward order")
    ap.add_argument("--self-ref", action="store_true",
                    help="with --summary: compare each variant's runs with an extra first run of that variant")
    ap.add_argument("--isolate", default="",
                    help="comma list of mc_* library calls to run alone on the device: a device synchronize before "
                         "and after each such call (is that kernel a victim or an aggressor of the two-stream race?)")
    ap.add_argument("--isolate-aten", default="",
                    help="comma list of aten op name prefixes (sum, mm, bmm, addmm, ...) to run alone on the device")
    ap.add_argument("--pre-sync", default="none", choices=["none", "other", "current", "device", "other_event", "clone_bias", "clone_D", "clone_A"],
                    help="before each scan backward: host-wait for the other stream / this stream / the device, or "
                         "make this stream wait (event) for the other stream's work so far")
    ap.add_argument("--fill-nan", action="store_true",
                    help="torch.use_deterministic_algorithms(warn_only) + fill_uninitialized_memory: every torch.empty "
                         "is NaN-filled, so a kernel reading memory it never wrote shows up")
    args = ap.parse_args()
    if args.fill_nan:
        torch.use_deterministic_algorithms(True, warn_only=True)
        torch.utils.deterministic.fill_uninitialized_memory = True

    from types import SimpleNamespace
    from mamba_clip_amd import ops, train
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.loss import ClipLoss
    from mamba_clip_amd.model import ClipModel, build_clip
    from mamba_clip_amd.tuning import load_gemm_tuning
    from mamba_clip_amd.utils.amp_utils import get_autocast

    dev = torch.device("cuda", 0)
    load_gemm_tuning(model=args.model)
    if args.isolate:
        from mamba_clip_amd import _lib
        iso = set(args.isolate.split(","))

        class _Iso:
            def __init__(self, lib):
                self._lib = lib

            def __getattr__(self, name):
                fn = getattr(self._lib, name)
                if name not in iso:
                    return fn

                def call(*a):
                    torch.cuda.synchronize()
                    rc = fn(*a)
                    torch.cuda.synchronize()
                    return rc
                return call
        _lib._lib = _Iso(_lib.load())
    targs = SimpleNamespace(precision="amp_bf16", lr=5e-4, wd=0.2, beta1=0.9, beta2=0.98, eps=1e-6,
                            grad_clip_norm=None, accum_freq=1)
    torch.manual_seed(0)
    model = build_clip(args.model).to(dev)
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    images, texts, targets = synthetic_batch(args.batch, 224, model.text.context_length, model.text.vocab_size,
                                             device=dev, seed=1000)
    loss_fn = ClipLoss()
    autocast = get_autocast(targs.precision)
    names = [n for n, _ in model.named_parameters()]
    img_names = {n for n in names if n.startswith("visual.")}

    iso_mode = None
    if args.isolate_aten:
        from torch.utils._python_dispatch import TorchDispatchMode
        pref = tuple(args.isolate_aten.split(","))

        class _IsoAten(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, a=(), kw=None):
                name = func.__name__.split(".")[0]
                if name in pref:
                    torch.cuda.synchronize()
                    out = func(*a, **(kw or {}))
                    torch.cuda.synchronize()
                    return out
                return func(*a, **(kw or {}))
        iso_mode = _IsoAten()

    nn_stream = torch.cuda.Stream(device=dev)
    if args.pre_sync != "none":
        from mamba_clip_amd import selective_scan_interface as ssi
        real_bwd = ssi.scan_bwd
        default = torch.cuda.default_stream(dev)

        def wrapped(*a, **k):
            cur = torch.cuda.current_stream(dev)
            other = model.side_stream_for(dev) if cur == default else default
            if args.pre_sync == "other":
                other.synchronize()
            elif args.pre_sync == "current":
                cur.synchronize()
            elif args.pre_sync == "device":
                torch.cuda.synchronize()
            elif args.pre_sync == "other_event":
                cur.wait_stream(other)
            elif args.pre_sync.startswith("clone_"):   # scan_bwd(u, delta, A, B, C, D, z, delta_bias, ...)
                a = list(a)
                j = {"clone_bias": 7, "clone_D": 5, "clone_A": 2}[args.pre_sync]
                a[j] = a[j].clone()
            return real_bwd(*a, **k)
        ssi.scan_bwd = wrapped

    def run(variant):
        if variant.endswith("_nn"):   # the whole step on a non-default stream (not HIP's null stream)
            cur = torch.cuda.current_stream()
            nn_stream.wait_stream(cur)
            with torch.cuda.stream(nn_stream):
                rec = run_(variant[:-3])
            cur.wait_stream(nn_stream)
            torch.cuda.synchronize()
            return rec
        if iso_mode is not None:
            with iso_mode:
                return run_(variant)
        return run_(variant)

    def run_(variant):
        model.load_state_dict(init)
        model.zero_grad(set_to_none=True)
        model.concurrent_towers = not variant.startswith("seq")
        os.environ.pop("MAMBA_CLIP_AMD_SIDE_TOWER", None)
        os.environ.pop("MAMBA_CLIP_AMD_FINE_STATES_MB", None)
        if variant.startswith("conc_text"):
            os.environ["MAMBA_CLIP_AMD_SIDE_TOWER"] = "text"
        elif variant.startswith("conc_image"):
            os.environ["MAMBA_CLIP_AMD_SIDE_TOWER"] = "image"
        if variant.endswith("_nofine"):
            os.environ["MAMBA_CLIP_AMD_FINE_STATES_MB"] = "0"
        for m in model.modules():
            if hasattr(m, "fused_attention"):
                m.fused_attention = not variant.endswith("_noattn")
        ops.WGRAD_HIP = variant.endswith("_wgradhip")
        torch.backends.cuda.preferred_blas_library("cublas" if variant.endswith("_rocblas") else "cublaslt")
        ops.WCAST_T = variant != "conc_nowt"
        ClipModel.shared_weight_casts = variant.endswith("_sharedcast")
        hip = train.HIP_ADAMW
        train.HIP_ADAMW = variant != "conc_torchadam"
        opt = train.create_optimizer(model, targs)
        train.HIP_ADAMW = hip
        rec = {}
        losses = []
        from mamba_clip_amd import selective_scan_interface as ssi
        rec["fine_live_mb"] = []
        for s in range(args.steps):
            opt.zero_grad(set_to_none=True)
            live0 = 0
            with autocast():
                out = model(images, texts)
            rec["fine_live_mb"].append((0, 0))
            if variant in ("conc_sync", "conc_fsync"):
                torch.cuda.synchronize()
            with autocast():
                total = loss_fn(**out)["contrastive_loss"]
            total.backward()
            if variant == "conc_sync":
                torch.cuda.synchronize()
            if s == 0:
                rec["img_f"] = out["image_features"].detach().clone()
                rec["txt_f"] = out["text_features"].detach().clone()
                rec["grads"] = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
            losses.append(total.detach().clone())
            train.optimizer_step(model, opt, None, targs)
            del out, total
        torch.cuda.synchronize()
        rec["loss"] = [float(x) for x in losses]
        rec["params"] = {n: p.detach().clone() for n, p in model.named_parameters()}

        def fp(t):   # exact fingerprint of a tensor's bits
            b = t.detach().contiguous().view(-1)
            b = b.view(torch.int16).to(torch.int64) if b.element_size() == 2 else b.view(torch.int32).to(torch.int64)
            w = torch.arange(1, b.numel() + 1, device=b.device, dtype=torch.int64) % 1000003
            return int((b * w).sum())
        rec["fp_grads"] = hash(tuple(fp(v) for v in rec["grads"].values()))
        rec["fingerprint"] = hash((rec["fp_grads"], tuple(fp(v) for v in rec["params"].values())))
        del opt
        return rec

    def diff(a, b):
        d = {"img_f_equal": torch.equal(a["img_f"], b["img_f"]), "txt_f_equal": torch.equal(a["txt_f"], b["txt_f"]),
             "loss": [x.hex() for x in b["loss"]], "loss_equal": a["loss"] == b["loss"]}
        bad = [n for n in names if n in a["grads"] and not torch.equal(a["grads"][n], b["grads"][n])]
        d["grads_differ"] = len(bad)
        d["grads_differ_image"] = [n for n in bad if n in img_names][:6]
        d["grads_differ_text"] = [n for n in bad if n not in img_names][:6]
        d["grads_differ_last_img"] = [n for n in bad if n in img_names][-3:]
        d["grads_differ_last_txt"] = [n for n in bad if n not in img_names][-3:]
        pb = [n for n in names if not torch.equal(a["params"][n], b["params"][n])]
        d["params_differ"] = len(pb)
        if bad:
            n = bad[0]
            d["first_grad_maxdiff"] = float((a["grads"][n].float() - b["grads"][n].float()).abs().max())
        return d

    order = list(reversed(names))    # roughly backward order within each tower
    if args.summary:
        ref = run("seq")
        summ = {}
        for variant in args.variants.split(","):
            bad_runs, firsts, t0 = 0, {}, time.time()
            if args.self_ref:
                run(variant)            # warm-up: a variant switch rebuilds plans / registrations on its first run
                ref = run(variant)
            fps, fpg = [], []
            for r in range(args.repeats):
                rec = run(variant)
                fps.append(rec["fingerprint"])
                fpg.append(rec["fp_grads"])
                bad = [n for n in order if not torch.equal(ref["grads"][n], rec["grads"][n])]
                pbad = sum(1 for n in names if not torch.equal(ref["params"][n], rec["params"][n]))
                if bad or pbad or rec["loss"] != ref["loss"]:
                    pnames = [n for n in order if not torch.equal(ref["params"][n], rec["params"][n])]
                    print(json.dumps({"variant": variant, "repeat": r, "first_bad": bad[:2],
                                      "loss_equal_per_step": [a == b for a, b in zip(ref["loss"], rec["loss"])],
                                      "n_params_differ": len(pnames), "params_differ_first": pnames[:4],
                                      "params_differ_img": sum(1 for n in pnames if n in img_names)}), flush=True)
                    bad_runs += 1
                    key = ",".join(bad[:2]) if bad else "params-only"
                    firsts[key] = firsts.get(key, 0) + 1
            summ[variant] = {"runs": args.repeats, "runs_differ": bad_runs, "first_bad": firsts,
                             "distinct_outcomes": len(set(fps)), "distinct_step1_grads": len(set(fpg)),
                             "ref_step1_grads_seen_again": fpg.count(ref["fp_grads"]),
                             "s": round(time.time() - t0, 1)}
            print(json.dumps({"variant": variant, **summ[variant]}), flush=True)
        if args.out:
            with open(args.out, "w") as f:
                json.dump({"caching": os.environ.get("PYTORCH_NO_CUDA_MEMORY_CACHING", "") == "",
                           "batch": args.batch, "steps": args.steps, "summary": summ}, f, indent=1)
        return
    ref = None
    prev = {}
    report = {"caching": os.environ.get("PYTORCH_NO_CUDA_MEMORY_CACHING", "") == "", "batch": args.batch,
              "steps": args.steps, "runs": []}
    for variant in args.variants.split(","):
        for r in range(args.repeats):
            t0 = time.time()
            rec = run(variant)
            base = ref if args.compare == "first" else prev.get(variant)
            if base is None:
                line = {"variant": variant, "repeat": r, "reference": True, "loss": [x.hex() for x in rec["loss"]]}
            else:
                line = {"variant": variant, "repeat": r, **diff(base, rec)}
                bad = [n for n in order if n in base["grads"] and not torch.equal(base["grads"][n], rec["grads"][n])]
                line["first_bad_grads_bwd_order"] = bad[:4]
            nan = [n for n, g in rec["grads"].items() if not bool(torch.isfinite(g).all())]
            if nan:
                line["nonfinite_grads"] = nan[:6]
            if ref is None:
                ref = rec
            prev[variant] = rec
            line["s"] = round(time.time() - t0, 2)
            report["runs"].append(line)
            print(json.dumps(line), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
