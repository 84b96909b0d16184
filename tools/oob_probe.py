#!/usr/bin/env python3
"""Out-of-bounds writes by ANY kernel of the two-stream training step: every device
allocation of the process comes from tools/libguard_alloc.so (a pluggable allocator with 256 KB guard
bands checked on free, on the freeing stream), the C2 step runs --steps times with the towers on two
streams, and every changed guard byte is reported with the block size and offset.  Also reports
whether the run-to-run determinism holds under this allocator."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
import torch  # noqa: E402

SO = os.path.join(ROOT, "tools", "libguard_alloc.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vit_b16-mamba130m")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--side-tower", default=None)
    args = ap.parse_args()
    alloc = torch.cuda.memory.CUDAPluggableAllocator(SO, "guard_malloc", "guard_free")
    torch.cuda.memory.change_current_allocator(alloc)
    lib = ctypes.CDLL(SO)
    lib.guard_report.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    lib.guard_check_live.argtypes = [ctypes.c_void_p]
    if args.side_tower:
        os.environ["MAMBA_CLIP_AMD_SIDE_TOWER"] = args.side_tower
    from types import SimpleNamespace
    from mamba_clip_amd import train
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.loss import ClipLoss
    from mamba_clip_amd.model import build_clip
    from mamba_clip_amd.tuning import load_gemm_tuning
    dev = torch.device("cuda", 0)
    load_gemm_tuning(model=args.model)
    torch.manual_seed(0)
    model = build_clip(args.model).to(dev)
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    images, texts, _ = synthetic_batch(args.batch, 224, model.text.context_length, model.text.vocab_size,
                                       device=dev, seed=1000)
    targs = SimpleNamespace(precision="amp_bf16", lr=5e-4, wd=0.2, beta1=0.9, beta2=0.98, eps=1e-6,
                            grad_clip_norm=None, accum_freq=1)
    loss_fn = ClipLoss()
    finals = []
    for rep in range(3):
        model.load_state_dict(init)
        opt = train.create_optimizer(model, targs)
        for s in range(args.steps):
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(images, texts)
                total = loss_fn(**out)["contrastive_loss"]
            total.backward()
            train.optimizer_step(model, opt, None, targs)
            del out, total
        torch.cuda.synchronize()
        finals.append([p.detach().clone() for p in model.parameters()])
        del opt
    lib.guard_check_live(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (3 * 64))()
    n = lib.guard_report(buf, 64)
    bad = [{"block_bytes": buf[3 * i], "side": "high" if buf[3 * i + 1] >> 32 else "low",
            "first_bad_word": buf[3 * i + 1] & 0xFFFFFFFF, "base": hex(buf[3 * i + 2])} for i in range(min(n, 64))]
    same = [all(torch.equal(a, b) for a, b in zip(finals[0], f)) for f in finals[1:]]
    print(json.dumps({"violations": n, "first": bad[:16], "runs_equal_to_first": same,
                      "side_tower": model.side_tower}), flush=True)


if __name__ == "__main__":
    main()
