#!/usr/bin/env python3
"""Is one Mamba layer's backward a function of its inputs alone while the other tower runs on a second
stream?    Per iteration: new input and output-gradient data; the C2 MambaLayer (bf16
autocast, channel-major mixer) runs forward + backward on the main stream while the side stream runs a
ViT-B/16 block forward + backward (library GEMMs, fused attention, LayerNorm / GELU kernels, torch
reductions); then the same layer step runs again with the device idle and every gradient (input and
parameters) is compared bitwise.  A mismatch names the gradients that differ and by how much."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--loads", default="none,vit_block")
    args = ap.parse_args()
    from mamba_clip_amd.model import MambaLayer, ViTBlock
    from mamba_clip_amd.tuning import load_gemm_tuning
    load_gemm_tuning(model="vit_b16-mamba130m")
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    layer = MambaLayer(768).to(dev)
    blk = ViTBlock(768, 12).to(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    B, L = 256, 80
    hid = torch.empty(B, L, 768, device=dev)
    res = torch.empty(B, L, 768, device=dev)
    gy = torch.empty(B, L, 768, device=dev)
    gr = torch.empty(B, L, 768, device=dev)
    vx = torch.randn(256, 197, 768, device=dev, generator=g)
    side = torch.cuda.Stream()
    names = ["hidden", "residual"] + [n for n, _ in layer.named_parameters()]

    def step():
        layer.zero_grad(set_to_none=True)
        h = hid.detach().to(torch.bfloat16).requires_grad_(True)
        r = res.detach().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out, r2 = layer(h, r)
        torch.autograd.backward([out, r2], [gy.to(out.dtype), gr])
        return [h.grad.clone(), r.grad.clone()] + [p.grad.clone() for _, p in layer.named_parameters()]

    def vit_load():
        x = vx.detach().to(torch.bfloat16).requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            m, h = blk(x, None)
            m, h = blk(m, h)
            loss = (m.float().sum() + h.float().sum()) * 1e-3
        loss.backward()
        # the pos_embed-style batch sum (torch reduce with a cross-workgroup combine)
        x.grad.sum(0, keepdim=True)

    for load in args.loads.split(","):
        bad, detail = 0, {}
        for it in range(args.iters):
            for t in (hid, res, gy, gr):
                t.normal_(generator=g)
            if load != "none":
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    vit_load()
            got = step()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            again = step()
            torch.cuda.synchronize()
            diff = [n for n, a, b in zip(names, got, again) if not torch.equal(a, b)]
            if diff:
                bad += 1
                for n, a, b in zip(names, got, again):
                    if n in diff:
                        d = (a.float() - b.float()).abs()
                        detail.setdefault(n, []).append((int((d > 0).sum()), float(d.max())))
        print(json.dumps({"load": load, "iters": args.iters, "iters_differ": bad,
                          "which": {k: v[:3] for k, v in detail.items()}}), flush=True)


if __name__ == "__main__":
    main()
