#!/usr/bin/env python3
"""Is a reduction's result a function of its input alone while a second stream runs library GEMMs?
  Every iteration draws NEW data (so a stale read of an earlier iteration's partials would
show), reduces it on the main stream while the side stream runs the ViT-shaped GEMMs, then reduces it
again with the device idle; the two results are compared bitwise.  Victims: torch's batch sum of a bf16
(256, 197, 768) tensor (the ViT pos_embed gradient), torch's fp32 column sum, and mc_sum_slabs."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=150)
    ap.add_argument("--loads", default="none,gemm_vit,attn,mix")
    args = ap.parse_args()
    from mamba_clip_amd import ops, selective_scan_interface as ssi
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    m = torch.empty(256, 197, 768, device=dev, dtype=bf)
    xf = torch.empty(50432 // 4, 768, device=dev)
    vit_x = torch.randn(50432, 768, device=dev, generator=g).to(bf)
    vit_w = torch.randn(3072, 768, device=dev, generator=g).to(bf)
    # the C2 mixer's scan backward (channel-major views, fine saved states)
    Bsz, D, L, N = 256, 1536, 80, 16

    def cm(rows):
        return torch.randn(rows, Bsz * L, device=dev, generator=g).to(bf).view(rows, Bsz, L).transpose(0, 1)
    u, z, dout = cm(D), cm(D), cm(D)
    delta = (cm(D).float() * 0.5).to(bf)
    A = -torch.exp(torch.log(torch.arange(1, N + 1, device=dev, dtype=torch.float32)).repeat(D, 1))
    BC = torch.randn(2 * N, Bsz * L, device=dev, generator=g).to(bf)
    Bm = BC[:N].view(N, Bsz, L).transpose(0, 1).unsqueeze(1)
    Cm = BC[N:].view(N, Bsz, L).transpose(0, 1).unsqueeze(1)
    Dv = torch.ones(D, device=dev)
    bias = torch.rand(D, device=dev, generator=g) - 4.0
    _, st, _ = ssi.scan_fwd(u, delta, A, Bm, Cm, Dv, z, bias, True, True, False)
    qkv = torch.randn(256, 197, 3 * 768, device=dev, generator=g).to(bf)
    side = torch.cuda.Stream()

    def scan_bwd():
        out = ssi.scan_bwd(u, delta, A, Bm, Cm, Dv, z, bias, True, dout, st)
        return torch.cat([o.float().reshape(-1) for o in out if o is not None])

    tokens = torch.randint(0, 50280, (256, 80), device=dev, generator=g)
    tokens[:, 77:] = 0
    gemb = torch.empty(256, 80, 768, device=dev)

    def emb_bwd():   # the text towers' token-embedding gradient (torch: sort + lookback scans + segment sums)
        return torch.ops.aten.embedding_dense_backward(gemb, tokens, 50280, -1, False)

    victims = {
        "emb_bwd": emb_bwd,
        "scan_bwd": scan_bwd,
        "sum0_bf16": lambda: m.sum(0, keepdim=True),
        "colsum_f32": lambda: torch.sum(xf, 0),
        "mc_sum_rows": lambda: ops.sum_rows(xf),
    }
    for load in args.loads.split(","):
        bad = {k: 0 for k in victims}
        worst = {}
        for it in range(args.iters):
            m.normal_(generator=g)
            xf.normal_(generator=g)
            dout.normal_(generator=g)
            gemb.normal_(generator=g)
            if load != "none":
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    if load in ("gemm_vit", "mix"):
                        for _ in range(3):
                            torch.nn.functional.linear(vit_x, vit_w)
                            torch.mm(vit_x.t(), vit_x)
                    if load in ("attn", "mix"):
                        for _ in range(2):
                            q = qkv.detach().requires_grad_(True)
                            o = ops.packed_attention(q, 12)
                            o.backward(torch.ones_like(o))
            got = {k: f().clone() for k, f in victims.items()}
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            for k, f in victims.items():
                again = f()
                if not torch.equal(got[k], again):
                    bad[k] += 1
                    d = (got[k].float() - again.float()).abs()
                    worst.setdefault(k, []).append((int((d > 0).sum()), float(d.max()), float(again.float().abs().max())))
        print(json.dumps({"load": load, "iters": args.iters, "mismatches": bad,
                          "diffs_first3": {k: v[:3] for k, v in worst.items()},
                          "main_stream_is_null": torch.cuda.current_stream().cuda_stream == 0}), flush=True)


if __name__ == "__main__":
    main()
