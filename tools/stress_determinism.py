#!/usr/bin/env python3
"""Is a kernel's output a function of its inputs alone, also while another HIP stream keeps the chip
busy?  Each op runs once on a quiet device (reference), then --iters times on the main stream while
a side stream runs a load (library GEMMs, our attention backward, or a second scan backward on its own
data); every output is compared bitwise with the reference.  C2 text-tower shapes (B 256, D 1536,
L 80, bf16, channel-major views as in the mixer)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--ops", default="scan_bwd,scan_bwd_nofine,scan_fwd,conv_bwd,rms_bwd")
    ap.add_argument("--loads", default="none,gemm,attn,scan")
    args = ap.parse_args()
    from mamba_clip_amd import ops, selective_scan_interface as ssi
    from mamba_clip_amd.tuning import load_gemm_tuning
    if os.environ.get("STRESS_TUNED", "1") == "1":
        load_gemm_tuning(model="vit_b16-mamba130m")

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    Bsz, D, L, N = 256, 1536, 80, 16
    bf = torch.bfloat16

    def cm(rows):   # channel-major (B, rows, L) view of a (rows, B*L) buffer
        return torch.randn(rows, Bsz * L, device=dev, generator=g).to(bf).view(rows, Bsz, L).transpose(0, 1)

    u, z, dout = cm(D), cm(D), cm(D)
    delta = (cm(D).float() * 0.5).to(bf)
    A = -torch.exp(torch.log(torch.arange(1, N + 1, device=dev, dtype=torch.float32)).repeat(D, 1))
    BC = torch.randn(2 * N, Bsz * L, device=dev, generator=g).to(bf)
    Bm = BC[:N].view(N, Bsz, L).transpose(0, 1).unsqueeze(1)
    Cm = BC[N:].view(N, Bsz, L).transpose(0, 1).unsqueeze(1)
    Dv = torch.ones(D, device=dev)
    bias = torch.rand(D, device=dev, generator=g) - 4.0

    def states_for(fine):
        os.environ["MAMBA_CLIP_AMD_FINE_STATES_MB"] = "8192" if fine else "0"
        _, st, _ = ssi.scan_fwd(u, delta, A, Bm, Cm, Dv, z, bias, True, True, False)
        return st

    st_fine, st_def = states_for(True), states_for(False)
    x_conv = cm(D)
    w_conv = torch.randn(D, 1, 4, device=dev, generator=g) * 0.3
    b_conv = torch.randn(D, device=dev, generator=g) * 0.1
    h_rms = torch.randn(Bsz * L, 768, device=dev, generator=g).to(bf)
    res_rms = torch.randn(Bsz * L, 768, device=dev, generator=g)
    w_rms = torch.rand(768, device=dev, generator=g) + 0.5

    w_in = torch.randn(3072, 768, device=dev, generator=g).to(bf)
    h_cm = torch.randn(768, Bsz * L, device=dev, generator=g).to(bf)
    w_out = torch.randn(768, D, device=dev, generator=g).to(bf)
    g_out = torch.randn(Bsz * L, 768, device=dev, generator=g).to(bf)
    g_s = torch.randn(8, 768, (Bsz * L) // 8, device=dev, generator=g).to(bf)
    x_s = torch.randn(8, (Bsz * L) // 8, 1536, device=dev, generator=g).to(bf)
    vit_x = torch.randn(50432, 768, device=dev, generator=g).to(bf)
    vit_w = torch.randn(3072, 768, device=dev, generator=g).to(bf)
    vit_m = torch.randn(256, 197, 768, device=dev, generator=g).to(bf)

    def run(op):
        if op == "scan_bwd":
            return ssi.scan_bwd(u, delta, A, Bm, Cm, Dv, z, bias, True, dout, st_fine)
        if op == "scan_bwd_nofine":
            return ssi.scan_bwd(u, delta, A, Bm, Cm, Dv, z, bias, True, dout, st_def)
        if op == "scan_fwd":
            return ssi.scan_fwd(u, delta, A, Bm, Cm, Dv, z, bias, True, True, False)
        if op == "conv_bwd":
            xr = x_conv.detach().requires_grad_(True)
            wr = w_conv.detach().requires_grad_(True)
            br = b_conv.detach().requires_grad_(True)
            y = ops.causal_conv1d(xr, wr, br, silu=True)
            y.backward(dout)
            return xr.grad, wr.grad, br.grad
        if op == "rms_bwd":
            hr = h_rms.detach().requires_grad_(True)
            rr = res_rms.detach().requires_grad_(True)
            wr = w_rms.detach().requires_grad_(True)
            y, hres = ops.add_rmsnorm(hr, rr, wr, 1e-5)
            (y.float().sum() + hres.sum() * 0.5).backward()
            return hr.grad, rr.grad, wr.grad
        if op == "gemm_in_proj":      # the mixer's in_proj forward: (3072 x 768) @ (768 x 20480)
            return torch.mm(w_in, h_cm)
        if op == "gemm_out_dgrad":    # out_proj's input gradient into the channel-major layout
            return torch.mm(w_out.t(), g_out.t()).t()
        if op == "sum0":             # the ViT's pos_embed gradient: a bf16 (B, 197, 768) summed over the batch
            return vit_m.sum(0, keepdim=True)
        if op == "sum_cls":          # cls_token: the batch sum of one row
            return vit_m[:, :1].sum(0, keepdim=True)
        if op == "colsum_f32":       # a bias gradient: fp32 column sums of (B*L, C)
            return torch.sum(vit_x, 0, dtype=torch.float32)
        if op == "bmm_f32":           # the split-K weight-gradient slabs (ops.wgrad library path)
            return torch.bmm(g_s, x_s, out_dtype=torch.float32)
        raise ValueError(op)

    # side loads (each keeps the side stream busy for longer than one op)
    side = torch.cuda.Stream()
    ga = torch.randn(8192, 8192, device=dev).to(bf)
    qkv = torch.randn(256, 197, 3 * 768, device=dev).to(bf)
    u2, z2, d2 = u.clone(), z.clone(), dout.clone()

    def load(kind):
        if kind == "gemm":
            for _ in range(6):
                ga @ ga
        elif kind == "gemm_vit":
            for _ in range(3):
                torch.nn.functional.linear(vit_x, vit_w)
                torch.mm(vit_x.t(), vit_x)
        elif kind == "attn":
            q = qkv.detach().requires_grad_(True)
            o = ops.packed_attention(q, 12)
            o.backward(torch.ones_like(o))
        elif kind == "scan":
            for _ in range(4):
                ssi.scan_bwd(u2, delta, A, Bm, Cm, Dv, z2, bias, True, d2, st_fine)
        elif kind == "scan_nofine":
            for _ in range(4):
                ssi.scan_bwd(u2, delta, A, Bm, Cm, Dv, z2, bias, True, d2, st_def)
        elif kind == "scan_fwd":
            for _ in range(4):
                ssi.scan_fwd(u2, delta, A, Bm, Cm, Dv, z2, bias, True, True, False)

    def eq(a, b):
        if isinstance(a, torch.Tensor):
            return torch.equal(a, b)
        if isinstance(a, (tuple, list)):
            return all(eq(x, y) for x, y in zip(a, b))
        return True

    def snap(x):
        if isinstance(x, torch.Tensor):
            return x.detach().clone()
        if isinstance(x, (tuple, list)):
            return [snap(v) for v in x]
        return x

    for op in args.ops.split(","):
        torch.cuda.synchronize()
        ref = snap(run(op))
        torch.cuda.synchronize()
        for kind in args.loads.split(","):
            bad = 0
            for _ in range(args.iters):
                if kind != "none":
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        load(kind)
                out = snap(run(op))
                if kind != "none":
                    torch.cuda.current_stream().wait_stream(side)
                torch.cuda.synchronize()
                if not eq(ref, out):
                    bad += 1
            print(json.dumps({"op": op, "load": kind, "iters": args.iters, "mismatches": bad}), flush=True)


if __name__ == "__main__":
    main()
