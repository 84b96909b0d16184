"""Time the fused logits+CE (mc_ce_fused_*) against the unfused path (S materialised:
gemm_nt + ce_stats x2 + ce_grad + transposed-operand gemm_nt x2) at a given N, E.

    python tools/time_ce.py --n 8192 --e 512 [--fp8]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd.ops import (ce_grad, ce_stats, clip_loss_fp8, gemm_nt, scaled_logits_ce)  # noqa: E402


def timed(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def unfused(X, Y, sc, gout):
    n = X.shape[0]
    S = gemm_nt(X, Y, alpha_dev=sc)
    lr, l1 = ce_stats(S, 0, 0, 0.5 / n)
    lc, l2 = ce_stats(S, 1, 0, 0.5 / n)
    G, ds = ce_grad(S, lr, 0, 0.5 / n, lc, 0, 0.5 / n, gout, X.dtype, sc)
    dX = gemm_nt(G, Y.t().contiguous(), alpha_dev=sc)
    dY = gemm_nt(G.t().contiguous(), X.t().contiguous(), alpha_dev=sc)
    return l1 + l2, dX, dY, ds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--e", type=int, default=512)
    ap.add_argument("--fp8", action="store_true")
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.nn.functional.normalize(torch.randn(a.n, a.e, device="cuda", generator=g), dim=-1).bfloat16()
    Y = torch.nn.functional.normalize(torch.randn(a.n, a.e, device="cuda", generator=g), dim=-1).bfloat16()
    sc = torch.tensor(30.0, device="cuda")
    gout = torch.tensor(1.0, device="cuda")
    Xg, Yg, sg = X.clone().requires_grad_(True), Y.clone().requires_grad_(True), sc.clone().requires_grad_(True)

    def fused():
        loss = scaled_logits_ce(Xg, Yg, sg, 0, 0.5 / a.n, 0, 0.5 / a.n)
        loss.backward()

    def fused_fwd():
        with torch.no_grad():
            scaled_logits_ce(X, Y, sc, 0, 0.5 / a.n, 0, 0.5 / a.n)

    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    b0 = torch.cuda.memory_allocated()
    t_f = timed(fused)
    pk_f = torch.cuda.max_memory_allocated() - b0
    t_ff = timed(fused_fwd)
    torch.cuda.reset_peak_memory_stats()
    b0 = torch.cuda.memory_allocated()
    t_u = timed(lambda: unfused(X, Y, sc, gout))
    pk_u = torch.cuda.max_memory_allocated() - b0
    flop = 2.0 * a.n * a.n * a.e
    print(f"N={a.n} E={a.e} bf16: fused fwd {t_ff:.3f} ms ({flop / t_ff / 1e9:.0f} TFLOP/s on the logits GEMM), "
          f"fused fwd+bwd {t_f:.3f} ms (peak +{pk_f / 2**20:.0f} MiB); "
          f"unfused fwd+bwd {t_u:.3f} ms (peak +{pk_u / 2**20:.0f} MiB)")
    if a.fp8:
        t8 = timed(lambda: clip_loss_fp8(X, Y, sc))
        print(f"N={a.n} E={a.e} fp8 fused loss (incl. quantisation): {t8:.3f} ms")


if __name__ == "__main__":
    main()
