"""Dev tool: weight-gradient GEMMs of the C2 towers (dW = g^T x, K = tokens), library layouts vs manual split-K."""
import time

import torch

dev, bf = "cuda", torch.bfloat16
try:
    from mamba_clip_amd.tuning import load_gemm_tuning  # noqa: F401
except Exception:  # noqa: BLE001
    pass


def bench(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def splitk(g, x, s):
    M = g.shape[0]
    gs = g.view(s, M // s, -1).transpose(1, 2)      # (s, N, M/s)
    xs = x.view(s, M // s, -1)                      # (s, M/s, K)
    return torch.bmm(gs, xs, out_dtype=torch.float32).sum(0) if hasattr(torch, "_bmm_out_dtype") else \
        torch.bmm(gs, xs).float().sum(0)


for (M, N, K) in [(50432, 3072, 768), (50432, 768, 3072), (50432, 2304, 768), (50432, 768, 768),
                  (20480, 3072, 768), (20480, 768, 1536), (20480, 1536, 80)]:
    g = torch.randn(M, N, device=dev, dtype=bf)
    x = torch.randn(M, K, device=dev, dtype=bf)
    fl = 2 * M * N * K
    res = {}
    res["mm(g.t(),x)"] = bench(lambda: torch.mm(g.t(), x))
    res["mm(x.t(),g).t()"] = bench(lambda: torch.mm(x.t(), g).t())
    gt = g.t().contiguous()
    res["mm(gT contig, x)"] = bench(lambda: torch.mm(gt, x))
    for s in (2, 4, 8):
        if M % s == 0:
            res[f"splitK{s} bmm+sum"] = bench(lambda s=s: splitk(g, x, s))
    line = " | ".join(f"{k} {v:.3f} ms ({fl / v / 1e9:.0f} TF/s)" for k, v in res.items())
    print(f"M{M} N{N} K{K}: {line}")
