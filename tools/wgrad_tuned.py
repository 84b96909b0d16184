"""Dev tool: the towers' weight-gradient GEMMs as ops.wgrad runs them (fp32 slabs + slab sum, library
heuristic: TunableOp does not cover fp32-output batched GEMMs) vs ONE bf16-output GEMM (the reference's
autocast form: dW rounded once to bf16) with its solution tuned by TunableOp here.  C2 shapes, HIP
events, us per call."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
import mamba_clip_amd  # noqa: E402,F401  (sets the package's GEMM environment first)
import torch  # noqa: E402
from mamba_clip_amd.ops import wgrad  # noqa: E402
from mamba_clip_amd.tuning import load_gemm_tuning  # noqa: E402

load_gemm_tuning()
dev, bf = "cuda", torch.bfloat16
tun = torch.cuda.tunable
out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/wgrad_tuned%d.csv"
tun.set_filename(out)
tun.set_max_tuning_duration(15)
tun.set_max_tuning_iterations(20)


def t(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


shapes = [("vit qkv", 50432, 2304, 768), ("vit proj", 50432, 768, 768), ("vit fc1", 50432, 3072, 768),
          ("vit fc2", 50432, 768, 3072), ("mamba in_proj", 20480, 3072, 768), ("mamba out_proj", 20480, 768, 1536)]
for name, M, N, K in shapes:
    g = torch.randn(M, N, device=dev, dtype=bf)
    x = torch.randn(M, K, device=dev, dtype=bf)
    fl = 2 * M * N * K
    cur = t(lambda: wgrad(g.t(), x))
    heur = t(lambda: torch.mm(g.t(), x))
    tun.tuning_enable(True)
    ref = torch.mm(g.t(), x)
    torch.cuda.synchronize()
    tun.tuning_enable(False)
    tuned = t(lambda: torch.mm(g.t(), x))
    xT = x.t().contiguous()
    tun.tuning_enable(True)
    torch.mm(xT, g)
    torch.cuda.synchronize()
    tun.tuning_enable(False)
    tunedT = t(lambda: torch.mm(xT, g))
    err = float((ref.float() - wgrad(g.t(), x)).abs().max() / wgrad(g.t(), x).abs().max())
    print(f"{name:14s} N{N} K{K} M{M}: wgrad fp32 slabs {cur:6.1f} ({fl / cur / 1e6:4.0f}) | bf16 mm heuristic {heur:6.1f} "
          f"({fl / heur / 1e6:4.0f}) | bf16 mm tuned {tuned:6.1f} ({fl / tuned / 1e6:4.0f}) | x^T-contig tuned (dW^T) "
          f"{tunedT:6.1f} ({fl / tunedT / 1e6:4.0f}) | rel err bf16 {err:.2e}", flush=True)
    del g, x, xT
tun.write_file()
