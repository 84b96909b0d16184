"""Dev tool: do better library solutions exist for the split-K weight-gradient GEMMs?  ops.wgrad's
strided-batched form (s token slabs) timed with the heuristic's pick (fp32 out, as shipped; bf16 out)
and with TunableOp's tuned pick (bf16 out: TunableOp does not cover fp32-output batched GEMMs).
C2 / C3 shapes, HIP events, us per call."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
import mamba_clip_amd  # noqa: E402,F401
import torch  # noqa: E402
from mamba_clip_amd.ops import _split_factor  # noqa: E402

dev, bf = "cuda", torch.bfloat16
tun = torch.cuda.tunable
tun.enable(True)
tun.tuning_enable(False)
tun.set_filename(sys.argv[1] if len(sys.argv) > 1 else "/tmp/wgt%d.csv")
tun.set_max_tuning_duration(20)
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


shapes = [("vit qkv", 50432, 2304, 768), ("vit fc1", 50432, 3072, 768), ("vit fc2", 50432, 768, 3072),
          ("vit proj", 50432, 768, 768), ("c3 vit fc1", 12608, 3072, 768), ("c3 bert fc1", 16384, 3072, 768)]
for name, M, N, K in shapes:
    g = torch.randn(M, N, device=dev, dtype=bf)
    x = torch.randn(M, K, device=dev, dtype=bf)
    s = _split_factor(M, N, K)
    Gs = g.t().unflatten(1, (s, M // s)).transpose(0, 1)
    Xs = x.unflatten(0, (s, M // s))
    f32 = t(lambda: torch.bmm(Gs, Xs, out_dtype=torch.float32))
    b16 = t(lambda: torch.bmm(Gs, Xs))
    tun.tuning_enable(True)
    torch.bmm(Gs, Xs)
    torch.cuda.synchronize()
    tun.tuning_enable(False)
    b16t = t(lambda: torch.bmm(Gs, Xs))
    fl = 2 * M * N * K
    print(f"{name:12s} s{s} N{N} K{K} M{M}: fp32-out heuristic {f32:6.1f} ({fl / f32 / 1e6:4.0f}) | bf16-out heuristic "
          f"{b16:6.1f} ({fl / b16 / 1e6:4.0f}) | bf16-out tuned {b16t:6.1f} ({fl / b16t / 1e6:4.0f})", flush=True)
    del g, x, Gs, Xs
