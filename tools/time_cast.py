"""Dev tool: the one-launch weight casts of ops.weight_cast_scope (plain mc_cast_f32_many, transposed
mc_cast_transpose_f32_many) over the ViT-B/16 tower's Linear weights, HIP events, us per call.
MAMBA_CLIP_AMD_LIB selects the build."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
import torch  # noqa: E402
import mamba_clip_amd.ops as O  # noqa: E402

ws = []
for _ in range(12):
    ws += [torch.randn(2304, 768, device="cuda"), torch.randn(768, 768, device="cuda"),
           torch.randn(3072, 768, device="cuda"), torch.randn(768, 3072, device="cuda")]
n = sum(w.numel() for w in ws)
tp = O._TransposePlan(ws, torch.bfloat16, "cuda")
cp = O._CastPlan(ws, torch.bfloat16, "cuda")
for name, plan in (("transposed", tp), ("plain", cp)):
    for _ in range(3):
        plan.run(ws)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        plan.run(ws)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 20 * 1e3
    print(f"{name:10s} {n / 1e6:.1f} M params: {us:7.1f} us  ({n * 6 / us / 1e3:.0f} GB/s)", flush=True)
