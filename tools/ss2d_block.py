"""Dev tool: the whole SS2D block (model.py:630-647) fwd+bwd, fused cross-scan glue (mc_ss2d.h) vs the
reference construction (permute + conv2d + SiLU + stack / transposes + merge + LayerNorm + gate, the
oracle restatements), HIP scan in both, at the medmamba VSSM stage shapes (B 32, 224x224 input).

    python tools/ss2d_block.py [--trace]     (--trace: one fused fwd+bwd of the 56x56 stage between
                                              two spin-kernel markers, for rocprofv3 --kernel-trace)
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
sys.path.insert(0, ROOT)
import mamba_clip_amd.model as M  # noqa: E402
from oracle.cpu_model import ss2d_conv_stack_ref, ss2d_merge_ln_gate_ref  # noqa: E402

FUSED = (M.ss2d_conv_stack, M.ss2d_merge_ln_gate)
REF = (ss2d_conv_stack_ref, ss2d_merge_ln_gate_ref)


def run(m, x, ops, iters):
    M.ss2d_conv_stack, M.ss2d_merge_ln_gate = ops
    try:
        def step():
            xg = x.detach().requires_grad_(True)
            m(xg).sum().backward()
        for _ in range(3):
            step()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            step()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters
    finally:
        M.ss2d_conv_stack, M.ss2d_merge_ln_gate = FUSED


if os.environ.get("SS2D_PROJ") == "0":          # A/B: the einsum projections instead of mc_ss2d_group_proj
    M.ss2d_proj_ok = lambda *a: False
torch.manual_seed(0)
if "--trace" in sys.argv:
    m = M.SS2D(d_model=32).cuda()
    x = torch.randn(32, 56, 56, 32, device="cuda")
    run(m, x, FUSED, 1)
    torch.cuda._sleep(100000)
    xg = x.detach().requires_grad_(True)
    m(xg).sum().backward()
    torch.cuda._sleep(100000)
    torch.cuda.synchronize()
    print("traced one fused SS2D fwd+bwd (B 32, 56x56, d_model 32)")
else:
    for d_model, hw in ((32, 56), (64, 28), (128, 14), (256, 7)):
        m = M.SS2D(d_model=d_model).cuda()
        x = torch.randn(32, hw, hw, d_model, device="cuda")
        tf, tr = run(m, x, FUSED, 20), run(m, x, REF, 20)
        print(f"SS2D B32 d_model {d_model} d_inner {2 * d_model} {hw}x{hw} fp32 fwd+bwd: fused {tf:.3f} ms, "
              f"reference construction {tr:.3f} ms", flush=True)
