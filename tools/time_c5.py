"""Dev tool: time the C5 similarity (fp8 GEMM, fp32 / bf16 logits) with HIP events."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd.ops import gemm_nt, quant_rows_fp8  # noqa: E402

dev = "cuda"
n, e = int(os.environ.get("N", 8192)), int(os.environ.get("E", 512))
g = torch.Generator(device=dev).manual_seed(5)
I = torch.nn.functional.normalize(torch.randn(n, e, device=dev, generator=g), dim=-1).bfloat16()
T = torch.nn.functional.normalize(torch.randn(n, e, device=dev, generator=g), dim=-1).bfloat16()
qi, si = quant_rows_fp8(I)
qt, st = quant_rows_fp8(T)
scale = torch.tensor(100.0, device=dev)
for name, fn in (("fp8 fp32-out", lambda: gemm_nt(qi, qt, alpha_dev=scale, scale_a=si, scale_b=st)),
                 ("fp8 bf16-out", lambda: gemm_nt(qi, qt, alpha_dev=scale, scale_a=si, scale_b=st, out_dtype=torch.bfloat16)),
                 ("bf16 fp32-out", lambda: gemm_nt(I, T, alpha_dev=scale))):
    for _ in range(3):
        fn()
    s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        fn()
    t.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(t) / 20
    print(f"{name}: {ms * 1e3:.1f} us  {2 * n * n * e / ms / 1e9:.0f} TFLOP/s")

# library reference point: hipBLASLt fp8 with row-wise scales through torch._scaled_mm
try:
    a8 = qi[:, :e].contiguous()
    b8 = qt[:, :e].contiguous().t()
    for od in (torch.bfloat16, torch.float32):
        fn = lambda: torch._scaled_mm(a8, b8, scale_a=si.view(-1, 1), scale_b=st.view(1, -1), out_dtype=od)  # noqa: E731
        for _ in range(3):
            fn()
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(20):
            fn()
        t.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(t) / 20
        print(f"torch._scaled_mm (hipBLASLt, TENSILE_STREAMK_DATA_PARALLEL={os.environ.get('TENSILE_STREAMK_DATA_PARALLEL')}) "
              f"{od}: {ms * 1e3:.1f} us  {2 * n * n * e / ms / 1e9:.0f} TFLOP/s")
except Exception as ex:  # noqa: BLE001
    print("torch._scaled_mm unavailable:", repr(ex)[:200])
