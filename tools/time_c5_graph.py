"""Dev tool: C5 similarity (fp8 GEMM, fp32 / bf16 logits, N 8192, E 512) timed three ways -- a plain
launch loop, the same calls captured once in a HIP graph and replayed (no host launch gaps), and one
call per event pair -- to separate the kernel's time from host launch overhead."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd.ops import gemm_nt, quant_rows_fp8  # noqa: E402

dev = "cuda"
n, e, iters = 8192, 512, 20
g = torch.Generator(device=dev).manual_seed(5)
I = torch.nn.functional.normalize(torch.randn(n, e, device=dev, generator=g), dim=-1).bfloat16()
T = torch.nn.functional.normalize(torch.randn(n, e, device=dev, generator=g), dim=-1).bfloat16()
qi, si = quant_rows_fp8(I)
qt, st = quant_rows_fp8(T)
scale = torch.tensor(100.0, device=dev)


def ev_time(fn):
    s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    fn()
    t.record()
    torch.cuda.synchronize()
    return s.elapsed_time(t) * 1e3


for od in (torch.float32, torch.bfloat16):
    call = lambda: gemm_nt(qi, qt, alpha_dev=scale, scale_a=si, scale_b=st, out_dtype=od)  # noqa: E731
    for _ in range(3):
        call()
    loop_us = ev_time(lambda: [call() for _ in range(iters)]) / iters
    single = sorted(ev_time(call) for _ in range(iters))
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            call()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        outs = [call() for _ in range(iters)]
    for _ in range(2):
        graph.replay()
    graph_us = min(ev_time(graph.replay) for _ in range(5)) / iters
    print(f"{str(od)[6:]} logits: loop {loop_us:.1f} us/call, one call per event pair median {single[iters // 2]:.1f} "
          f"min {single[0]:.1f} us, graph replay {graph_us:.1f} us/call", flush=True)
    del outs, graph
