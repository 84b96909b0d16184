"""Dev tool: time mc_attn_fwd / mc_attn_bwd kernels alone (C ABI, HIP events), with and without the
in-kernel column sums (dsum).  MAMBA_CLIP_AMD_LIB selects an A/B library build.
usage: python tools/time_attn_bwd.py [--shape B,N,H] [--iters 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="256,197,12")
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
B, N, H = map(int, args.shape.split(","))
D, C = 64, H * 64
lib = _lib.load()
dev = "cuda"
y = torch.randn(B, N, 3 * C, device=dev, dtype=torch.bfloat16)
o = torch.empty(B, N, C, device=dev, dtype=torch.bfloat16)
g = torch.randn(B, N, C, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B, H, N, device=dev)
dy = torch.empty_like(y)
dsum = torch.empty(B, 3 * C, device=dev)
es = 2
f = _lib.AttnFwdParams()
f.batch, f.heads, f.seqlen, f.head_dim, f.dtype, f.scale = B, H, N, D, _lib.MC_DTYPE_BF16, D ** -0.5
f.q, f.k, f.v = y.data_ptr(), y.data_ptr() + C * es, y.data_ptr() + 2 * C * es
f.q_bs, f.q_ns, f.q_hs = y.stride(0), y.stride(1), D
f.o, f.o_bs, f.o_ns, f.o_hs, f.lse = o.data_ptr(), o.stride(0), o.stride(1), D, lse.data_ptr()
b = _lib.AttnBwdParams()
b.batch, b.heads, b.seqlen, b.head_dim, b.dtype, b.scale = B, H, N, D, _lib.MC_DTYPE_BF16, D ** -0.5
b.q, b.k, b.v = f.q, f.k, f.v
b.q_bs, b.q_ns, b.q_hs = f.q_bs, f.q_ns, f.q_hs
b.o, b.dout, b.o_bs, b.o_ns, b.o_hs, b.lse = o.data_ptr(), g.data_ptr(), o.stride(0), o.stride(1), D, lse.data_ptr()
b.dq, b.dk, b.dv = dy.data_ptr(), dy.data_ptr() + C * es, dy.data_ptr() + 2 * C * es
b.dq_bs, b.dq_ns, b.dq_hs = dy.stride(0), dy.stride(1), D
st = _lib.stream_handle()


def t(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(args.iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / args.iters * 1e3


fwd = t(lambda: _lib.check(lib.mc_attn_fwd(f, st), "fwd"))
b.dsum = None
bwd0 = t(lambda: _lib.check(lib.mc_attn_bwd(b, st), "bwd"))
b.dsum = dsum.data_ptr()
bwd1 = t(lambda: _lib.check(lib.mc_attn_bwd(b, st), "bwd"))
print(f"{os.environ.get('MAMBA_CLIP_AMD_LIB', 'in-tree')}: B{B} N{N} H{H}: fwd {fwd:.1f} us  bwd {bwd0:.1f} us  "
      f"bwd+colsum {bwd1:.1f} us", flush=True)
