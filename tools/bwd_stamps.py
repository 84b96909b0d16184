"""Dev tool: per-segment cycle split of scan_bwd_kernel from a diagnostic build with -DMC_BWD_STAMPS.

Build: make -C mamba-clip_amd stamps   (-> mamba_clip_amd/libmamba_clip_amd_stamps.so)
Run:   MAMBA_CLIP_AMD_LIB=<that .so> python tools/bwd_stamps.py [--shape B,D,L,N]
Segments per wave, summed over its tiles: prologue (row / B/C / state loads,
prep math, barriers), pair loop, outputs (row re-read, output math, stores).
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
from mamba_clip_amd import _lib  # noqa: E402
from mamba_clip_amd.selective_scan_interface import scan_fwd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="256,1536,80,16")
args = ap.parse_args()
Bsz, D, L, N = map(int, args.shape.split(","))
dev, bf = "cuda", torch.bfloat16
torch.manual_seed(0)
u = torch.randn(Bsz, D, L, device=dev, dtype=bf)
delta = (0.5 * torch.randn(Bsz, D, L, device=dev)).to(bf)
z = torch.randn(Bsz, D, L, device=dev, dtype=bf)
A = -torch.exp(torch.log(torch.arange(1, N + 1, dtype=torch.float32, device=dev)).repeat(D, 1))
Bm = torch.randn(Bsz, 1, N, L, device=dev, dtype=bf)
Cm = torch.randn(Bsz, 1, N, L, device=dev, dtype=bf)
Dv = torch.ones(D, device=dev)
bias = torch.rand(D, device=dev) * 4 - 5
out, states, _, out_y = scan_fwd(u, delta, A, Bm, Cm, Dv, z, bias, True, True, False, want_y=True)
dout = torch.randn_like(u)
lib = _lib.load()
ws_b = lib.mc_scan_bwd_workspace_bytes(Bsz, D, L, N, 1)
ws = torch.zeros(ws_b, device=dev, dtype=torch.uint8)


def a256(x):
    return (x + 255) // 256 * 256


np_ = 8 if N <= 8 else (16 if N <= 16 else 32)
nblk = (D + 63) // 64
off = a256(Bsz * L * 2 * np_ * 4) + a256(Bsz * nblk * np_ * 2 * L * 4) + a256(Bsz * D * np_ * 4)
p = _lib.ScanBwdParams()
p.batch, p.dim, p.seqlen, p.dstate, p.n_groups = Bsz, D, L, N, 1
p.itype, p.wtype, p.delta_softplus = _lib.dtype_code(bf), _lib.dtype_code(bf), 1
for name, t in (("u", u), ("delta", delta), ("z", z), ("dout", dout)):
    setattr(p, f"{name}_batch_stride", t.stride(0))
    setattr(p, f"{name}_dim_stride", t.stride(1))
du, ddelta, dz = torch.empty_like(u), torch.empty_like(u), torch.empty_like(u)
for name, t in (("du", du), ("ddelta", ddelta), ("dz", dz)):
    setattr(p, f"{name}_batch_stride", t.stride(0))
    setattr(p, f"{name}_dim_stride", t.stride(1))
p.B_batch_stride, p.B_group_stride, p.B_dstate_stride = Bm.stride(0), Bm.stride(1), Bm.stride(2)
p.C_batch_stride, p.C_group_stride, p.C_dstate_stride = Cm.stride(0), Cm.stride(1), Cm.stride(2)
dB, dC = torch.empty_like(Bm), torch.empty_like(Cm)
dA, dD, dbias = torch.empty(D, N, device=dev), torch.empty(D, device=dev), torch.empty(D, device=dev)
p.u, p.delta, p.A, p.B, p.C = u.data_ptr(), delta.data_ptr(), A.data_ptr(), Bm.data_ptr(), Cm.data_ptr()
p.D, p.z, p.delta_bias, p.dout, p.chunk_states = Dv.data_ptr(), z.data_ptr(), bias.data_ptr(), dout.data_ptr(), states.data_ptr()
p.du, p.ddelta, p.dz, p.dB, p.dC = du.data_ptr(), ddelta.data_ptr(), dz.data_ptr(), dB.data_ptr(), dC.data_ptr()
p.dA, p.dD, p.ddelta_bias = dA.data_ptr(), dD.data_ptr(), dbias.data_ptr()
p.workspace, p.workspace_bytes = ws.data_ptr(), ws_b
p.out_y, p.out_y_batch_stride, p.out_y_dim_stride = out_y.data_ptr(), out_y.stride(0), out_y.stride(1)
for _ in range(2):
    _lib.check(lib.mc_scan_bwd(p, _lib.stream_handle(u.device)), "mc_scan_bwd")
torch.cuda.synchronize()
nwaves = Bsz * nblk
dbg = ws[off: off + nwaves * 32].cpu().numpy().view(np.uint64).reshape(nwaves, 4).astype(np.float64)
tot = dbg[:, :3].sum(1)
print(f"waves {nwaves}, tiles/wave {int(dbg[0, 3])}, mean cycles/wave {tot.mean():.0f}")
for i, name in enumerate(("prologue", "pair loop", "outputs")):
    print(f"  {name:10s} {dbg[:, i].mean():10.0f} cycles/wave ({dbg[:, i].sum() / tot.sum() * 100:5.1f} %)")
