#!/usr/bin/env python3
"""Forward / input-gradient GEMMs of the C2 Linears on the hand-written 256x256 kernel (mc_gemm_wgrad,
fp32 out: the operands map onto its feature-major / token-major layouts) vs the library (F.linear /
torch.mm, bf16 out, the shipped tuning).  HIP events, interleaved rounds, median.  One JSON line per
shape and pass."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
import torch  # noqa: E402

from mamba_clip_amd import ops  # noqa: E402
from mamba_clip_amd.tuning import load_gemm_tuning  # noqa: E402

DEV = torch.device("cuda", 0)
SHAPES = [("vit_qkv", 50432, 2304, 768), ("vit_proj", 50432, 768, 768), ("vit_fc1", 50432, 3072, 768),
          ("vit_fc2", 50432, 768, 3072), ("mamba_in_proj", 20480, 3072, 768), ("mamba_out_proj", 20480, 768, 1536)]


def timed(fn, iters=20, rounds=5):
    for _ in range(3):
        fn()
    st = torch.cuda.current_stream()
    res = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / iters * 1e3)
    return sorted(res)[len(res) // 2]


def main():
    load_gemm_tuning(model="vit_b16-mamba130m")
    g = torch.Generator(device=DEV).manual_seed(0)
    for name, T, N, K in SHAPES:
        x = (torch.rand(T, K, device=DEV, generator=g) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device=DEV, generator=g) * 2 - 1).bfloat16()
        dy = (torch.rand(T, N, device=DEV, generator=g) * 2 - 1).bfloat16()
        flop = 2.0 * T * N * K
        for pas, lib_fn, hip_fn in (
                ("fwd", lambda: torch.nn.functional.linear(x, w), lambda: ops.wgrad_hip(x, w.t())),
                ("dgrad", lambda: torch.mm(dy, w), lambda: ops.wgrad_hip(dy, w))):
            ref = lib_fn().float()
            out = hip_fn()
            if out is None:
                print(json.dumps({"shape": name, "pass": pas, "hip": "unsupported"}), flush=True)
                continue
            err = float((out - ref).abs().max() / ref.abs().max())
            lib_us, hip_us = timed(lib_fn), timed(hip_fn)
            print(json.dumps({"shape": name, "pass": pas, "T": T, "N": N, "K": K, "lib_us": round(lib_us, 1),
                              "hip_fp32out_us": round(hip_us, 1), "lib_tflops": round(flop / lib_us / 1e6, 1),
                              "hip_tflops": round(flop / hip_us / 1e6, 1), "rel_err": err}), flush=True)


def epilogues():
    """mc_linear with its fused epilogues vs the library chains they replace, at the C2 ViT shapes."""
    from mamba_clip_amd import _lib
    g = torch.Generator(device=DEV).manual_seed(1)
    T, C, Hd = 50432, 768, 3072
    bf = torch.bfloat16
    x = (torch.rand(T, C, device=DEV, generator=g) * 2 - 1).to(bf)
    w1 = ((torch.rand(Hd, C, device=DEV, generator=g) * 2 - 1) * 0.04).to(bf)
    b1 = ((torch.rand(Hd, device=DEV, generator=g) * 2 - 1) * 0.1).to(bf)
    w2 = ((torch.rand(C, Hd, device=DEV, generator=g) * 2 - 1) * 0.02).to(bf)
    b2 = ((torch.rand(C, device=DEV, generator=g) * 2 - 1) * 0.1).to(bf)
    wt1, wt2 = w1.t().contiguous(), w2.t().contiguous()
    gy = (torch.rand(T, C, device=DEV, generator=g) * 2 - 1).to(bf)
    h, a = ops.linear_hip(x, w1, b1, _lib.MC_LINEAR_EPI_BIAS_GELU)
    lib = _lib.load()

    def lib_gelu_bwd():
        ga = torch.mm(gy, wt2.t())
        gh = torch.empty_like(ga)
        db = torch.empty(Hd, device=DEV)
        ws_b = lib.mc_grad_colsum_workspace_bytes(T, Hd)
        ws = ops._ws(ws_b, DEV)
        _lib.check(lib.mc_gelu_bwd(T, Hd, _lib.dtype_code(bf), h.data_ptr(), Hd, ga.data_ptr(), Hd, gh.data_ptr(), Hd,
                                   db.data_ptr(), ws.data_ptr(), ws_b, _lib.stream_handle(DEV)), "mc_gelu_bwd")
        return gh

    cases = [
        ("fc1_fwd_bias_gelu", 2.0 * T * Hd * C,
         lambda: torch.nn.functional.gelu(torch.nn.functional.linear(x, w1, b1)),
         lambda: ops.linear_hip(x, w1, b1, _lib.MC_LINEAR_EPI_BIAS_GELU)),
        ("fc2_fwd_bias", 2.0 * T * Hd * C, lambda: torch.nn.functional.linear(a, w2, b2),
         lambda: ops.linear_hip(a, w2, b2)),
        ("fc2_dgrad_gelu_grad_colsum", 2.0 * T * Hd * C, lib_gelu_bwd,
         lambda: ops.linear_hip(gy, wt2, None, _lib.MC_LINEAR_EPI_GELU_GRAD, h=h, want_colsum=True)),
        ("fc1_dgrad", 2.0 * T * Hd * C, lambda: torch.mm(a, wt1.t()), lambda: ops.linear_hip(a, wt1)),
        ("qkv_fwd_bias", 2.0 * T * 3 * C * C, lambda: torch.nn.functional.linear(x, w1[:3 * C], b1[:3 * C]),
         lambda: ops.linear_hip(x, w1[:3 * C], b1[:3 * C])),
        ("proj_fwd_bias", 2.0 * T * C * C, lambda: torch.nn.functional.linear(x, w1[:C], b1[:C]),
         lambda: ops.linear_hip(x, w1[:C], b1[:C])),
    ]
    for name, flop, lib_fn, hip_fn in cases:
        lib_us, hip_us = timed(lib_fn), timed(hip_fn)
        os.environ["MC_LINEAR_STAGGER"] = "0"
        hip_us_nostag = timed(hip_fn)
        os.environ.pop("MC_LINEAR_STAGGER")
        print(json.dumps({"case": name, "lib_chain_us": round(lib_us, 1), "hip_us": round(hip_us, 1),
                          "hip_us_rows_in_step": round(hip_us_nostag, 1),
                          "hip_gemm_tflops": round(flop / hip_us / 1e6, 1)}), flush=True)


def small_k():
    """mc_gemm_small_k vs torch.mm at the C2 dt_proj forward: (1536 x 48) @ (48 x 20480) rows of the x_dbl slab."""
    g = torch.Generator(device=DEV).manual_seed(2)
    bf = torch.bfloat16
    w = ((torch.rand(1536, 48, device=DEV, generator=g) * 2 - 1) * 0.1).to(bf)
    slab = (torch.rand(80, 20480, device=DEV, generator=g) * 2 - 1).to(bf)
    x = slab[:48]
    lib_us, hip_us = timed(lambda: torch.mm(w, x)), timed(lambda: ops.gemm_small_k(w, x))
    nbytes = 1536 * 20480 * 2 + 48 * 20480 * 2
    print(json.dumps({"case": "dt_proj_fwd_1536x48x20480", "lib_us": round(lib_us, 1), "hip_us": round(hip_us, 1),
                      "hip_GBps": round(nbytes / hip_us / 1e3, 1)}), flush=True)
    wx = ((torch.rand(80, 1536, device=DEV, generator=g) * 2 - 1) * 0.05).to(bf)
    xc = (torch.rand(1536, 20480, device=DEV, generator=g) * 2 - 1).to(bf)
    lib_us, hip_us = timed(lambda: torch.mm(wx, xc)), timed(lambda: ops.gemm_skinny_m(wx, xc))
    nbytes = 1536 * 20480 * 2 + 80 * 20480 * 2
    print(json.dumps({"case": "x_proj_fwd_80x1536x20480", "lib_us": round(lib_us, 1), "hip_us": round(hip_us, 1),
                      "hip_GBps": round(nbytes / hip_us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    if "--small-k" in sys.argv:
        small_k()
        sys.exit(0)
    if "--epilogues" in sys.argv:
        load_gemm_tuning(model="vit_b16-mamba130m")
        epilogues()
        sys.exit(0)
    main()
