#!/usr/bin/env python3
"""Same-process A/B of the towers' weight-gradient GEMMs at the C2 shapes: the library split-K slabs
(ops.wgrad with MAMBA_CLIP_AMD_WGRAD_HIP off: bmm(out_dtype=fp32) + mc_sum_slabs) vs mc_gemm_wgrad
(csrc/gemm_wgrad.hip), HIP events, interleaved rounds; plus a split-count sweep of the HIP kernel.
Prints one JSON line per shape: us and TFLOP/s per arm, max |diff| relative to max |ref|."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
import torch  # noqa: E402

from mamba_clip_amd import ops  # noqa: E402
from mamba_clip_amd.tuning import load_gemm_tuning  # noqa: E402

DEV = torch.device("cuda", 0)
# name, N (out features), K (in features), T (tokens), G feature-major?, X feature-major?
SHAPES = [
    ("vit_qkv", 2304, 768, 50432, False, False),
    ("vit_proj", 768, 768, 50432, False, False),
    ("vit_fc1", 3072, 768, 50432, False, False),
    ("vit_fc2", 768, 3072, 50432, False, False),
    ("vit_patch", 768, 768, 50176, False, False),
    ("mamba_in_proj", 3072, 768, 20480, True, True),
    ("mamba_out_proj", 768, 1536, 20480, False, True),
    ("mamba_x_proj", 80, 1536, 20480, True, True),
    ("mamba_dt_proj", 1536, 48, 20480, True, True),
]


def operands(N, K, T, a_fm, b_fm):
    g = torch.Generator(device=DEV).manual_seed(N * 7 + K)
    G = torch.randn(N, T, device=DEV, generator=g).bfloat16() if a_fm else \
        torch.randn(T, N, device=DEV, generator=g).bfloat16().t()
    X = torch.randn(K, T, device=DEV, generator=g).bfloat16().t() if b_fm else \
        torch.randn(T, K, device=DEV, generator=g).bfloat16()
    return G, X


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
    only = sys.argv[1:] or None
    for name, N, K, T, a_fm, b_fm in SHAPES:
        if only and name not in only:
            continue
        G, X = operands(N, K, T, a_fm, b_fm)
        flop = 2.0 * N * K * T
        ops.WGRAD_HIP = False
        lib_us = timed(lambda: ops.wgrad(G, X))
        ref = ops.wgrad(G, X)
        pipes = {}
        for pipe in ("2", "4", "5"):
            os.environ["MC_WGRAD_PIPE"] = pipe
            pipes[pipe] = round(timed(lambda: ops.wgrad_hip(G, X)), 1)
        os.environ["MC_WGRAD_PIPE"] = "5"
        hip_us = pipes["5"]
        out = ops.wgrad_hip(G, X)
        err = float((out - ref).abs().max() / ref.abs().max())
        sweep = {}
        for s in (1, 2, 4, 7, 9, 14, 16, 28, 32):
            if T // 64 >= s:
                sweep[s] = round(timed(lambda: ops.wgrad_hip(G, X, splits=s), iters=10, rounds=3), 1)
        print(json.dumps({"shape": name, "N": N, "K": K, "T": T, "lib_us": round(lib_us, 1), "hip_us": round(hip_us, 1),
                          "lib_tflops": round(flop / lib_us / 1e6, 1), "hip_tflops": round(flop / hip_us / 1e6, 1),
                          "rel_err_vs_lib": err, "pipe_us": pipes,
                          "hip_split_sweep_us": sweep}), flush=True)


if __name__ == "__main__":
    main()
