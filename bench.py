#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json metric): image-text pairs/sec + selective_scan HBM GB/s.

    python bench.py [--gpus N] [--steps K] [--warmup W]

Workload (value): C2 = ViT-B/16 image tower + Mamba-130M text tower, 224x224
synthetic images + 77-token synthetic text, batch 256 per GPU, bf16 autocast,
full step = forward + ClipLoss (HIP contrastive kernels; RCCL feature
all-gather for N > 1) + backward (DDP RCCL all-reduce) + fused AdamW +
logit_scale clamp.  Random-init weights, synthetic data resident in HBM.
value = N * batch * K / max-over-ranks(time of K steps).

roofline: the selective-scan forward at C4 (B=64, D=3072, L=4096, N=16, bf16,
z-gated, softplus) -- the kernel BASELINE.json's HBM target
names -- timed with HIP events on the stream it is launched on;
achieved = 6.4594 GB algorithmic bytes per call / average call time.

cpu_baseline: the fp32 CPU restatement (oracle/cpu_model.py) of the same
C2 training step on a bounded sample (batch 8), rank 0 at N = 1 only.

For N > 1 run under torch.distributed.run (one process per GPU, RCCL);
`--gpus N` without a launcher re-launches itself as a child torchrun job.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E peak (MI355X_MICROARCH.md)
MFMA_BF16_DENSE_TFLOPS = 2500.0  # dense bf16 MFMA peak (no sparsity)
MFMA_FP8_DENSE_TFLOPS = 5000.0   # dense fp8 MFMA peak (no sparsity)
C2_FLOP_PER_PAIR = 146e9         # fwd+bwd, SURVEY.md 8(d)
# per-model workload labels and fwd+bwd FLOP per pair (C2 146 G, C3 243 G)
WORKLOADS = {
    "vit_b16-mamba130m": ("C2: ViT-B/16 image + Mamba-130M text, contrastive train step (fwd+bwd+AdamW), amp_bf16",
                          C2_FLOP_PER_PAIR),
    "biomedclip-vit_b16-pubmedbert256": ("C3: BiomedCLIP ViT-B/16 image + PubMedBERT-256 text, contrastive train "
                                         "step (fwd+bwd+AdamW), amp_bf16", 243e9),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="pairs per GPU")
    ap.add_argument("--model", default="vit_b16-mamba130m")
    ap.add_argument("--scan-iters", type=int, default=20)
    ap.add_argument("--graph-streams", type=int, default=2, choices=(1, 2),
                    help="with --graph 1: capture the towers on two streams (2) or one (1)")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: replay the step as one HIP graph (train.GraphedStep; single process), 0: eager, "
                         "-1: graph when world size is 1 and inputs are resident (default 0 until measured)")
    ap.add_argument("--input", choices=["resident", "host"], default="resident",
                    help="resident: one synthetic batch in HBM (the `value` definition); host: ISIC-shaped raw "
                         "uint8 crops streamed from pinned host memory each step (data.HostToDeviceLoader)")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=8)
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every CPU this process may run on (see _cpu_threads)")
    return ap.parse_args()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(args):
    """--gpus N > 1 without a launcher: run torchrun as a child and exit with its code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def scan_roofline(iters, warmup=10):
    """selective_scan_fwd at C4 timed with HIP events on its launch stream.

    10 untimed calls first: right after the MFMA-heavy training steps the first ~8 calls run
    slower (rocprof trace, profiles/r02: 3.5 -> 2.6 ms while the clocks settle), and the
    roofline is about the kernel's steady state."""
    import torch
    from mamba_clip_amd.selective_scan_interface import scan_fwd
    dev = torch.device("cuda", torch.cuda.current_device())
    Bsz, D, L, N = 64, 3072, 4096, 16
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    u = torch.randn(Bsz, D, L, device=dev, generator=g, dtype=bf)
    z = torch.randn(Bsz, D, L, device=dev, generator=g, dtype=bf)
    delta = (torch.randn(Bsz, D, L, device=dev, generator=g) * 0.5).to(bf)
    dt = torch.exp(torch.rand(D, device=dev, generator=g) * (math.log(0.1) - math.log(1e-3)) + math.log(1e-3))
    dt = dt.clamp(min=1e-4)
    bias = dt + torch.log(-torch.expm1(-dt))
    A = -torch.exp(torch.log(torch.arange(1, N + 1, device=dev, dtype=torch.float32)).repeat(D, 1)
                   + 0.1 * torch.randn(D, N, device=dev, generator=g))
    Bm = torch.randn(Bsz, 1, N, L, device=dev, generator=g, dtype=bf)
    Cm = torch.randn(Bsz, 1, N, L, device=dev, generator=g, dtype=bf)
    Dv = torch.ones(D, device=dev)
    call = lambda: scan_fwd(u, delta, A, Bm, Cm, Dv, z, bias, True, False, False)  # noqa: E731
    for _ in range(warmup):
        call()
    stream = torch.cuda.current_stream(dev)      # the lib launches on torch's current stream
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    t0.record(stream)
    for _ in range(iters):
        call()
    t1.record(stream)
    torch.cuda.synchronize(dev)
    ms = t0.elapsed_time(t1) / iters
    nbytes = Bsz * D * L * 8 + 2 * Bsz * 1 * N * L * 2 + (D * N + 2 * D) * 4
    achieved = nbytes / (ms * 1e-3) / 1e9
    del u, z, delta, Bm, Cm
    torch.cuda.empty_cache()
    copy_gbs = _copy_bandwidth(dev)
    traffic, traffic_src = _pmc_traffic()
    valu_frac, valu_src = _pmc_valu()
    return {"kernel": "selective_scan_fwd (scan_fwd_pair_kernel, B/C rows read in-kernel) @ C4 B64 D3072 L4096 N16 bf16 z softplus",
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_unit": "bytes per launch",
            "traffic_source": traffic_src, "traffic_measured_in_this_run": False,
            # the kernel is VALU-issue bound, not HBM bound: VALU busy cycles / SIMD cycles (PMC)
            "valu_frac": valu_frac, "valu_frac_source": valu_src,
            "ms_per_call": round(ms, 4), "algorithmic_bytes": nbytes,
            # also report the achievable copy bandwidth measured on this box
            "copy_gbs_measured": round(copy_gbs, 1), "frac_of_copy": round(achieved / copy_gbs, 4)}


def _copy_bandwidth(dev, nbytes=2 << 30, iters=10):
    """Achievable streaming rate: the library's float4 non-temporal copy kernel (mc_stream_copy,
    include/mc_ops.h) over a 2 GiB buffer, read + write bytes / time, HIP events on its stream.
    (MI355X_MICROARCH.md measures 6.29 TB/s for a float4 copy; torch's copy_ runs slower.)"""
    import torch
    from mamba_clip_amd import _lib
    lib = _lib.load()
    src = torch.empty(nbytes // 2, dtype=torch.bfloat16, device=dev).normal_()
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream(dev)
    h = _lib.stream_handle(dev)
    copy = lambda: _lib.check(lib.mc_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, h),  # noqa: E731
                              "mc_stream_copy")
    for _ in range(2):
        copy()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    t0.record(stream)
    for _ in range(iters):
        copy()
    t1.record(stream)
    torch.cuda.synchronize(dev)
    ms = t0.elapsed_time(t1) / iters
    if not torch.equal(src[:1 << 20], dst[:1 << 20]):
        raise RuntimeError("mc_stream_copy: copy mismatch")
    del src, dst
    torch.cuda.empty_cache()
    return 2 * nbytes / (ms * 1e-3) / 1e9


def similarity_c5(iters=20, warmup=3):
    """Config 5 similarity matmul: gathered N = 1024 x 8 = 8192 frozen features, E = 512, fp8 MFMA.

    Times (HIP events on the launch stream) the row-wise e4m3 quantisation of both
    operands + the fp8 GEMM (fp32 logits), the fp8 GEMM alone, and the bf16 GEMM
    on the same features for comparison.  Algorithmic work: 2*N*N*E flop; the fp32
    logit write (N*N*4 B) is the HBM side of the roofline.
    """
    import torch
    import torch.nn.functional as F
    from mamba_clip_amd.ops import gemm_nt, quant_rows_fp8, similarity_fp8
    dev = torch.device("cuda", torch.cuda.current_device())
    n, e = 8192, 512
    g = torch.Generator(device=dev).manual_seed(5)
    I = F.normalize(torch.randn(n, e, device=dev, generator=g), dim=-1).bfloat16()
    T = F.normalize(torch.randn(n, e, device=dev, generator=g), dim=-1).bfloat16()
    scale = torch.tensor(100.0, device=dev)
    qi, si = quant_rows_fp8(I)
    qt, st = quant_rows_fp8(T)
    stream = torch.cuda.current_stream(dev)

    def timed(fn):
        for _ in range(warmup):
            fn()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        t0.record(stream)
        for _ in range(iters):
            fn()
        t1.record(stream)
        torch.cuda.synchronize(dev)
        return t0.elapsed_time(t1) / iters

    ms_all = timed(lambda: similarity_fp8(I, T, scale))
    ms_gemm = timed(lambda: gemm_nt(qi, qt, alpha_dev=scale, scale_a=si, scale_b=st))
    ms_gemm_bf16out = timed(lambda: gemm_nt(qi, qt, alpha_dev=scale, scale_a=si, scale_b=st, out_dtype=torch.bfloat16))
    ms_bf16 = timed(lambda: gemm_nt(I, T, alpha_dev=scale))
    # bf16 logits as shipped (similarity_fp8 -> the same panel kernel, bf16 epilogue), quantisation included
    ms_bf16_out = timed(lambda: similarity_fp8(I, T, scale, out_dtype=torch.bfloat16))
    flop = 2.0 * n * n * e
    tflops = flop / (ms_gemm * 1e-3) / 1e12
    tflops_b = flop / (ms_gemm_bf16out * 1e-3) / 1e12
    write_gbs = n * n * 4 / (ms_gemm * 1e-3) / 1e9
    return {"kernel": "mc_gemm_nt fp8 e4m3 -> sim8_panel_kernel (256-row A panel in registers, 64-column B tiles "
                      "by LDS-DMA, v_mfma_scale_f32_32x32x64_f8f6f4 with unit block scales, per-row / per-column "
                      "dequant factors in an LDS-staged epilogue) @ C5 N=8192 E=512",
            "vendor_kernels": False,
            "ms_quant_plus_gemm": round(ms_all, 4), "ms_gemm": round(ms_gemm, 4),
            "ms_gemm_bf16_logits": round(ms_gemm_bf16out, 4), "ms_quant_plus_gemm_bf16_logits": round(ms_bf16_out, 4),
            "ms_gemm_bf16_operands": round(ms_bf16, 4),
            "achieved_tflops": round(tflops, 1), "achieved_tflops_bf16_logits": round(tflops_b, 1),
            "peak_tflops_fp8_dense": MFMA_FP8_DENSE_TFLOPS,
            "frac_mfma": round(tflops / MFMA_FP8_DENSE_TFLOPS, 4),
            "logit_write_gbs": round(write_gbs, 1), "frac_hbm_write": round(write_gbs / HBM_PEAK_GBS, 4)}


def _pmc_traffic():
    """HBM bytes per launch of the same kernel at the same config, from the committed rocprofv3
    FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.sh; calibration in the JSON).  PMC counters
    cannot be read from inside a timed run, so the newest committed measurement is reported."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "scan_fwd_c4_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return (int(d["hbm_bytes"]) if d.get("hbm_bytes") else None), os.path.relpath(files[-1], ROOT)


def _pmc_valu():
    """VALU issue fraction of the same kernel at the same config: 4 * SQ_ACTIVE_INST_VALU
    (quad-cycles) / (1024 SIMDs * GRBM_GUI_ACTIVE / 8 XCDs), from the committed rocprofv3 pass
    (tools/pmc_valu.sh; counters and derivation in the JSON)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "scan_fwd_c4_valu.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return d.get("valu_frac"), os.path.relpath(files[-1], ROOT)


def _cpu_threads(args):
    """Host threads for the CPU baseline: --cpu-threads, else every CPU this process may run on
    (sched_getaffinity; os.cpu_count() when affinity is unavailable).  A GPU box that declares a
    smaller CPU share through OMP_NUM_THREADS gets that share (more threads than cores only
    oversubscribes them)."""
    if args.cpu_threads > 0:
        return args.cpu_threads
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(share)) if share.isdigit() and int(share) > 0 else n


def cpu_baseline(args, model_name):
    import torch
    from oracle.cpu_model import cpu_train_pairs_per_sec
    threads = _cpu_threads(args)
    prev = torch.get_num_threads()
    pps, secs = cpu_train_pairs_per_sec(model_name, batch=args.cpu_batch, steps=args.cpu_steps, warmup=1,
                                        threads=threads)
    torch.set_num_threads(prev)
    return {"value": round(pps, 4), "unit": "image-text pairs/sec", "cores": threads, "kind": "port",
            "sample": f"median of {args.cpu_steps} timed fp32 CPU train steps (+1 warmup) of {model_name} at "
                      f"batch {args.cpu_batch} via oracle/cpu_model.py ({secs:.1f} s timed)"}


def cpu_baseline_scan(args):
    """The scan half of the metric on the host: the oracle's restatement of the reference semantics
    (model.py:83-169) on one C4 sequence batch (B=1 of 64, D=3072, L=4096, N=16, bf16 I/O)."""
    import torch
    from oracle.cpu_model import cpu_scan_gbps
    threads = _cpu_threads(args)
    prev = torch.get_num_threads()
    gbs, secs = cpu_scan_gbps(batch=1, dim=3072, seqlen=4096, dstate=16, threads=threads)
    torch.set_num_threads(prev)
    return {"value": round(gbs, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"selective_scan fwd, oracle/scan_ref.py (reference semantics), B=1 x D=3072 x L=4096 x N=16 "
                      f"bf16 I/O, algorithmic bytes as the roofline ({secs:.1f} s)"}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args))

    import torch
    import torch.distributed as dist

    from mamba_clip_amd import _lib
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.loss import ClipLoss
    from mamba_clip_amd.model import build_clip
    from mamba_clip_amd.train import create_optimizer, train_step, wrap_ddp
    from mamba_clip_amd.tuning import load_gemm_tuning
    from mamba_clip_amd.utils import init_device

    _lib.load()                                   # fail loudly if the HIP library is missing
    targs = SimpleNamespace(precision="amp_bf16", lr=5e-4, wd=0.2, beta1=0.9, beta2=0.98, eps=1e-6,
                            grad_clip_norm=None, dist_backend="nccl", ddp_static_graph=True, accum_freq=1)
    device = init_device(targs)
    rank, world = targs.rank, targs.world_size
    gemm_tuned = load_gemm_tuning(model=args.model)   # committed per-shape hipBLASLt/rocBLAS selection
    targs.lr *= world                             # pipeline.py:532
    use_graph = args.graph == 1 or (args.graph == -1 and world == 1 and args.input == "resident")
    if use_graph and (world > 1 or args.input != "resident"):
        raise SystemExit("--graph 1 needs one process and resident inputs")
    targs.capturable = use_graph

    torch.manual_seed(0)
    model = build_clip(args.model).to(device)
    model = wrap_ddp(model, targs, device)
    optimizer = create_optimizer(model, targs)
    loss = ClipLoss(rank=rank, world_size=world)
    inner = model.module if hasattr(model, "module") else model
    images, texts, targets = synthetic_batch(args.batch, 224, inner.text.context_length, inner.text.vocab_size,
                                             device=device, seed=1000 + rank)
    model.train()
    if args.input == "host":
        # each rank streams its own shard: 8 batches of raw crops, cycled epoch after epoch
        from mamba_clip_amd.data import HostToDeviceLoader, IsicShapedDataset
        shard = IsicShapedDataset(8 * args.batch, 224, inner.text.context_length, inner.text.vocab_size,
                                  seed=1000 + rank)
        loader = HostToDeviceLoader(shard, args.batch, device, seed=rank)

        def batches():
            epoch = 0
            while True:
                loader.set_epoch(epoch)
                yield from loader
                epoch += 1
        feed = batches()

        def step():
            return train_step(model, *next(feed), loss, optimizer, None, targs)
    elif use_graph:
        from mamba_clip_amd.train import GraphedStep
        # the towers' two streams are captured as two graph branches (reproducible since round 6)
        step = GraphedStep(model, images, texts, targets, loss, optimizer, targs,
                           concurrent=bool(getattr(inner, "concurrent_towers", False)) and args.graph_streams == 2)
    else:
        def step():
            return train_step(model, images, texts, targets, loss, optimizer, None, targs)

    for _ in range(args.warmup):
        losses = step()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    stream = torch.cuda.current_stream(device)
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record(stream)
    for k in range(args.steps):
        losses = step()
        marks[k + 1].record(stream)          # per-step HIP events: no host sync inside the timed loop
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    final_loss = float(losses["loss"].item())
    if not math.isfinite(final_loss):
        raise RuntimeError(f"non-finite training loss {final_loss}")

    step_ms = sorted(marks[k].elapsed_time(marks[k + 1]) for k in range(args.steps))
    median_ms = step_ms[len(step_ms) // 2] if len(step_ms) % 2 else 0.5 * (step_ms[len(step_ms) // 2 - 1]
                                                                             + step_ms[len(step_ms) // 2])
    value = world * args.batch * args.steps / elapsed
    seq_len = int(inner.text.context_length)
    workload, flop_pair = WORKLOADS.get(args.model, (f"{args.model}: contrastive train step (fwd+bwd+AdamW), "
                                                     "amp_bf16", C2_FLOP_PER_PAIR))
    result = {
        "metric": "image-text pairs/sec (whole node) + selective_scan HBM GB/s",
        "value": round(value, 2), "unit": "image-text pairs/sec", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "median_ms_per_step": round(median_ms, 3),
        "median_pairs_per_sec": round(world * args.batch / (median_ms * 1e-3), 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": (f"synthetic (random-init weights; N(0,1) 224x224 images, U[1,vocab) {seq_len}-token text, EOT last)"
                 if args.input == "resident" else
                 f"synthetic ISIC-shaped shard streamed from pinned host memory each step (raw 224x224x3 uint8 "
                 f"crops normalised on the GPU, U[1,vocab) {seq_len}-token text; random-init weights)"),
        "config": {"workload": workload,
                   "model": args.model, "global_batch": world * args.batch, "per_gpu_batch": args.batch,
                   "seq_len": seq_len, "image_size": 224, "input": args.input,
                   "step_launch": (f"hip-graph replay ({args.graph_streams} streams)" if use_graph else "eager"),
                   "parallelism": f"dp{world}",
                   "library_gemm_selection": "tunableop-file" if gemm_tuned else "default-heuristic"},
        "mfma_estimate": {"flop_per_pair": flop_pair,
                          "achieved_tflops_per_gpu": round(value / world * flop_pair / 1e12, 1),
                          "peak": MFMA_BF16_DENSE_TFLOPS,
                          "frac": round(value / world * flop_pair / 1e12 / MFMA_BF16_DENSE_TFLOPS, 4)},
        "final_loss": round(final_loss, 5),
    }
    if args.input == "host":
        feed.close()                              # joins the loader's host thread
    del images, texts, targets, optimizer
    torch.cuda.empty_cache()
    if rank == 0 and not args.no_roofline:
        result["roofline"] = scan_roofline(args.scan_iters)
    if rank == 0 and not args.no_roofline:
        result["similarity_fp8"] = similarity_c5()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, args.model)
        result["cpu_baseline_scan"] = cpu_baseline_scan(args)
    if world > 1:
        dist.barrier()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
