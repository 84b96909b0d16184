"""`mamba-clip` entry point for the hot path (reference: src/mamba_clip/cli/main.py:123-533, pipeline.py).

Keeps the reference's training flags that act on the contrastive step
(optimizer, schedule, precision, stage-1/stage-2 model, tower locking,
local_loss / gather_with_grad, accumulation, DDP) and adds --synthetic
(device-resident synthetic batches of the configured shapes; the CSV/HDF5
data pipeline is out of scope) and --benchmark (print one JSON
throughput line).  Launch multi-GPU with torch.distributed.run.
"""
import argparse
import json
import logging
import math
import sys
import time

import torch


def build_parser():
    p = argparse.ArgumentParser("mamba-clip", description=__doc__.split("\n")[0])
    p.add_argument("--data-path", type=str, default=None, help="CSV data path (not supported: use --synthetic)")
    p.add_argument("--synthetic", action="store_true", help="device-resident synthetic batches")
    p.add_argument("--train-num-samples", type=int, default=None,
                   help="samples per epoch (synthetic: default 16 batches)")
    p.add_argument("--num-classes", type=int, default=2)
    p.add_argument("--balanced-mixup", type=float, default=None)
    p.add_argument("--device", type=str, default="cuda")
    p.add_argument("--workers", type=int, default=0, help="accepted for compatibility (no loader workers)")
    p.add_argument("--batch-size", type=int, default=64, help="per-GPU batch size")
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--epochs-cooldown", type=int, default=None)
    p.add_argument("--lr", type=float, default=5e-4)
    p.add_argument("--beta1", type=float, default=0.9)
    p.add_argument("--beta2", type=float, default=0.98)
    p.add_argument("--eps", type=float, default=1e-6)
    p.add_argument("--wd", type=float, default=0.2)
    p.add_argument("--warmup", type=int, default=0, help="warmup steps")
    p.add_argument("--skip-scheduler", action="store_true")
    p.add_argument("--lr-scheduler", type=str, default="cosine", choices=["cosine", "const", "const-cooldown"])
    p.add_argument("--lr-restart-interval", type=int, default=None)
    p.add_argument("--lr-cooldown-end", type=float, default=0.0)
    p.add_argument("--lr-cooldown-power", type=float, default=1.0)
    p.add_argument("--precision", type=str, default="amp_bf16",
                   choices=["amp", "amp_bf16", "amp_bfloat16", "bf16", "pure_bf16", "fp16", "pure_fp16", "fp32"])
    p.add_argument("--stage", type=int, default=1, choices=[1, 2])
    p.add_argument("--model", type=str, default="vit_b16-mamba130m",
                   help="stage-1 model config (offline: vit_b16-mamba130m, tiny-mamba-clip, mamba790m-text, "
                        "biomedclip-vit_b16-pubmedbert256)")
    p.add_argument("--model-stage-1", type=str, default=None, help="alias of --model for stage 2")
    p.add_argument("--model-stage-2", type=str, default="ClipClassifier")
    p.add_argument("--use-inner-prod", action="store_true")
    p.add_argument("--use-visual-only", action="store_true")
    p.add_argument("--use-text-only", action="store_true")
    p.add_argument("--lock-image", action="store_true")
    p.add_argument("--lock-text", action="store_true")
    p.add_argument("--lock-text-unlocked-layers", type=int, default=0)
    p.add_argument("--lock-text-freeze-layer-norm", action="store_true")
    p.add_argument("--grad-checkpointing", action="store_true")
    p.add_argument("--local-loss", action="store_true")
    p.add_argument("--gather-with-grad", action="store_true")
    p.add_argument("--accum-freq", type=int, default=1)
    p.add_argument("--dist-url", type=str, default="env://")
    p.add_argument("--dist-backend", type=str, default="nccl")
    p.add_argument("--ddp-static-graph", action="store_true")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--grad-clip-norm", type=float, default=None)
    p.add_argument("--log-every-n-steps", type=int, default=10)
    p.add_argument("--benchmark", action="store_true", help="print one JSON throughput line at the end")
    return p


def _make_scheduler(optimizer, args, total_steps):
    from ..scheduler import const_lr, const_lr_cooldown, cosine_lr
    if args.lr_scheduler == "cosine":
        return cosine_lr(optimizer, args.lr, args.warmup, total_steps, args.lr_restart_interval)
    if args.lr_scheduler == "const":
        return const_lr(optimizer, args.lr, args.warmup, total_steps, args.lr_restart_interval)
    if args.epochs_cooldown is None:
        raise ValueError("--lr-scheduler const-cooldown needs --epochs-cooldown")
    cooldown = (total_steps // max(args.epochs, 1)) * args.epochs_cooldown
    return const_lr_cooldown(optimizer, args.lr, args.warmup, total_steps, cooldown, args.lr_restart_interval,
                             args.lr_cooldown_power, args.lr_cooldown_end)


def build_model(args, device):
    from ..model import ClipClassifier, init_model
    name = args.model_stage_1 or args.model
    model, _, _, _ = init_model(name)
    if args.stage == 1:
        if args.lock_image:
            model.lock_image_tower()
        if args.lock_text:
            model.lock_text_tower(args.lock_text_unlocked_layers, args.lock_text_freeze_layer_norm)
        if args.grad_checkpointing:
            model.set_grad_checkpointing(True)
        return model.to(device)
    for p in model.parameters():          # stage 2: frozen stage-1 towers + MLP head
        p.requires_grad_(False)
    head = ClipClassifier(model, num_classes=args.num_classes, use_visual_only=args.use_visual_only,
                          use_text_only=args.use_text_only, use_inner_prod=args.use_inner_prod)
    return head.to(device)


def main(argv=None):
    args = build_parser().parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(message)s")
    if not args.synthetic:
        raise SystemExit("mamba-clip: only --synthetic data is supported by this build (data pipeline is out of scope)")

    from .. import _lib
    from ..data import get_synthetic_data
    from ..loss import ClipLoss, cross_entropy_loss
    from ..train import create_optimizer, create_scaler, train_one_epoch, wrap_ddp
    from ..tuning import load_gemm_tuning
    from ..utils import init_device, is_master

    _lib.load()
    device = init_device(args)
    load_gemm_tuning(model=getattr(args, "model_stage_1", None) or getattr(args, "model", None))
    torch.manual_seed(args.seed + args.rank)
    model = build_model(args, device)
    inner = model.clip_model if args.stage == 2 else model
    text = inner.text
    args.lr *= args.world_size                                    # pipeline.py:532
    model = wrap_ddp(model, args, device)
    optimizer = create_optimizer(model, args)
    scaler = create_scaler(args, device)
    if args.stage == 1:
        loss = ClipLoss(local_loss=args.local_loss, gather_with_grad=args.gather_with_grad, cache_labels=True,
                        rank=args.rank, world_size=args.world_size)
    else:
        loss = cross_entropy_loss
    n_batches = max(1, (args.train_num_samples or 16 * args.batch_size) // args.batch_size)
    img_size = getattr(inner.visual, "patch_embed", None)
    img_size = img_size.grid * img_size.patch if img_size is not None else 224
    data = get_synthetic_data(args.batch_size, n_batches, img_size, text.context_length, text.vocab_size, device,
                              seed=1000 + args.rank, balanced=args.balanced_mixup is not None,
                              num_classes=args.num_classes)
    total_steps = n_batches // args.accum_freq * args.epochs
    scheduler = _make_scheduler(optimizer, args, total_steps)

    t0 = time.time()
    for epoch in range(args.epochs):
        metrics = train_one_epoch(model, data, loss, epoch, optimizer, scaler, scheduler, args)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    elapsed = time.time() - t0
    if is_master(args):
        pairs = args.batch_size * n_batches * args.epochs * args.world_size
        logging.info(f"done: {pairs} pairs in {elapsed:.2f} s ({pairs / elapsed:.1f} pairs/s); {metrics}")
        if args.benchmark:
            print(json.dumps({"pairs_per_sec": pairs / elapsed, "seconds": elapsed, "world_size": args.world_size,
                              "final": {k: (v if math.isfinite(v) else None) for k, v in metrics.items()}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
