"""Stage-1 CLIP training step on MI355X (reference: src/mamba_clip/train.py:92-372, pipeline.py:266-311).

One optimizer step = scheduler(step) -> zero_grad -> autocast forward of both
towers -> ClipLoss (HIP contrastive kernels, RCCL feature all-gather) ->
backward (DDP bucketed RCCL all-reduce overlapped with the tail of backward)
-> optional grad clip -> AdamW -> logit_scale.clamp_(0, ln 100).

Batches are either (images, texts, targets) / (images, targets), or -- with
--balanced-mixup -- the ComboLoader pair ((images, texts, targets),
(bal_images, bal_texts, bal_targets)) as train.py:131-151 unpacks it.

Differences from the reference are deliberate fixes:
balanced-mixup variables are only touched when balanced mixup is on (A.1:
the reference raises UnboundLocalError without it), and the accumulation path
passes the concatenated features to the loss (the reference builds `inputs`
and then ignores it).  Everything the reference computes is kept, including
that get_model_inputs mixes the one-hot targets but returns only the model
inputs, so the loss sees the original targets (train.py:66-89, 189).
"""
import logging
import math
import os
import time

import numpy as np
import torch
import torch.nn.functional as F

from .data import normalize_images
from .optim import HipAdamW
from .utils.amp_utils import get_autocast, get_input_dtype
from .utils.dist_utils import is_master


class AverageMeter:
    def __init__(self):
        self.reset()

    def reset(self):
        self.val = self.avg = self.sum = 0.0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


def unwrap_model(model):
    return model.module if hasattr(model, "module") else model


def postprocess_clip_output(model_out):
    return {"image_features": model_out[0], "text_features": model_out[1], "logit_scale": model_out[2]}


def backward(total_loss, scaler):
    if scaler is not None:
        scaler.scale(total_loss).backward()
    else:
        total_loss.backward()


def get_model_inputs(args, images, texts, targets=None, balanced_images=None, balanced_texts=None,
                     balanced_targets=None):
    """train.py:66-89: optional balanced mixup, then (images,) or (images, texts)."""
    if getattr(args, "balanced_mixup", None):
        lam = np.random.beta(a=args.balanced_mixup, b=1)
        if images.dtype == torch.uint8:   # raw crops: mix the normalised images (the reference mixes those)
            images, balanced_images = normalize_images(images), normalize_images(balanced_images)
        images = (1 - lam) * images + lam * balanced_images
        if lam > 0.5 and texts is not None and balanced_texts is not None:
            texts = balanced_texts
        n_classes = args.num_classes
        targets = F.one_hot(targets, n_classes)
        targets = (1 - lam) * targets + lam * F.one_hot(balanced_targets, n_classes)
    return (images,) if texts is None else (images, texts)


# ---------------------------------------------------------------- optimizer / DDP (pipeline.py:266-311)
def _no_decay(name, p):
    return p.ndim < 2 or "bn" in name or "ln" in name or "bias" in name or "logit_scale" in name


HIP_ADAMW = os.environ.get("MAMBA_CLIP_AMD_HIP_ADAMW", "1") != "0"   # A/B toggle (torch fused AdamW when 0)


def create_optimizer(model, args):
    """AdamW with two groups: gains/biases/logit_scale at wd 0, the rest at args.wd.

    On the GPU the fused (single multi-tensor kernel) AdamW is used: same update
    rule as torch.optim.AdamW's foreach path, one launch per step.
    """
    named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
    groups = [{"params": [p for n, p in named if _no_decay(n, p)], "weight_decay": 0.0},
              {"params": [p for n, p in named if not _no_decay(n, p)], "weight_decay": args.wd}]
    on_gpu = all(p.is_cuda for _, p in named)
    capturable = bool(on_gpu and getattr(args, "capturable", False))
    if on_gpu and not capturable and HIP_ADAMW and all(p.dtype == torch.float32 for _, p in named):
        # one HIP launch over every parameter (optim.HipAdamW, mc_adamw_step): same rule and state layout
        return HipAdamW(groups, lr=args.lr, betas=(args.beta1, args.beta2), eps=args.eps)
    # capturable: the step counts live on the device, so a HIP-graph replay (GraphedStep) advances them
    return torch.optim.AdamW(groups, lr=args.lr, betas=(args.beta1, args.beta2), eps=args.eps,
                             fused=True if on_gpu else None,
                             capturable=capturable)


def create_scaler(args, device):
    if args.precision != "amp":
        return None
    return torch.amp.GradScaler("cuda" if device.type == "cuda" else "cpu")


def wrap_ddp(model, args, device):
    """One process per GPU; gradients all-reduced over RCCL in 100 MB buckets during backward."""
    if not getattr(args, "distributed", False):
        return model
    kw = dict(static_graph=getattr(args, "ddp_static_graph", False), gradient_as_bucket_view=True,
              bucket_cap_mb=getattr(args, "ddp_bucket_mb", 100))
    if device.type == "cuda":
        kw["device_ids"] = [device]
    # MAMBA_CLIP_AMD_DDP_SIDE_STREAM=0 keeps the towers on one stream under DDP (the two-stream comm hook
    # below is covered by gloo tests; ADVICE r04 asks for a switch until an RCCL run has covered it)
    two = os.environ.get("MAMBA_CLIP_AMD_DDP_SIDE_STREAM", "1") != "0"
    side = model.side_stream_for(device) if (two and device.type == "cuda" and hasattr(model, "side_stream_for")) else None
    if side is not None and hasattr(model, "side_tower_module"):
        # DDP keeps every parameter's AccumulateGrad node alive from here on, and a node runs on the
        # stream current at its creation.  Created now on the main stream, each text-tower gradient
        # would make the main stream wait for the side stream's backward at that point (autograd's
        # stream-mismatch sync), serialising the towers again; created under the side stream, the
        # text tower's gradients are accumulated (and DDP's bucket copies made) where they are produced.
        with torch.cuda.stream(side):
            model._side_grad_accumulators = [p.view_as(p).grad_fn.next_functions[0][0]
                                             for p in model.side_tower_module().parameters() if p.requires_grad]
    ddp = torch.nn.parallel.DistributedDataParallel(model, **kw)
    if side is not None:
        # ClipModel runs its text tower on a second stream; a bucket may then hold gradients written
        # on either stream, so its all-reduce is launched behind both
        ddp.register_comm_hook((torch.cuda.current_stream(device), model), _join_streams_allreduce)
        model.ddp_streams_joined = True
    return ddp


def _join_streams_allreduce(state, bucket):
    """DDP comm hook: the launching stream waits for the forward's main stream and the side stream
    (events at this point), then the stock averaging all-reduce of the bucket.  Both streams are
    resolved at call time: the main one as the last forward recorded it, the side one as the model
    picks it now (the wrap-time stream is only the fallback)."""
    from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
    main_at_wrap, model = state
    dev = bucket.buffer().device
    main = getattr(model, "last_main_stream", None) or main_at_wrap
    # the join happens on a third stream: neither tower's stream is held up waiting for the other
    join = _comm_join_stream(dev)
    join.wait_stream(main)
    join.wait_stream(model.side_stream_for(dev))
    bucket.buffer().record_stream(join)
    with torch.cuda.stream(join):
        return default_hooks.allreduce_hook(None, bucket)


_JOIN_STREAMS = {}


def _comm_join_stream(dev):
    key = torch.device(dev)
    if key not in _JOIN_STREAMS:
        _JOIN_STREAMS[key] = torch.cuda.Stream(device=key)
    return _JOIN_STREAMS[key]


# ---------------------------------------------------------------- one optimizer step
def _loss_terms(loss, model_out, targets):
    if isinstance(model_out, dict) and "logits" in model_out:
        model_out = {"input": model_out["logits"]}
    elif not isinstance(model_out, dict):
        model_out = {"input": model_out}
    losses = loss(**model_out, target=targets)
    if isinstance(losses, dict):
        total = sum(losses.values())
        losses["loss"] = total
    else:
        total, losses = losses, {"loss": losses}
    return total, losses


def optimizer_step(model, optimizer, scaler, args):
    """train.py:292-315: (unscale, clip,) step, then clamp logit_scale to [0, ln 100]."""
    clip = getattr(args, "grad_clip_norm", None)
    if scaler is not None:
        if clip is not None:
            scaler.unscale_(optimizer)
            torch.nn.utils.clip_grad_norm_(model.parameters(), clip, norm_type=2.0)
        scaler.step(optimizer)
        scaler.update()
    else:
        if clip is not None:
            torch.nn.utils.clip_grad_norm_(model.parameters(), clip, norm_type=2.0)
        optimizer.step()
    inner = unwrap_model(model)
    if hasattr(inner, "logit_scale"):
        with torch.no_grad():
            inner.logit_scale.clamp_(0, math.log(100))


def split_batch(batch, balanced_mixup):
    """train.py:131-157: -> (images, texts, targets, balanced) with balanced = (img, txt, tgt) or None."""
    def unpack(b):
        return (b[0], b[1], b[2]) if len(b) == 3 else (b[0], None, b[1])
    if balanced_mixup:
        return unpack(batch[0]) + (unpack(batch[1]),)
    return unpack(batch) + (None,)


def _balanced_to(balanced, device, input_dtype):
    if balanced is None:
        return None
    img, txt, tgt = balanced
    return (_images_to(img, device, input_dtype), txt.to(device=device) if txt is not None else None,
            tgt.to(device=device))


def _images_to(images, device, input_dtype):
    """Float batches take the input dtype; raw uint8 crops stay bytes (normalised in the patch kernel)."""
    dt = input_dtype if images.is_floating_point() else None
    return images.to(device=device, dtype=dt, non_blocking=True)


def train_step(model, images, texts, targets, loss, optimizer, scaler, args, autocast=None, balanced=None):
    """One accum_freq == 1 step on device-resident inputs; returns the loss dict (device tensors).

    balanced: the balanced-mixup partner batch (images, texts, targets), required
    when args.balanced_mixup is set (train.py:131-151, 169-177).
    """
    autocast = autocast or get_autocast(args.precision)
    if getattr(args, "balanced_mixup", None) and balanced is None:
        raise ValueError("balanced_mixup needs the paired balanced batch ((img, txt, tgt), (bal_img, bal_txt, bal_tgt))")
    optimizer.zero_grad(set_to_none=True)
    with autocast():
        model_out = model(*get_model_inputs(args, images, texts, targets, *(balanced or (None, None, None))))
        total, losses = _loss_terms(loss, model_out, targets)
    backward(total, scaler)
    optimizer_step(model, optimizer, scaler, args)
    return losses


class GraphedStep:
    """train_step (forward, ClipLoss, backward, AdamW, logit-scale clamp) on fixed device inputs,
    captured once as a HIP graph and replayed: at small per-GPU batches the step is bound by the host
    launching ~1000 kernels (C3 b 64: 4.4 ms of a 34 ms step idle in the kernel trace).  Every kernel of
    the eager step runs in the replay (nothing is cached across steps); the optimizer must be
    capturable (device-side step counts: create_optimizer with args.capturable), single-process only
    (DDP's bucketed all-reduce stays eager).  Replays write the same buffers: `losses` holds the loss
    dict of the latest replay."""

    @staticmethod
    def autocast_for(args):
        """The step's autocast without the weight-cast cache (not capture-safe: cached casts would
        outlive the capture's pool); numerically the same casts."""
        if not args.precision.startswith("amp"):
            return None
        dt = torch.bfloat16 if args.precision in ("amp_bf16", "amp_bfloat16") else torch.float16
        return lambda: torch.autocast("cuda", dtype=dt, cache_enabled=False)

    def __init__(self, model, images, texts, targets, loss, optimizer, args, warmup=3, concurrent=False):
        if getattr(args, "balanced_mixup", None):
            # the mixup draws lam (and the lam > 0.5 text swap) on the host: a replay would repeat the
            # capture's draw forever
            raise ValueError("GraphedStep: balanced_mixup draws host-side randomness per step; run it eager")
        if concurrent and os.environ.get("GPU_MAX_HW_QUEUES", "").strip() == "1":
            # Capturing the towers' fork / join with both streams on one hardware queue ended the process
            # with SIGSEGV inside the HIP runtime's capture path (round 5); one hardware queue
            # serialises the two streams anyway, so the one-stream capture loses nothing there.
            raise ValueError("GraphedStep(concurrent=True) is not supported with GPU_MAX_HW_QUEUES=1 "
                             "(the two streams share one hardware queue): use concurrent=False")
        autocast = self.autocast_for(args)
        inner = unwrap_model(model)
        # One stream by default: replay order = eager order, and the replays are bitwise repeatable.
        # concurrent=True captures the towers' two-stream fork / join as two graph branches; since the
        # round-6 scan fix two captures replay to the same bits and track the eager
        # two-stream step to the one-stream bounds (tests/test_graph_gpu.py).  The flag is restored after
        # the capture, so later eager steps run the towers concurrently again.
        prev = getattr(inner, "concurrent_towers", False)
        if not concurrent:
            inner.concurrent_towers = False
        run = lambda: train_step(model, images, texts, targets, loss, optimizer, None, args, autocast)  # noqa: E731
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):        # warmup off the default stream (lazy state, allocator pools)
            for _ in range(warmup):
                run()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        optimizer.zero_grad(set_to_none=True)     # gradients are allocated inside the capture's pool
        try:
            with torch.cuda.graph(self.graph):
                self.losses = run()
        finally:
            if hasattr(inner, "concurrent_towers"):
                inner.concurrent_towers = prev

    def __call__(self):
        self.graph.replay()
        return self.losses


def train_step_accum(model, batches, loss, optimizer, scaler, args, autocast=None):
    """Gradient-cache accumulation over `batches` (train.py:218-291).

    Features of every micro-batch are computed without grad; then each micro-batch
    is re-run with grad and its loss uses the other micro-batches' cached
    features as extra negatives.  A batch is (images, texts, targets) or, with
    balanced mixup, (images, texts, targets, balanced); the mixup is drawn in the
    caching pass (the reference re-draws it in the re-run too, from stale
    balanced tensors: train.py:249-257).
    """
    autocast = autocast or get_autocast(args.precision)
    cached = {}
    mixed = []
    with torch.no_grad(), autocast():
        for batch in batches:
            images, texts, targets = batch[:3]
            bal = batch[3] if len(batch) > 3 else None
            inp = get_model_inputs(args, images, texts, targets, *(bal or (None, None, None)))
            mixed.append(inp)
            out = model(*inp)
            for k, v in out.items():
                if k not in ("logit_scale", "logit_bias"):
                    cached.setdefault(k, []).append(v)
    optimizer.zero_grad(set_to_none=True)
    losses = None
    for j, batch in enumerate(batches):
        targets = batch[2]
        with autocast():
            out = model(*mixed[j])
            inputs = {k: out[k] for k in ("logit_scale", "logit_bias") if k in out}
            for k, vals in cached.items():
                inputs[k] = torch.cat(vals[:j] + [out[k]] + vals[j + 1:])
            total, losses = _loss_terms(loss, inputs, targets)
        backward(total, scaler)
    optimizer_step(model, optimizer, scaler, args)
    return losses


def train_one_epoch(model, data, loss, epoch, optimizer, scaler, scheduler, args, tb_writer=None):
    """Epoch loop with the reference's logging cadence (samples/s per GPU and whole job)."""
    device = torch.device(args.device)
    autocast = get_autocast(args.precision)
    input_dtype = get_input_dtype(args.precision)
    model.train()
    data["train"].set_epoch(epoch)
    dataloader = data["train"].dataloader
    accum = getattr(args, "accum_freq", 1)
    num_batches_per_epoch = dataloader.num_batches // accum
    batch_time_m, data_time_m, losses_m = AverageMeter(), AverageMeter(), {}
    pending = []
    end = time.time()
    for i, batch in enumerate(dataloader):
        i_accum = i // accum
        step = num_batches_per_epoch * epoch + i_accum
        if scheduler is not None and not getattr(args, "skip_scheduler", False):
            scheduler(step)
        images, texts, targets, balanced = split_batch(batch, getattr(args, "balanced_mixup", None))
        balanced = _balanced_to(balanced, device, input_dtype)
        images = _images_to(images, device, input_dtype)
        texts = texts.to(device=device, non_blocking=True) if texts is not None else None
        targets = targets.to(device=device, non_blocking=True)
        data_time_m.update(time.time() - end)
        if accum == 1:
            losses = train_step(model, images, texts, targets, loss, optimizer, scaler, args, autocast, balanced)
        else:
            pending.append((images, texts, targets, balanced))
            if (i + 1) % accum:
                continue
            losses = train_step_accum(model, pending, loss, optimizer, scaler, args, autocast)
            pending = []
        batch_time_m.update(time.time() - end)
        end = time.time()
        batch_count = i_accum + 1
        if is_master(args) and (i_accum % getattr(args, "log_every_n_steps", 100) == 0
                                or batch_count == num_batches_per_epoch):
            bs = len(images)
            for k, v in losses.items():
                losses_m.setdefault(k, AverageMeter()).update(v.item(), bs)
            per_gpu = accum * bs / max(batch_time_m.val, 1e-9)
            logging.info(
                f"Train Epoch: {epoch} [{batch_count}/{num_batches_per_epoch}] "
                f"Data (t): {data_time_m.avg:.3f} Batch (t): {batch_time_m.avg:.3f}, "
                f"{per_gpu * args.world_size:#g}/s, {per_gpu:#g}/s/gpu "
                f"LR: {optimizer.param_groups[0]['lr']:5f} "
                + " ".join(f"{k}: {m.val:#.5g} ({m.avg:#.5g})" for k, m in losses_m.items()))
            if tb_writer is not None:
                tb_writer.add_scalar("train/samples_per_second", per_gpu * args.world_size, step)
            batch_time_m.reset()
            data_time_m.reset()
    return {k: m.avg for k, m in losses_m.items()}
