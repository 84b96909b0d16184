"""ClipLoss -- drop-in for /root/reference/src/mamba_clip/loss.py on MI355X.

Same names, arguments and outputs as the reference:
  create_loss(args)                                  loss.py:6-13
  all_gather(img, txt, local_loss, gather_with_grad, rank, world_size)   loss.py:16-44
  cross_entropy_loss(input, target, weight=None)     loss.py:47-53
  ClipLoss(local_loss, gather_with_grad, cache_labels, rank, world_size)
      .get_ground_truth(device, num_logits)          loss.py:76-87
      .get_logits(image_features, text_features, logit_scale)   loss.py:89-113
      .forward(image_features, text_features, logit_scale, output_dict=True, target=None)
                                                     loss.py:124-147
What changes is HOW: the features are gathered with ONE RCCL all_gather per
step (image and text stacked), the logits come from the MFMA GEMM of
libmamba_clip_amd.so with logit_scale read on the device, and both softmax
cross-entropies (and their gradients, incl. d logit_scale) are fused kernels
over the fp32 logits -- no host sync, no eager softmax.
"""
import torch
import torch.distributed as dist
import torch.distributed.nn  # noqa: F401  (gather_with_grad; the reference forgets it: SURVEY Appendix A.4)
import torch.nn.functional as F

from .ops import gemm_nt, scaled_logits_ce


def create_loss(args):
    return ClipLoss(
        local_loss=args.local_loss,
        gather_with_grad=args.gather_with_grad,
        cache_labels=True,
        rank=args.rank,
        world_size=args.world_size,
    )


def _gather_stacked(image_features, text_features, world_size):
    """One all_gather of the stacked (2, b, E) features (no autograd)."""
    b = image_features.shape[0]
    stacked = torch.stack([image_features.detach(), text_features.detach()]).contiguous()   # (2, b, E)
    out = torch.empty((world_size * 2,) + tuple(stacked.shape[1:]), device=stacked.device, dtype=stacked.dtype)
    dist.all_gather_into_tensor(out, stacked)          # concatenated along dim 0: rank-major
    out = out.view(world_size, 2, b, -1)
    imgs = out[:, 0].reshape(world_size * b, -1)
    txts = out[:, 1].reshape(world_size * b, -1)
    return imgs, txts


def all_gather(image_features, text_features, local_loss=False, gather_with_grad=False, rank=0, world_size=1):
    """Gather features from every rank (loss.py:16-44 semantics).

    gather_with_grad: autograd-aware gather (backward reduces the feature
    gradients back to their owners).  Otherwise a plain gather whose local
    slice is re-inserted so gradients flow through the local features
    (unless local_loss, where the gathered copies stay gradient-free).
    """
    if gather_with_grad:
        all_image = torch.cat(torch.distributed.nn.all_gather(image_features), dim=0)
        all_text = torch.cat(torch.distributed.nn.all_gather(text_features), dim=0)
        return all_image, all_text
    imgs, txts = _gather_stacked(image_features, text_features, world_size)
    if not local_loss:
        b = image_features.shape[0]
        imgs = torch.cat([imgs[: rank * b], image_features, imgs[(rank + 1) * b:]], dim=0)
        txts = torch.cat([txts[: rank * b], text_features, txts[(rank + 1) * b:]], dim=0)
    return imgs, txts


def cross_entropy_loss(input, target, weight=None):
    """Soft (float targets, e.g. balanced-mixup one-hots) or hard-label CE (loss.py:47-53)."""
    if target.dtype in (torch.float, torch.double):
        return -(input.log_softmax(dim=-1) * target).sum(dim=-1).mean()
    return F.cross_entropy(input, target, weight=weight)


class ClipLoss(torch.nn.Module):
    def __init__(self, local_loss=False, gather_with_grad=False, cache_labels=False, rank=0, world_size=1):
        super().__init__()
        self.local_loss = local_loss
        self.gather_with_grad = gather_with_grad
        self.cache_labels = cache_labels
        self.rank = rank
        self.world_size = world_size
        self.prev_num_logits = 0
        self.labels = {}

    def get_ground_truth(self, device, num_logits) -> torch.Tensor:
        if self.prev_num_logits != num_logits or device not in self.labels:
            labels = torch.arange(num_logits, device=device, dtype=torch.long)
            if self.world_size > 1 and self.local_loss:
                labels = labels + num_logits * self.rank
            if self.cache_labels:
                self.labels[device] = labels
                self.prev_num_logits = num_logits
        else:
            labels = self.labels[device]
        return labels

    def _features(self, image_features, text_features):
        if self.world_size > 1:
            return all_gather(image_features, text_features, self.local_loss, self.gather_with_grad,
                              self.rank, self.world_size)
        return image_features, text_features

    def get_logits(self, image_features, text_features, logit_scale):
        """Materialised (logits_per_image, logits_per_text), as the reference returns them."""
        scale = logit_scale.reshape(()).float()
        dt = image_features.dtype if image_features.dtype == torch.bfloat16 else torch.float32
        if self.world_size > 1:
            all_i, all_t = self._features(image_features, text_features)
            if self.local_loss:
                li = gemm_nt(image_features.to(dt), all_t.to(dt), alpha_dev=scale)
                lt = gemm_nt(text_features.to(dt), all_i.to(dt), alpha_dev=scale)
            else:
                li = gemm_nt(all_i.to(dt), all_t.to(dt), alpha_dev=scale)
                lt = li.T
        else:
            li = gemm_nt(image_features.to(dt), text_features.to(dt), alpha_dev=scale)
            lt = li.T
        return li, lt

    def forward(self, image_features, text_features, logit_scale, output_dict=True, target=None):
        # `target` is accepted and ignored, as in the reference (loss.py:136-140)
        if self.world_size > 1 and self.local_loss:
            all_i, all_t = self._features(image_features, text_features)
            b = image_features.shape[0]
            off = b * self.rank
            coef = 0.5 / b
            loss = (scaled_logits_ce(image_features, all_t, logit_scale, off, coef)
                    + scaled_logits_ce(text_features, all_i, logit_scale, off, coef))
        else:
            all_i, all_t = self._features(image_features, text_features)
            n = all_i.shape[0]
            loss = scaled_logits_ce(all_i, all_t, logit_scale, 0, 0.5 / n, 0, 0.5 / n)
        # the fused kernels use label(i) = i (+ b*rank for local_loss), i.e. exactly
        # get_ground_truth's arange; keep its cache state as the reference does
        local = self.world_size > 1 and self.local_loss
        self.get_ground_truth(image_features.device, image_features.shape[0] if local else all_i.shape[0])
        return {"contrastive_loss": loss} if output_dict else loss
