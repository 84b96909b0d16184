"""Out-of-bounds write screen for every HIP kernel of the training step (tests/guard_alloc.py): each
device buffer the package's Python layer allocates (kernel outputs and workspaces) sits between two
64 KB sentinel bands; a full forward + ClipLoss + backward + AdamW step at the real tower widths must
leave every band intact.  With two HIP streams an out-of-bounds write lands in whatever the other
tower has allocated next to it, at a time that varies run to run -- the failure mode of a
cross-stream nondeterminism hunt."""
import pytest
import torch

from guard_alloc import check, guarded

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _modules():
    from mamba_clip_amd import loss, ops, optim, selective_scan_interface
    return [ops, selective_scan_interface, loss, optim]


@pytest.mark.parametrize("name,batch", [("vit_b16-mamba130m", 16), ("biomedclip-vit_b16-pubmedbert256", 8)])
@pytest.mark.parametrize("concurrent", [False, True])
def test_training_step_writes_stay_in_bounds(name, batch, concurrent):
    from types import SimpleNamespace
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.loss import ClipLoss
    from mamba_clip_amd.model import build_clip
    from mamba_clip_amd.train import create_optimizer, train_step
    torch.manual_seed(0)
    model = build_clip(name).to(DEV)
    model.concurrent_towers = concurrent
    args = SimpleNamespace(precision="amp_bf16", lr=5e-4, wd=0.2, beta1=0.9, beta2=0.98, eps=1e-6,
                           grad_clip_norm=None, accum_freq=1)
    opt = create_optimizer(model, args)
    images, texts, targets = synthetic_batch(batch, 224, model.text.context_length, model.text.vocab_size,
                                             device=DEV, seed=5)
    with guarded(_modules()) as log:
        for _ in range(2):    # the second step also runs the transposed weight copies
            losses = train_step(model, images, texts, targets, ClipLoss(), opt, None, args)
        torch.cuda.synchronize()
    assert len(log) > 100, f"only {len(log)} guarded allocations: the proxy is not in the allocation path"
    bad = check(log)
    assert not bad, f"{len(bad)} buffers written out of bounds: {bad[:5]}"
    assert torch.isfinite(losses["loss"]).all()


def test_guard_detects_an_out_of_bounds_write():
    """The screen itself: a write one element past a guarded buffer is reported."""
    from mamba_clip_amd import ops
    with guarded([ops]) as log:
        t = ops.torch.empty(1000, device=DEV)
    t.as_strided((1,), (1,), t.storage_offset() + 1000).fill_(1.0)
    bad = check(log)
    assert len(bad) == 1 and not bad[0]["high_guard_ok"] and bad[0]["high_first_bad"] == 0
