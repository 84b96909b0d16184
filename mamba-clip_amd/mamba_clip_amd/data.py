"""Synthetic batches shaped like the reference's CsvDataset output (data.py:37-178).

Dataset/CSV/image decoding is out of the hot path (out of scope);
training and the bench consume (images, texts, targets) of the right shapes
and dtypes, generated once on the device (inputs resident in HBM).
Text rows end with the end-of-text token at the last position (pooling index).
"""
from dataclasses import dataclass

import torch


def synthetic_batch(batch, image_size, context_length, vocab_size, num_classes=2, device="cpu", seed=0,
                    image_dtype=torch.float32):
    g = torch.Generator(device="cpu").manual_seed(seed)
    images = torch.randn(batch, 3, image_size, image_size, generator=g).to(device=device, dtype=image_dtype)
    texts = torch.randint(1, vocab_size - 1, (batch, context_length), generator=g)
    texts[:, -1] = vocab_size - 1                               # end-of-text id at the pooled position
    targets = torch.randint(0, num_classes, (batch,), generator=g)
    return images, texts.to(device), targets.to(device)


class _SyntheticLoader:
    """Yields the same device-resident batch num_batches times; with balanced=True
    the ComboLoader pair (batch, balanced batch) that --balanced-mixup consumes
    (reference data.py:218-239, train.py:131-151)."""

    def __init__(self, batch, num_batches, balanced=False, **kw):
        self.batch, self.num_batches, self.kw, self.balanced = batch, num_batches, kw, balanced
        self.num_samples = batch * num_batches
        self._cached = None

    def __len__(self):
        return self.num_batches

    def __iter__(self):
        if self._cached is None:
            b = synthetic_batch(self.batch, **self.kw)
            if self.balanced:
                b = (b, synthetic_batch(self.batch, **dict(self.kw, seed=self.kw.get("seed", 0) + 7919)))
            self._cached = b
        for _ in range(self.num_batches):
            yield self._cached


@dataclass
class DataInfo:
    """dataloader + sampler pair (reference data.py DataInfo); set_epoch is a no-op for resident data."""
    dataloader: object
    sampler: object = None

    def set_epoch(self, epoch):
        if self.sampler is not None and hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)


def get_synthetic_data(batch, num_batches, image_size, context_length, vocab_size, device, seed=0,
                       image_dtype=torch.float32, balanced=False, num_classes=2):
    loader = _SyntheticLoader(batch, num_batches, balanced=balanced, image_size=image_size,
                              context_length=context_length, vocab_size=vocab_size, num_classes=num_classes,
                              device=device, seed=seed, image_dtype=image_dtype)
    return {"train": DataInfo(loader)}
