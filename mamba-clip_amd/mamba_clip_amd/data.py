"""Synthetic batches shaped like the reference's dataset output, and the ISIC-shaped host input path.

Decoding (JPEG / HDF5 bytes -> PIL) and the CSV metadata are out of the hot path;
training and the bench consume (images, texts, targets) of the right shapes and dtypes:
  - synthetic_batch: generated once on the device (inputs resident in HBM); images either the
    reference's transformed float NCHW batch or raw decoded uint8 NHWC crops;
  - IsicShapedDataset + HostToDeviceLoader: an ISIC-2024-shaped dataset of
    decoded 224x224 uint8 crops in host memory (what IsicChallengeDataset.__getitem__ yields before
    ToTensor / Normalize, data.py:297-383) streamed to the GPU as raw bytes through pinned staging
    buffers on a copy stream; ToTensor + Normalize run on the device, fused into the towers' patch
    embedding (ops.patch_im2col -> mc_patch_embed_input), so the PCIe copy is 4x smaller than the
    reference's normalised fp32 batch.
Text rows end with the end-of-text token at the last position (pooling index).
"""
import queue
import threading
from dataclasses import dataclass

import torch


def synthetic_batch(batch, image_size, context_length, vocab_size, num_classes=2, device="cpu", seed=0,
                    image_dtype=torch.float32):
    """image_dtype float: (B, 3, S, S) N(0, 1) (a normalised batch); torch.uint8: (B, S, S, 3) raw bytes."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    if image_dtype == torch.uint8:
        images = torch.randint(0, 256, (batch, image_size, image_size, 3), dtype=torch.uint8, generator=g).to(device)
    else:
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
        for obj in (self.sampler, self.dataloader):
            if obj is not None and hasattr(obj, "set_epoch"):
                obj.set_epoch(epoch)


def get_synthetic_data(batch, num_batches, image_size, context_length, vocab_size, device, seed=0,
                       image_dtype=torch.float32, balanced=False, num_classes=2):
    loader = _SyntheticLoader(batch, num_batches, balanced=balanced, image_size=image_size,
                              context_length=context_length, vocab_size=vocab_size, num_classes=num_classes,
                              device=device, seed=seed, image_dtype=image_dtype)
    return {"train": DataInfo(loader)}


def normalize_images(img_u8, mean=None, std=None):
    """(B, H, W, C) uint8 -> (B, C, H, W) fp32: ToTensor + Normalize (data.py:102-106), for the paths that
    need a float image before the towers (balanced mixup); the towers take raw bytes directly."""
    from .ops import IMAGE_MEAN, IMAGE_STD
    C = img_u8.shape[-1]
    m = torch.tensor((mean or IMAGE_MEAN)[:C], device=img_u8.device).view(1, C, 1, 1)
    s = torch.tensor((std or IMAGE_STD)[:C], device=img_u8.device).view(1, C, 1, 1)
    return (img_u8.permute(0, 3, 1, 2).float() / 255.0 - m) / s


class IsicShapedDataset:
    """ISIC-2024-shaped samples: decoded RGB crops (H, W, 3) uint8 as IsicChallengeDataset yields them after
    ResizeKeepRatio + CenterCropOrPad (data.py:101-104, 297-314), a tokenised report of the sample's
    metadata (data.py:316-328; synthetic ids here, EOT last) and the malignancy target (heavily
    imbalanced: `positive_fraction`, ISIC 2024 is ~0.1 % positive).  Held in host memory as three
    contiguous tensors, indexable per sample like a torch Dataset."""

    def __init__(self, num_samples, image_size=224, context_length=77, vocab_size=50000, positive_fraction=0.01,
                 seed=0):
        g = torch.Generator().manual_seed(seed)
        self.images = torch.randint(0, 256, (num_samples, image_size, image_size, 3), dtype=torch.uint8, generator=g)
        self.texts = torch.randint(1, vocab_size - 1, (num_samples, context_length), generator=g)
        self.texts[:, -1] = vocab_size - 1
        self.targets = (torch.rand(num_samples, generator=g) < positive_fraction).long()

    def __len__(self):
        return self.images.shape[0]

    def __getitem__(self, idx):
        return self.images[idx], self.texts[idx], self.targets[idx]


class HostToDeviceLoader:
    """Batches of an IsicShapedDataset on `device`: a shuffled, rank-sharded order per epoch
    (DistributedSampler semantics, drop_last: every rank gets len(dataset) // (world * batch) batches),
    a host thread gathering each batch into one of `slots` pinned staging buffers, and the H2D copy
    issued on a dedicated copy stream one batch ahead of the consumer, so the copy of batch i + 1
    overlaps the step on batch i.  Yielded tensors are safe on the consumer's current stream
    (it waits on the copy; record_stream keeps the allocator from reusing them early)."""

    def __init__(self, dataset, batch, device, rank=0, world_size=1, seed=0, slots=3):
        self.ds, self.batch, self.device = dataset, batch, torch.device(device)
        self.rank, self.world, self.seed, self.epoch, self.slots = rank, world_size, seed, 0, slots
        self.num_batches = len(dataset) // (world_size * batch)
        self.num_samples = self.num_batches * batch
        self._stream = None
        self._pinned = None

    def set_epoch(self, epoch):
        self.epoch = epoch

    def __len__(self):
        return self.num_batches

    def _order(self):
        g = torch.Generator().manual_seed(self.seed + self.epoch)
        perm = torch.randperm(len(self.ds), generator=g)[: self.num_batches * self.batch * self.world]
        return perm[self.rank::self.world].reshape(self.num_batches, self.batch)

    def _alloc(self):
        if self._pinned is None:
            ds, b, cuda = self.ds, self.batch, self.device.type == "cuda"

            def buf(shape, dt):
                t = torch.empty(shape, dtype=dt)
                return t.pin_memory() if cuda else t
            self._pinned = [(buf((b,) + tuple(ds.images.shape[1:]), torch.uint8),
                             buf((b,) + tuple(ds.texts.shape[1:]), ds.texts.dtype),
                             buf((b,), ds.targets.dtype)) for _ in range(self.slots)]
            self._stream = torch.cuda.Stream(self.device) if cuda else None

    def __iter__(self):
        self._alloc()
        order = self._order()
        free, ready = queue.Queue(), queue.Queue(maxsize=self.slots)
        for k in range(self.slots):
            free.put((k, None))
        stop = threading.Event()

        def produce():
            for idx in order:
                k, ev = free.get()
                if stop.is_set():
                    return
                if ev is not None:
                    ev.synchronize()          # the slot's previous H2D copy has finished reading it
                img, txt, tgt = self._pinned[k]
                torch.index_select(self.ds.images, 0, idx, out=img)
                torch.index_select(self.ds.texts, 0, idx, out=txt)
                torch.index_select(self.ds.targets, 0, idx, out=tgt)
                ready.put(k)

        th = threading.Thread(target=produce, daemon=True)
        th.start()

        def issue():
            k = ready.get()
            if self._stream is None:       # CPU device (host-side tests): plain copies
                dev = tuple(t.clone() for t in self._pinned[k])
                free.put((k, None))
                return dev
            with torch.cuda.stream(self._stream):
                dev = tuple(t.to(self.device, non_blocking=True) for t in self._pinned[k])
                ev = torch.cuda.Event()
                ev.record(self._stream)
            free.put((k, ev))
            return dev

        try:
            nxt = issue() if self.num_batches else None
            for i in range(self.num_batches):
                cur = nxt
                if self._stream is not None:
                    main = torch.cuda.current_stream(self.device)
                    main.wait_stream(self._stream)
                    for t in cur:
                        t.record_stream(main)
                nxt = issue() if i + 1 < self.num_batches else None
                yield cur
        finally:
            stop.set()
            for _ in range(self.slots):
                free.put((0, None))
            th.join()


def get_isic_shaped_data(batch, num_samples, image_size, context_length, vocab_size, device, rank=0, world_size=1,
                         seed=0, positive_fraction=0.01):
    ds = IsicShapedDataset(num_samples, image_size, context_length, vocab_size, positive_fraction, seed)
    return {"train": DataInfo(HostToDeviceLoader(ds, batch, device, rank, world_size, seed))}
