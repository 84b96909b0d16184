"""Host side of the ISIC-shaped input path (mamba_clip_amd/data.py): the rank-sharded per-epoch order
(DistributedSampler semantics, drop_last), batches equal to the dataset's own samples, the producer
thread's shutdown, and the raw-image normalisation vs the reference transform's restatement
(oracle/cpu_model.py to_tensor_normalize, data.py:102-106)."""
import threading

import torch

from mamba_clip_amd.data import HostToDeviceLoader, IsicShapedDataset, normalize_images, synthetic_batch
from oracle.cpu_model import to_tensor_normalize


def _ds(n=40):
    return IsicShapedDataset(n, image_size=16, context_length=8, vocab_size=100, positive_fraction=0.3, seed=3)


def test_dataset_shapes_and_eot():
    ds = _ds()
    img, txt, tgt = ds[5]
    assert img.shape == (16, 16, 3) and img.dtype == torch.uint8
    assert txt.shape == (8,) and int(txt[-1]) == 99 and int(txt[:-1].min()) >= 1
    assert set(ds.targets.tolist()) <= {0, 1}


def test_loader_batches_are_dataset_samples_and_ranks_disjoint():
    ds = _ds(43)
    seen = []
    for rank in range(2):
        ld = HostToDeviceLoader(ds, 4, "cpu", rank=rank, world_size=2, seed=1)
        assert len(ld) == 43 // 8
        order = ld._order()
        n = 0
        for (img, txt, tgt), idx in zip(ld, order):
            assert torch.equal(img, ds.images[idx]) and torch.equal(txt, ds.texts[idx])
            assert torch.equal(tgt, ds.targets[idx])
            n += 1
        assert n == len(ld)
        seen.append(set(order.flatten().tolist()))
    assert not (seen[0] & seen[1]) and len(seen[0]) == len(seen[1]) == 20


def test_loader_epochs_reshuffle_and_early_break_joins_thread():
    ds = _ds()
    ld = HostToDeviceLoader(ds, 4, "cpu", seed=0)
    o0 = ld._order()
    ld.set_epoch(1)
    assert not torch.equal(o0, ld._order())
    before = threading.active_count()
    it = iter(ld)
    next(it)
    it.close()
    assert threading.active_count() == before


def test_normalize_images_matches_reference_transform():
    img = synthetic_batch(3, 20, 8, 100, image_dtype=torch.uint8)[0]
    assert img.shape == (3, 20, 20, 3) and img.dtype == torch.uint8
    torch.testing.assert_close(normalize_images(img), to_tensor_normalize(img), rtol=0, atol=2e-6)
