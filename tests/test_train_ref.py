"""The training step's host logic against the REFERENCE's own outputs (CPU, no HIP).

Fixtures (tests/golden/make_golden.py `gen_train`) come from running the
reference's pipeline.prepare_params and train_one_epoch (pipeline.py:205-408,
train.py:92-385; balanced mixup on, train.py:131-151) on the toy models of
tests/toy_models.py, and its scheduler.py at steps 0..39.  Here the same toy
weights go through OUR create_optimizer / scheduler / train_one_epoch with the
loss computed by the CPU oracle restatement of loss.py (oracle/cpu_model) --
the HIP loss is checked separately on the GPU (tests/test_loss_gpu.py).
"""
import json
import math
import os
import socket
from functools import partial
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT, golden_meta, load_golden
import toy_models as T


def _args(meta_args, **kw):
    a = dict(json.loads(meta_args))
    a.update(kw)
    return SimpleNamespace(**a)


def _sched(name, opt, args, n_batches):
    from mamba_clip_amd.scheduler import cosine_lr
    assert name == "cosine"
    # pipeline.py:326-348: warmup / total in optimizer steps
    per_epoch = n_batches // args.accum_freq
    return cosine_lr(opt, args.lr, per_epoch * args.warmup, per_epoch * args.epochs)


@pytest.mark.parametrize("kind", ["clip", "classifier"])
def test_train_one_epoch_matches_reference(kind):
    from mamba_clip_amd.loss import cross_entropy_loss
    from mamba_clip_amd.train import create_optimizer, train_one_epoch
    from oracle.cpu_model import oracle_clip_loss
    name = f"train_{kind}_mixup.safetensors"
    g, meta = load_golden(name), golden_meta(name)
    args = _args(meta["args"])
    model = T.ToyClip() if kind == "clip" else T.ToyClassifier()
    model.load_state_dict({k[5:]: v for k, v in g.items() if k.startswith("init.")})
    opt = create_optimizer(model, args)
    # AdamW groups: same membership and order as pipeline.py:280-308
    ids = {id(p): n for n, p in model.named_parameters()}
    assert [[ids[id(p)] for p in grp["params"]] for grp in opt.param_groups] == json.loads(meta["groups"])
    assert [grp["weight_decay"] for grp in opt.param_groups] == [0.0, args.wd]
    data = {"train": T.ToyData(T.toy_batches(3, args.batch_size, seed=11), args.batch_size)}
    sched = _sched(args.lr_scheduler, opt, args, 3)
    lrs, losses = [], []

    def rec_sched(step):
        lrs.append(sched(step))

    inner = oracle_clip_loss if kind == "clip" else partial(cross_entropy_loss, weight=torch.tensor([1.0, 3.0]))

    def rec_loss(**kw):
        out = inner(**kw)
        losses.append(float((out["contrastive_loss"] if isinstance(out, dict) else out).detach()))
        return out

    np.random.seed(int(meta["mix_seed"]))
    for epoch in range(args.epochs):
        train_one_epoch(model, data, rec_loss, epoch, opt, None, rec_sched, args)
    assert data["train"].epochs == list(range(args.epochs))
    np.testing.assert_allclose(lrs, g["lrs"].numpy(), rtol=1e-12, atol=0)
    np.testing.assert_allclose(losses, g["losses"].numpy(), rtol=2e-5, atol=1e-6)
    final = {k[6:]: v for k, v in g.items() if k.startswith("final.")}
    for k, v in model.state_dict().items():
        torch.testing.assert_close(v, final[k], rtol=1e-4, atol=2e-6, msg=lambda m: f"{k}: {m}")
    if kind == "clip":
        assert 0.0 <= float(model.logit_scale.detach()) <= math.log(100)


def test_schedulers_match_reference():
    from mamba_clip_amd import scheduler as S
    g, meta = load_golden("schedulers.safetensors"), golden_meta("schedulers.safetensors")

    class Opt:
        def __init__(self):
            self.param_groups = [{"lr": 0.0}, {"lr": 0.0}]

    for name, (fn, pos, kw) in json.loads(meta["cases"]).items():
        o = Opt()
        f = getattr(S, fn)(o, *pos, **kw)
        got = []
        for s in range(40):
            got.append(f(s))
            assert all(grp["lr"] == got[-1] for grp in o.param_groups)
        np.testing.assert_allclose(got, g[name].numpy(), rtol=1e-12, atol=1e-18, err_msg=name)


def test_get_model_inputs_mixup_semantics():
    """train.py:66-89: lam ~ Beta(m, 1) from np.random; images mixed; texts swapped when lam > 0.5;
    only the model inputs are returned (the mixed one-hot targets are computed and dropped)."""
    from mamba_clip_amd.train import get_model_inputs
    args = SimpleNamespace(balanced_mixup=0.7, num_classes=3)
    g = torch.Generator().manual_seed(0)
    img, bimg = torch.randn(4, 3, 8, 8, generator=g), torch.randn(4, 3, 8, 8, generator=g)
    txt, btxt = torch.randint(0, 9, (4, 5), generator=g), torch.randint(0, 9, (4, 5), generator=g)
    tgt, btgt = torch.tensor([0, 1, 2, 0]), torch.tensor([2, 2, 1, 0])
    for seed in range(6):
        np.random.seed(seed)
        lam = np.random.beta(a=0.7, b=1)
        np.random.seed(seed)
        out = get_model_inputs(args, img, txt, tgt, bimg, btxt, btgt)
        assert len(out) == 2
        torch.testing.assert_close(out[0], (1 - lam) * img + lam * bimg)
        assert torch.equal(out[1], btxt if lam > 0.5 else txt)
    off = SimpleNamespace(balanced_mixup=None)
    assert get_model_inputs(off, img, None, tgt)[0] is img and len(get_model_inputs(off, img, None, tgt)) == 1


def test_train_step_rejects_mixup_without_balanced_batch():
    from mamba_clip_amd.train import create_optimizer, train_step
    args = SimpleNamespace(balanced_mixup=0.5, num_classes=2, precision="fp32", lr=1e-3, wd=0.1, beta1=0.9,
                           beta2=0.98, eps=1e-6)
    m = T.ToyClassifier()
    with pytest.raises(ValueError, match="balanced"):
        train_step(m, torch.zeros(2, *T.IMG), torch.ones(2, T.CTX, dtype=torch.long), torch.zeros(2, dtype=torch.long),
                   None, create_optimizer(m, args), None, args)


def test_cli_balanced_mixup_synthetic_batches():
    """--balanced-mixup makes the synthetic loader yield ComboLoader pairs that split_batch unpacks."""
    from mamba_clip_amd.data import get_synthetic_data
    from mamba_clip_amd.train import split_batch
    d = get_synthetic_data(4, 2, 16, 6, 50, "cpu", balanced=True)
    batch = next(iter(d["train"].dataloader))
    images, texts, targets, bal = split_batch(batch, 0.5)
    assert images.shape == (4, 3, 16, 16) and texts.shape == (4, 6) and bal[0].shape == images.shape
    assert not torch.equal(images, bal[0])
    plain = next(iter(get_synthetic_data(4, 2, 16, 6, 50, "cpu")["train"].dataloader))
    assert split_batch(plain, None)[3] is None


# ---------------------------------------------------------------- init_device under gloo (utils/dist_utils.py:34-88)
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init_device_worker(rank, world, port, q):
    try:
        import sys
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
        import torch.distributed as dist
        from mamba_clip_amd.utils import dist_utils as U
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                          LOCAL_RANK=str(rank))
        args = SimpleNamespace(dist_backend="gloo", dist_url="env://", device="cuda")
        dev = U.init_device(args)
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t)
        name = U.broadcast_object(args, f"run-from-{args.rank}")
        q.put((rank, {"rank": args.rank, "world": args.world_size, "local": args.local_rank,
                      "distributed": args.distributed, "device": str(dev), "sum": float(t), "name": name,
                      "master": U.is_master(args), "backend": dist.get_backend()}))
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((rank, {"error": repr(e) + traceback.format_exc()}))


def test_init_device_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_init_device_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
        o = out[r]
        assert (o["rank"], o["world"], o["local"], o["distributed"]) == (r, world, r, True)
        assert o["device"] == "cpu" and o["backend"] == "gloo" and o["sum"] == 3.0
        assert o["name"] == "run-from-0" and o["master"] == (r == 0)


def test_init_device_single_process(monkeypatch):
    from mamba_clip_amd.utils.dist_utils import init_device
    for v in ("WORLD_SIZE", "SLURM_NTASKS"):
        monkeypatch.delenv(v, raising=False)
    args = SimpleNamespace(device="cuda")
    assert init_device(args).type == "cpu" and args.world_size == 1 and not args.distributed and args.rank == 0
