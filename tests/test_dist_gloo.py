"""Multi-process (gloo, CPU) checks of the distributed ClipLoss host logic:
feature gather (one stacked all_gather), local-slice re-insertion, local_loss
label offsets and loss coefficients, gather_with_grad -- against the golden
vectors produced by the reference loss.py under gloo (tests/golden).

The HIP kernels cannot run on CPU, so here the dense op `scaled_logits_ce`
is replaced by a CPU restatement (the oracle acts as the checker).  The HIP
op itself is checked on the GPU in test_loss_gpu.py on every path this host
logic drives: square global logits, and the local_loss rectangular (b x N)
logits with row offset b*rank and no column term
(test_scaled_logits_ce_local_loss_rectangular, and per rank against these same
gloo goldens in test_local_loss_matches_reference_gloo_golden)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT, load_golden


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cpu_scaled_logits_ce(X, Y, scale, row_off=0, coef_r=1.0, col_off=0, coef_c=0.0):
    S = scale * X @ Y.T
    r = torch.arange(S.shape[0])
    loss = coef_r * (torch.logsumexp(S, 1) - S[r, r + row_off]).sum()
    if coef_c:
        c = torch.arange(S.shape[1])
        loss = loss + coef_c * (torch.logsumexp(S, 0) - S[c + col_off, c]).sum()
    return loss


def _worker(rank, world, port, q):
    try:
        _worker_body(rank, world, port, q)
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, {"error": repr(e)}))


def _worker_body(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
    import torch.distributed as dist
    import mamba_clip_amd.loss as L
    L.scaled_logits_ce = _cpu_scaled_logits_ce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = load_golden(f"clip_loss_gloo_w{world}.safetensors")
    b = g["img"].shape[0] // world
    res = {}
    for ll in (False, True):
        for gg in (False, True):
            img = g["img"][rank * b:(rank + 1) * b].clone().requires_grad_(True)
            txt = g["txt"][rank * b:(rank + 1) * b].clone().requires_grad_(True)
            scale = torch.tensor(10.0, requires_grad=True)
            crit = L.ClipLoss(local_loss=ll, gather_with_grad=gg, cache_labels=True, rank=rank, world_size=world)
            loss = crit(img, txt, scale)["contrastive_loss"]
            loss.backward()
            key = f"ll{int(ll)}_gg{int(gg)}"
            ok = (torch.allclose(loss.detach().reshape(1), g[f"r{rank}.{key}.loss"], rtol=1e-5, atol=1e-6)
                  and torch.allclose(img.grad, g[f"r{rank}.{key}.grad_img"], rtol=1e-4, atol=1e-6)
                  and torch.allclose(txt.grad, g[f"r{rank}.{key}.grad_txt"], rtol=1e-4, atol=1e-6)
                  and torch.allclose(scale.grad.reshape(1), g[f"r{rank}.{key}.grad_scale"], rtol=1e-4, atol=1e-6))
            res[key] = bool(ok)
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_clip_loss_distributed_matches_reference(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for rank, res in results.items():
        assert all(res.values()), f"rank {rank}: {res}"


# ---------------------------------------------------------------- DDP train step (train.py step semantics)
def _ddp_worker(rank, world, port, q):
    try:
        import sys
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
        from types import SimpleNamespace
        import torch.distributed as dist
        import mamba_clip_amd.loss as L
        from mamba_clip_amd.model import build_clip
        from mamba_clip_amd.train import create_optimizer, train_step, wrap_ddp
        from oracle.cpu_model import oracle_ops
        L.scaled_logits_ce = _cpu_scaled_logits_ce
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        args = SimpleNamespace(precision="fp32", lr=1e-3, wd=0.1, beta1=0.9, beta2=0.98, eps=1e-8,
                               grad_clip_norm=None, distributed=True, ddp_static_graph=False, rank=rank,
                               world_size=world)
        g = torch.Generator().manual_seed(5)
        B = 4 * world
        images = torch.randn(B, 3, 32, 32, generator=g)
        texts = torch.randint(1, 999, (B, 16), generator=g)
        texts[:, -1] = 999
        targets = torch.zeros(B, dtype=torch.long)
        sl = slice(rank * 4, (rank + 1) * 4)
        with oracle_ops():
            torch.manual_seed(0)
            model = wrap_ddp(build_clip("tiny-mamba-clip"), args, torch.device("cpu"))
            loss = L.ClipLoss(rank=rank, world_size=world)
            # gradients: DDP averages the per-rank gradients of the GLOBAL loss w.r.t. the local
            # features, so world * grad == the single-process gradient on the whole batch
            out = model(images[sl], texts[sl])
            loss(**out)["contrastive_loss"].backward()
            grads = torch.cat([p.grad.flatten() for p in model.module.parameters()]) * world
            opt = create_optimizer(model, args)
            train_step(model, images[sl], texts[sl], targets[sl], loss, opt, None, args)
            params = torch.cat([p.detach().flatten() for p in model.module.parameters()])
            res = {"params": params.numpy(), "grads": grads.numpy()}
            if rank == 0:   # single process on the whole global batch, same init
                torch.manual_seed(0)
                ref = build_clip("tiny-mamba-clip")
                ref_out = ref(images, texts)
                L.ClipLoss()(**ref_out)["contrastive_loss"].backward()
                res["ref_grads"] = torch.cat([p.grad.flatten() for p in ref.parameters()]).numpy()
        q.put((rank, res))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, {"error": repr(e) + traceback.format_exc()}))


def test_ddp_train_step_matches_single_process_gloo_w2():
    """wrap_ddp + ClipLoss(rank, world) + train_step on 2 gloo ranks == one process on the global batch."""
    import numpy as np
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
    np.testing.assert_array_equal(out[0]["params"], out[1]["params"])          # replicas stay identical
    np.testing.assert_array_equal(out[0]["grads"], out[1]["grads"])            # all-reduced gradients
    # every rank evaluates the full global loss, so the shared logit_scale (parameter 0 of ClipModel:
    # registered first) gets the FULL gradient after DDP averaging, the towers 1/world of it
    # (the reference's semantics as well)
    g, ref = out[0]["grads"], out[0]["ref_grads"]
    scale = np.abs(ref).max()
    np.testing.assert_allclose(g[1:], ref[1:], rtol=1e-4, atol=1e-6 * scale)
    np.testing.assert_allclose(g[0] / world, ref[0], rtol=1e-4)


# ---------------------------------------------------------------- stage-2 head under DDP (pipeline.py:587-636)
def _stage2_worker(rank, world, port, q):
    try:
        import sys
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
        from functools import partial
        from types import SimpleNamespace
        import torch.distributed as dist
        from mamba_clip_amd.loss import cross_entropy_loss
        from mamba_clip_amd.model import ClipClassifier, build_clip
        from mamba_clip_amd.train import create_optimizer, train_step, wrap_ddp
        from oracle.cpu_model import oracle_ops
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        args = SimpleNamespace(precision="fp32", lr=1e-3, wd=0.1, beta1=0.9, beta2=0.98, eps=1e-8,
                               grad_clip_norm=None, distributed=True, ddp_static_graph=False, rank=rank,
                               world_size=world)
        g = torch.Generator().manual_seed(9)
        B = 4 * world
        images = torch.randn(B, 3, 32, 32, generator=g)
        texts = torch.randint(1, 999, (B, 16), generator=g)
        targets = torch.randint(0, 2, (B,), generator=g)
        sl = slice(rank * 4, (rank + 1) * 4)
        loss = partial(cross_entropy_loss, weight=torch.tensor([1.0, 2.0]))
        with oracle_ops():
            torch.manual_seed(0)
            head = ClipClassifier(build_clip("tiny-mamba-clip"), num_classes=2)
            init = {k: v.clone() for k, v in head.state_dict().items()}
            model = wrap_ddp(head, args, torch.device("cpu"))
            opt = create_optimizer(model, args)
            n_train = sum(p.numel() for p in model.parameters() if p.requires_grad)
            logits = model(images[sl], texts[sl])
            loss(logits, targets[sl]).backward()
            grads = torch.cat([p.grad.flatten() for p in model.module.fc.parameters()])
            opt.zero_grad()
            train_step(model, images[sl], texts[sl], targets[sl], loss, opt, None, args)
            res = {"params": torch.cat([p.detach().flatten() for p in model.module.parameters()]).numpy(),
                   "grads": grads.numpy(), "n_train": n_train}
            if rank == 0:   # one process over the whole global batch, same init
                ref = ClipClassifier(build_clip("tiny-mamba-clip"), num_classes=2)
                ref.load_state_dict(init)
                loss(ref(images, texts), targets).backward()
                res["ref_grads"] = torch.cat([p.grad.flatten() for p in ref.fc.parameters()]).numpy()
                res["fc_numel"] = sum(p.numel() for p in ref.fc.parameters())
        q.put((rank, res))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, {"error": repr(e) + traceback.format_exc()}))


def test_stage2_head_ddp_gloo_w2():
    """Stage 2 as replicas: only the head trains, DDP all-reduces just the head's gradients
    (identical on both ranks after the all-reduce) and the replicas stay bit-identical after the step."""
    import numpy as np
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stage2_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
    np.testing.assert_array_equal(out[0]["params"], out[1]["params"])
    np.testing.assert_array_equal(out[0]["grads"], out[1]["grads"])
    assert out[0]["n_train"] == out[0]["fc_numel"]           # frozen towers: only the fc head is trained
    assert np.isfinite(out[0]["grads"]).all() and np.abs(out[0]["grads"]).max() > 0


# ---------------------------------------------------------------- DDP + two-stream towers on the GPU
def _ddp_streams_worker(rank, world, port, q):
    try:
        import sys
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
        from types import SimpleNamespace
        import torch.distributed as dist
        from mamba_clip_amd.loss import ClipLoss
        from mamba_clip_amd.model import build_clip
        from mamba_clip_amd.train import wrap_ddp
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)            # both ranks share the box's GPU (gloo moves CUDA tensors)
        args = SimpleNamespace(distributed=True, ddp_static_graph=False, ddp_bucket_mb=1)
        g = torch.Generator().manual_seed(5 + rank)
        images = torch.randn(8, 3, 32, 32, generator=g).to(dev)
        texts = torch.randint(1, 999, (8, 16), generator=g).to(dev)
        res = {}
        for conc in (True, False):
            torch.manual_seed(0)
            inner = build_clip("tiny-mamba-clip").to(dev)
            inner.concurrent_towers = conc
            model = wrap_ddp(inner, args, dev)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(images, texts)
                loss = ClipLoss(rank=rank, world_size=world)(**out)["contrastive_loss"]
            loss.backward()
            torch.cuda.synchronize()
            res[conc] = (torch.cat([p.grad.float().flatten() for p in inner.parameters()]).cpu().numpy(),
                         inner.ddp_streams_joined)
        q.put((rank, {"conc": res[True][0], "seq": res[False][0], "joined": res[True][1]}))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, {"error": repr(e) + traceback.format_exc()}))


def _ddp_streams_steps_worker(rank, world, port, q, steps=3):
    """Three optimizer steps under DDP with static_graph (bucket rebuild after the first iteration, the
    side-stream AccumulateGrad nodes reused): every step's all-reduced gradients, towers on two streams
    and on one."""
    try:
        import sys
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
        from types import SimpleNamespace
        import torch.distributed as dist
        from mamba_clip_amd.loss import ClipLoss
        from mamba_clip_amd.model import build_clip
        from mamba_clip_amd.train import wrap_ddp
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        args = SimpleNamespace(distributed=True, ddp_static_graph=True, ddp_bucket_mb=1)
        res = {}
        for conc in (True, False):
            torch.manual_seed(0)
            inner = build_clip("tiny-mamba-clip").to(dev)
            inner.concurrent_towers = conc
            model = wrap_ddp(inner, args, dev)
            opt = torch.optim.SGD(inner.parameters(), lr=0.05)
            grads, joined = [], []
            for step in range(steps):
                g = torch.Generator().manual_seed(100 * step + 5 + rank)
                images = torch.randn(8, 3, 32, 32, generator=g).to(dev)
                texts = torch.randint(1, 999, (8, 16), generator=g).to(dev)
                opt.zero_grad(set_to_none=True)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = model(images, texts)
                    loss = ClipLoss(rank=rank, world_size=world)(**out)["contrastive_loss"]
                loss.backward()
                torch.cuda.synchronize()
                grads.append(torch.cat([p.grad.float().flatten() for p in inner.parameters()]).cpu().numpy())
                joined.append(bool(inner.ddp_streams_joined))
                opt.step()
            torch.cuda.synchronize()
            res[conc] = (grads, joined)
        q.put((rank, {"conc": res[True][0], "seq": res[False][0], "joined": res[True][1]}))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, {"error": repr(e) + traceback.format_exc()}))


@pytest.mark.gpu
def test_ddp_two_stream_towers_three_steps_static_graph_gloo_gpu_w2():
    """the two-stream DDP path over 3 optimizer steps with static_graph (DDP rebuilds
    its buckets after the first iteration and reuses the side-stream AccumulateGrad nodes): every step's
    all-reduced gradients bitwise equal to the one-stream run, and equal on both ranks."""
    import numpy as np
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_streams_steps_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
        assert all(out[r]["joined"])
        assert len(out[r]["conc"]) == 3
        for step, (gc, gs) in enumerate(zip(out[r]["conc"], out[r]["seq"])):
            np.testing.assert_array_equal(gc, gs, err_msg=f"rank {r} step {step}")
    for step in range(3):
        np.testing.assert_array_equal(out[0]["conc"][step], out[1]["conc"][step])


@pytest.mark.gpu
def test_ddp_two_stream_towers_gloo_gpu_w2():
    """wrap_ddp with ClipModel's text tower on a second stream (comm hook joining the streams before
    each bucket's all-reduce; 1 MB buckets so buckets mix both towers): all-reduced gradients
    bitwise equal to the one-stream run, and equal on both ranks."""
    import numpy as np
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_streams_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
        assert out[r]["joined"]
        np.testing.assert_array_equal(out[r]["conc"], out[r]["seq"])
    np.testing.assert_array_equal(out[0]["conc"], out[1]["conc"])
