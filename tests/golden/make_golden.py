"""Generate the committed golden fixtures from the REFERENCE itself.

Run in the build container only (needs /root/reference; the GPU box never
runs this):   PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it produces (small safetensors files next to this script):

* scan_*.safetensors -- inputs, outputs, last states and gradients of the
  reference's selective-scan semantics.  The reference repo does not vendor
  mamba_ssm; it embeds the reference semantics as text inside
  ``flops_selective_scan_ref`` (model.py:83-169).  This script reads that text
  out of /root/reference at generation time (``ast`` walk over the ``if False``
  string blocks), wraps it in a function with mamba_ssm's signature and
  EXECUTES it.  Nothing of that text is stored in this repo: only the
  resulting vectors.
* clip_loss_*.safetensors -- the reference's loss.py imported as-is: loss and
  gradients single-process and under gloo world sizes 2 and 4 for every
  (local_loss, gather_with_grad) combination.
* ss2d_*.safetensors -- the reference's SS2D / SS_Conv_SSM modules
  (model.py:297-723) imported with stub modules for the absent third-party
  packages (open_clip, timm, mamba_ssm); the scan inside is the executed
  reference text above.  State dict, input, output and input gradient.
  ss2d_c1_d128_h16w16 is C1's exact shape; vssm_tiny_d16 a reduced VSSM
  (model.py:868-995) end to end.
* train_{clip,classifier}_mixup.safetensors -- the reference's own
  pipeline.prepare_params (AdamW groups + cosine schedule, pipeline.py:205-408)
  and train_one_epoch (train.py:92-385, balanced mixup on: the only way it
  runs) for two epochs of a toy model
  (tests/toy_models.py): per-step losses and lrs, initial and final weights,
  the optimizer's group membership.
* schedulers.safetensors -- scheduler.py's three schedules, with and without
  restarts, at steps 0..39.

Select generators on the command line (scan loss ss2d c1 train); none = all.
"""
import ast
import os
import sys
import textwrap
import types

import torch
import torch.multiprocessing as mp
from safetensors.torch import save_file

REF_SRC = "/root/reference/src"
MODEL_PY = os.path.join(REF_SRC, "mamba_clip", "model.py")
HERE = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# selective scan: execute the reference's embedded text
# --------------------------------------------------------------------------
def load_reference_scan():
    tree = ast.parse(open(MODEL_PY).read())
    frags = []
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name == "flops_selective_scan_ref":
            for s in ast.walk(node):
                if (isinstance(s, ast.If) and isinstance(s.test, ast.Constant)
                        and s.test.value is False):
                    for b in s.body:
                        if (isinstance(b, ast.Expr) and isinstance(b.value, ast.Constant)
                                and isinstance(b.value.value, str)):
                            frags.append(textwrap.dedent(b.value.value))
    assert len(frags) == 4, f"expected 4 embedded fragments, found {len(frags)}"
    body = "\n".join(frags) + "\nreturn out if not return_last_state else (out, last_state)\n"
    fn_src = ("def selective_scan_reference(u, delta, A, B, C, D=None, z=None, "
              "delta_bias=None, delta_softplus=False, return_last_state=False):\n"
              + textwrap.indent(body, "    "))
    import torch.nn.functional as F
    from einops import rearrange, repeat
    ns = {"torch": torch, "F": F, "rearrange": rearrange, "repeat": repeat}
    exec(compile(fn_src, "<reference model.py:83-169>", "exec"), ns)
    return ns["selective_scan_reference"]


def make_scan_inputs(gen, batch, dim, L, N, G, itype, wtype, has_D=True, has_z=False,
                     has_bias=True, grouped4d=True):
    """Synthetic inputs following SURVEY.md 8(d): S4D-real A, softplus^-1 dt bias."""
    u = torch.randn(batch, dim, L, generator=gen).to(itype)
    delta = (0.5 * torch.randn(batch, dim, L, generator=gen)).to(itype)
    A = -torch.exp(torch.log(torch.arange(1, N + 1, dtype=torch.float32)).repeat(dim, 1)
                   + 0.1 * torch.randn(dim, N, generator=gen))
    if grouped4d:
        Bm = torch.randn(batch, G, N, L, generator=gen).to(wtype)
        Cm = torch.randn(batch, G, N, L, generator=gen).to(wtype)
    else:
        Bm = torch.randn(batch, N, L, generator=gen).to(wtype)
        Cm = torch.randn(batch, N, L, generator=gen).to(wtype)
    D = torch.ones(dim) + 0.1 * torch.randn(dim, generator=gen) if has_D else None
    z = torch.randn(batch, dim, L, generator=gen).to(itype) if has_z else None
    bias = None
    if has_bias:
        dt = torch.exp(torch.rand(dim, generator=gen) * (torch.log(torch.tensor(0.1))
                       - torch.log(torch.tensor(1e-3))) + torch.log(torch.tensor(1e-3)))
        dt = dt.clamp(min=1e-4)
        bias = dt + torch.log(-torch.expm1(-dt))
    return dict(u=u, delta=delta, A=A, B=Bm, C=Cm, D=D, z=z, delta_bias=bias)


SCAN_CASES = {
    # name: (batch, dim, L, N, G, itype, wtype, D, z, bias, softplus, grouped4d, last)
    "ss2d_f32": (2, 64, 36, 16, 4, torch.float32, torch.float32, True, False, True, True, True, False),
    "mamba_bf16_z": (2, 64, 77, 16, 1, torch.bfloat16, torch.bfloat16, True, True, True, True, True, False),
    "mamba_bf16_3d_last": (2, 64, 100, 16, 1, torch.bfloat16, torch.bfloat16, True, True, True, True, False, True),
    "plain_f32_nosp": (1, 64, 33, 8, 1, torch.float32, torch.float32, False, False, False, False, True, True),
    "f16_z_g2": (2, 64, 64, 16, 2, torch.float16, torch.float32, True, True, True, True, True, True),
    "len1_f32": (3, 64, 1, 4, 1, torch.float32, torch.float32, True, True, True, True, True, True),
    "ragged_ch_f32": (2, 96, 45, 16, 3, torch.float32, torch.bfloat16, True, True, True, True, True, True),
    # the shipped lane-pair kernels' shapes (scan_fwd_pair.hip / scan_bwd_pair.hip: 16-bit rows and
    # B / C, N = 16, L % 8 == 0, G = 1): C2's text tower (77 tokens padded to 80, 3 chunks, the last
    # half masked), a 256-position and a 1024-position sequence (the C4 regime at a small width)
    "pair_c2_l80_bf16": (2, 64, 80, 16, 1, torch.bfloat16, torch.bfloat16, True, True, True, True, True, False),
    "pair_l256_bf16": (2, 64, 256, 16, 1, torch.bfloat16, torch.bfloat16, True, True, True, True, True, True),
    "pair_l1024_bf16": (1, 32, 1024, 16, 1, torch.bfloat16, torch.bfloat16, True, True, True, True, True, True),
    "pair_l128_f16_3d": (2, 64, 128, 16, 1, torch.float16, torch.float16, True, True, True, True, False, False),
}


def gen_scan(ref_scan):
    for idx, (name, cfg) in enumerate(SCAN_CASES.items()):
        (batch, dim, L, N, G, itype, wtype, hD, hz, hb, sp, g4, last) = cfg
        gen = torch.Generator().manual_seed(1234 + idx)
        x = make_scan_inputs(gen, batch, dim, L, N, G, itype, wtype, hD, hz, hb, g4)
        res = ref_scan(**x, delta_softplus=sp, return_last_state=last)
        out, last_state = (res if last else (res, None))
        # gradients of the reference text (it computes in fp32 internally)
        leaves = {k: v.detach().float().requires_grad_(True) for k, v in x.items()
                  if v is not None}
        args = {k: leaves.get(k) for k in x}
        gout = ref_scan(**args, delta_softplus=sp)
        dout = torch.randn(gout.shape, generator=gen)
        if name.startswith("pair_"):
            # the pair-kernel cases are compared with these gradients directly: dout as the 16-bit
            # output gradient autograd hands the kernel (exactly representable in itype)
            dout = dout.to(itype).float()
        gout.backward(dout)
        tensors = {f"in.{k}": v.contiguous() for k, v in x.items() if v is not None}
        tensors["out"] = out.contiguous()
        tensors["out_f32"] = gout.detach().contiguous()
        if last_state is not None:
            tensors["last_state"] = last_state.contiguous()
        tensors["dout"] = dout
        for k, v in leaves.items():
            tensors[f"grad.{k}"] = v.grad.contiguous()
        meta = dict(softplus=str(int(sp)), last=str(int(last)), name=name,
                    source="executed reference text model.py:83-169")
        save_file(tensors, os.path.join(HERE, f"scan_{name}.safetensors"), metadata=meta)
        print("wrote scan", name, {k: tuple(v.shape) for k, v in tensors.items()})


# --------------------------------------------------------------------------
# ClipLoss: the reference's loss.py, as-is
# --------------------------------------------------------------------------
def _loss_inputs(world, b, E, seed=0):
    g = torch.Generator().manual_seed(seed)
    img = torch.nn.functional.normalize(torch.randn(world * b, E, generator=g), dim=-1)
    txt = torch.nn.functional.normalize(torch.randn(world * b, E, generator=g), dim=-1)
    return img, txt


def _loss_worker(rank, world, b, E, port, outq):
    sys.path.insert(0, REF_SRC)
    import torch.distributed as dist
    import torch.distributed.nn  # noqa: F401  reference defect A.4: loss.py never imports it
    from mamba_clip.loss import ClipLoss
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    img_all, txt_all = _loss_inputs(world, b, E)
    res = {}
    for local_loss in (False, True):
        for gwg in (False, True):
            img = img_all[rank * b:(rank + 1) * b].clone().requires_grad_(True)
            txt = txt_all[rank * b:(rank + 1) * b].clone().requires_grad_(True)
            scale = torch.tensor(10.0, requires_grad=True)
            crit = ClipLoss(local_loss=local_loss, gather_with_grad=gwg, cache_labels=True,
                            rank=rank, world_size=world)
            loss = crit(img, txt, scale)["contrastive_loss"]
            loss.backward()
            key = f"ll{int(local_loss)}_gg{int(gwg)}"
            res[f"{key}.loss"] = loss.detach().reshape(1)
            res[f"{key}.grad_img"] = img.grad.detach()
            res[f"{key}.grad_txt"] = txt.grad.detach()
            res[f"{key}.grad_scale"] = scale.grad.detach().reshape(1)
    outq.put((rank, {k: v.numpy() for k, v in res.items()}))
    dist.barrier()
    dist.destroy_process_group()


def gen_loss():
    sys.path.insert(0, REF_SRC)
    from mamba_clip.loss import ClipLoss
    # single process
    for (N, E) in ((8, 16), (64, 32)):
        img, txt = _loss_inputs(1, N, E, seed=7)
        img.requires_grad_(True)
        txt.requires_grad_(True)
        scale = torch.tensor(14.285714, requires_grad=True)
        loss = ClipLoss()(img, txt, scale)["contrastive_loss"]
        loss.backward()
        save_file({"img": img.detach(), "txt": txt.detach(), "scale": scale.detach().reshape(1),
                   "loss": loss.detach().reshape(1), "grad_img": img.grad, "grad_txt": txt.grad,
                   "grad_scale": scale.grad.reshape(1)},
                  os.path.join(HERE, f"clip_loss_single_n{N}_e{E}.safetensors"))
        print("wrote clip loss single", N, E, float(loss))
    # gloo multi-process
    ctx = mp.get_context("spawn")
    for world in (2, 4):
        b, E = 4, 16
        q = ctx.Queue()
        port = 29600 + world
        procs = [ctx.Process(target=_loss_worker, args=(r, world, b, E, port, q))
                 for r in range(world)]
        for p in procs:
            p.start()
        results = dict(q.get() for _ in range(world))
        for p in procs:
            p.join()
        img, txt = _loss_inputs(world, b, E)
        tensors = {"img": img, "txt": txt}
        for r, res in results.items():
            for k, v in res.items():
                tensors[f"r{r}.{k}"] = torch.from_numpy(v).contiguous()
        save_file(tensors, os.path.join(HERE, f"clip_loss_gloo_w{world}.safetensors"),
                  metadata={"b": str(b), "E": str(E), "scale": "10.0"})
        print("wrote clip loss gloo", world)


# --------------------------------------------------------------------------
# SS2D glue: the reference's modules with stubbed third-party imports
# --------------------------------------------------------------------------
def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__spec__ = types.SimpleNamespace(name=name, loader=None, parent=name.rpartition(".")[0],
                                       submodule_search_locations=[])
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def import_reference_model(ref_scan):
    import transformers  # noqa: F401  (import before stubbing timm)
    from einops import rearrange, repeat
    _stub("mamba_ssm")
    _stub("mamba_ssm.ops")
    _stub("mamba_ssm.ops.selective_scan_interface", rearrange=rearrange, repeat=repeat,
          selective_scan_fn=ref_scan)

    class _Dummy:  # noqa: D401
        def __init__(self, *a, **k):
            raise RuntimeError("open_clip is not available offline")
    _stub("open_clip", CustomTextCLIP=_Dummy, create_model_from_pretrained=_Dummy,
          get_tokenizer=_Dummy, trace_model=_Dummy)
    _stub("open_clip.transform", PreprocessCfg=_Dummy)
    _stub("open_clip_train")
    _stub("open_clip_train.train", unwrap_model=lambda m: getattr(m, "module", m))

    class DropPath(torch.nn.Identity):
        def __init__(self, drop_prob=0.0):
            super().__init__()
            self.drop_prob = drop_prob
    _stub("timm")
    _stub("timm.layers")
    _stub("timm.layers.drop", DropPath=DropPath)
    sys.path.insert(0, REF_SRC)
    _stub("mamba_clip.data", get_transform=lambda *a, **k: None, ComboLoader=_Dummy,
          get_combo_loader=_Dummy, get_data=_Dummy, modify_loader=_Dummy)
    import importlib
    return importlib.import_module("mamba_clip.model")


def gen_ss2d(ref_scan):
    model = import_reference_model(ref_scan)
    for name, (d_model, H, W, batch) in {"d32_h6w5": (32, 6, 5, 2), "d16_h4w4": (16, 4, 4, 3)}.items():
        torch.manual_seed(42)
        m = model.SS2D(d_model=d_model).eval()
        x = torch.randn(batch, H, W, d_model, requires_grad=True)
        y = m(x)
        gy = torch.randn_like(y)
        y.backward(gy)
        tensors = {f"sd.{k}": v.detach().contiguous() for k, v in m.state_dict().items()}
        tensors.update({"x": x.detach(), "y": y.detach(), "gy": gy, "gx": x.grad})
        save_file(tensors, os.path.join(HERE, f"ss2d_{name}.safetensors"),
                  metadata={"d_model": str(d_model)})
        print("wrote ss2d", name, tuple(y.shape))
    # one SS_Conv_SSM block (conv branch + SS2D branch + channel shuffle + residual)
    torch.manual_seed(43)
    blk = model.SS_Conv_SSM(hidden_dim=32).eval()
    x = torch.randn(2, 4, 4, 32)
    y = blk(x)
    tensors = {f"sd.{k}": v.detach().contiguous() for k, v in blk.state_dict().items()}
    tensors.update({"x": x, "y": y.detach()})
    save_file(tensors, os.path.join(HERE, "ss_conv_ssm_h32.safetensors"))
    print("wrote ss_conv_ssm")


def gen_c1(ref_scan):
    """C1's exact SS2D shape (d_model=128 on 16x16, batch 8; BASELINE configs[0]) and a
    reduced VSSM (every stage, PatchEmbed2D / PatchMerging2D / SS_Conv_SSM, a 1x1 last
    stage) -- forward, input gradient and (SS2D) every parameter gradient.

    The large inputs are NOT stored: they are regenerated from the seed by the test
    (torch's CPU generator is deterministic for this torch version); a checksum of
    them is stored so a mismatch fails loudly instead of silently comparing garbage."""
    model = import_reference_model(ref_scan)
    torch.manual_seed(2024)
    m = model.SS2D(d_model=128).eval()
    g = torch.Generator().manual_seed(2025)
    x = torch.randn(8, 16, 16, 128, generator=g)
    gy = torch.randn(8, 16, 16, 128, generator=g)
    xg = x.clone().requires_grad_(True)
    y = m(xg)
    y.backward(gy)
    tensors = {f"sd.{k}": v.detach().contiguous() for k, v in m.state_dict().items()}
    tensors.update({f"grad.{k}": p.grad.detach().contiguous() for k, p in m.named_parameters()})
    tensors.update({"y": y.detach(), "gx": xg.grad,
                    "x_checksum": torch.stack([x.double().sum(), x.double().abs().sum(), gy.double().sum()])})
    save_file(tensors, os.path.join(HERE, "ss2d_c1_d128_h16w16.safetensors"),
              metadata={"d_model": "128", "x": "randn(8,16,16,128) then gy, Generator seed 2025"})
    print("wrote ss2d c1", tuple(y.shape))

    torch.manual_seed(45)
    v = model.VSSM(patch_size=4, in_chans=3, num_classes=2, depths=[1, 1, 2, 1], dims=[16, 32, 64, 128],
                   d_state=16).eval()
    g = torch.Generator().manual_seed(46)
    x = torch.randn(2, 3, 32, 32, generator=g).requires_grad_(True)
    y = v(x)
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy)
    tensors = {f"sd.{k}": t.detach().contiguous() for k, t in v.state_dict().items()}
    tensors.update({"x": x.detach(), "y": y.detach(), "gy": gy, "gx": x.grad,
                    "grad.head.weight": v.head.weight.grad})
    save_file(tensors, os.path.join(HERE, "vssm_tiny_d16.safetensors"),
              metadata={"depths": "1,1,2,1", "dims": "16,32,64,128", "img": "32"})
    print("wrote vssm tiny", tuple(y.shape))


# --------------------------------------------------------------------------
# train step / optimizer groups / schedulers: the reference's train.py,
# pipeline.prepare_params and scheduler.py, as-is, on toy models
# --------------------------------------------------------------------------
TRAIN_ARGS = dict(force_image_size=None, seed=0, rank=0, local_rank=0, siglip=False, use_bnb_linear=None,
                  trace=False, lock_image=False, lock_text=False, grad_checkpointing=False, name="toy",
                  distributed=False, wd=0.1, lr=1e-2, beta1=0.9, beta2=0.98, eps=1e-6, precision="fp32",
                  resume=None, accum_freq=1, epochs=2, lr_restart_interval=None, warmup=1,
                  lr_scheduler="cosine", tensorboard=False, hyperparameter_tuning=False, wandb=False,
                  torchcompile=False, ddp_static_graph=False, use_bn_sync=False, device="cpu",
                  skip_scheduler=False, balanced_mixup=0.5, num_classes=2, grad_clip_norm=1.0,
                  log_every_n_steps=1, world_size=1, batch_size=4)
TRAIN_BATCHES, TRAIN_B, MIX_SEED = 3, 4, 321


def gen_train(ref_scan):
    import json
    import tempfile
    from functools import partial
    from types import SimpleNamespace
    import numpy as np
    sys.path.insert(0, os.path.dirname(HERE))
    import toy_models as T
    import_reference_model(ref_scan)           # stubs for open_clip & co, then pipeline imports
    import importlib
    pipeline = importlib.import_module("mamba_clip.pipeline")
    ref_train = importlib.import_module("mamba_clip.train")
    ref_loss = importlib.import_module("mamba_clip.loss")
    for kind in ("clip", "classifier"):
        torch.manual_seed(7)
        model = T.ToyClip() if kind == "clip" else T.ToyClassifier()
        init_sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
        data = {"train": T.ToyData(T.toy_batches(TRAIN_BATCHES, TRAIN_B, seed=11), TRAIN_B)}
        with tempfile.TemporaryDirectory() as logs:
            os.makedirs(os.path.join(logs, "toy"))
            args = SimpleNamespace(**TRAIN_ARGS, logs=logs)
            params, args = pipeline.prepare_params(model, data, torch.device("cpu"), args)
        opt, sched = params["optimizer"], params["scheduler"]
        ids = {id(p): n for n, p in model.named_parameters()}
        groups = [[ids[id(p)] for p in g["params"]] for g in opt.param_groups]
        lrs, losses = [], []

        def rec_sched(step, _s=sched):
            lrs.append(float(_s(step)))

        inner = (ref_loss.ClipLoss() if kind == "clip"
                 else partial(ref_loss.cross_entropy_loss, weight=torch.tensor([1.0, 3.0])))

        def rec_loss(**kw):
            out = inner(**kw)
            losses.append(float((out["contrastive_loss"] if isinstance(out, dict) else out).detach()))
            return out

        np.random.seed(MIX_SEED)
        for epoch in range(args.epochs):
            ref_train.train_one_epoch(model, data, rec_loss, epoch, opt, params["scaler"], rec_sched, args)
        tensors = {f"init.{k}": v.contiguous() for k, v in init_sd.items()}
        tensors.update({f"final.{k}": v.detach().contiguous() for k, v in model.state_dict().items()})
        tensors["losses"] = torch.tensor(losses, dtype=torch.float64)
        tensors["lrs"] = torch.tensor(lrs, dtype=torch.float64)
        meta = {"groups": json.dumps(groups), "kind": kind, "mix_seed": str(MIX_SEED),
                "args": json.dumps({k: v for k, v in TRAIN_ARGS.items() if k != "logs"})}
        save_file(tensors, os.path.join(HERE, f"train_{kind}_mixup.safetensors"), metadata=meta)
        print("wrote train", kind, losses)

    # schedulers: (factory, positional args after the optimizer) -> lr at steps 0..39
    sched_mod = importlib.import_module("mamba_clip.scheduler")

    class _Opt:
        def __init__(self):
            self.param_groups = [{"lr": 0.0}]
    cases = {
        "cosine": ("cosine_lr", (1e-3, 5, 40), {}),
        "cosine_restart": ("cosine_lr", (1e-3, 3, 40), {"restart_interval": 13}),
        "const": ("const_lr", (2e-3, 7, 40), {}),
        "const_restart": ("const_lr", (2e-3, 4, 40), {"restart_interval": 9}),
        "cooldown": ("const_lr_cooldown", (1e-3, 5, 40, 10), {"cooldown_power": 2.0, "cooldown_end_lr": 1e-5}),
        "cooldown_restart": ("const_lr_cooldown", (1e-3, 2, 40, 4), {"restart_interval": 10}),
    }
    tensors = {}
    for name, (fn, pos, kw) in cases.items():
        o = _Opt()
        f = getattr(sched_mod, fn)(o, *pos, **kw)
        vals = []
        for s in range(40):
            r = f(s)
            assert r == o.param_groups[0]["lr"]
            vals.append(float(r))
        tensors[name] = torch.tensor(vals, dtype=torch.float64)
    import json as _j
    save_file(tensors, os.path.join(HERE, "schedulers.safetensors"),
              metadata={"cases": _j.dumps({k: [v[0], list(v[1]), v[2]] for k, v in cases.items()})})
    print("wrote schedulers")


GENERATORS = {"scan": lambda r: gen_scan(r), "loss": lambda r: gen_loss(), "ss2d": gen_ss2d, "c1": gen_c1,
              "train": gen_train}

if __name__ == "__main__":
    ref_scan = load_reference_scan()
    for name in (sys.argv[1:] or list(GENERATORS)):
        GENERATORS[name](ref_scan)
