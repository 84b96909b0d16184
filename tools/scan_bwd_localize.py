#!/usr/bin/env python3
"""Localise the two-stream C2 step's run-to-run divergence.

Runs the C2 forward + ClipLoss + backward (towers on two streams, default hardware queues) --runs times
from the same parameters.  The first scan backward of the step (text layer 23) is wrapped: right AFTER
the real call (so the kernel itself runs in the step's normal concurrency) every input and output is
cloned on the same stream.  After the step the device is synchronised and the same backward is re-run
twice on the cloned inputs on a quiet device ("solo").  Per run it reports, bitwise:
  - which outputs differ between the in-step call and the solo re-run (inputs identical by construction),
  - which inputs / outputs differ from run 0,
  - for ddelta elements that differ in-step vs solo: where they sit in the pair kernel's decomposition
    (workgroup block of 128 channels, wave, chunk of 32 positions, 8-position sub-tile, lane half) and
    the batch index,
  - the layer-23 dt_proj / D / A_log gradients vs run 0.
  python3 tools/scan_bwd_localize.py --batch 32 --runs 6
"""
import argparse
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mamba-clip_amd"))
import torch  # noqa: E402

OUT_NAMES = ("du", "ddelta", "dA", "dB", "dC", "dD", "dz", "dbias")
IN_NAMES = ("u", "delta", "A", "B", "C", "D", "z", "delta_bias", "softplus", "dout", "states")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--call", type=int, default=0, help="which scan backward of the step to wrap (0 = layer 23)")
    ap.add_argument("--concurrent", type=int, default=1)
    ap.add_argument("--pre-clone", action="store_true", help="also clone the inputs right BEFORE the call")
    ap.add_argument("--debug", action="store_true",
                    help="diagnostic library (-DMC_BWD_DEBUG): compare the pair kernel's per-sub-tile carry snapshots")
    ap.add_argument("--generic", action="store_true",
                    help="every scan backward of the step on the generic kernel (B / C passed as fp32)")
    args = ap.parse_args()

    from mamba_clip_amd import selective_scan_interface as ssi
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.loss import ClipLoss
    from mamba_clip_amd.model import build_clip
    from mamba_clip_amd.tuning import load_gemm_tuning

    dev = torch.device("cuda", 0)
    load_gemm_tuning(model="vit_b16-mamba130m")
    torch.manual_seed(0)
    model = build_clip("vit_b16-mamba130m").to(dev)
    model.concurrent_towers = bool(args.concurrent)
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    images, texts, _ = synthetic_batch(args.batch, 224, model.text.context_length, model.text.vocab_size,
                                       device=dev, seed=1000)
    loss_fn = ClipLoss()
    real_bwd = ssi.scan_bwd
    state = {"n": 0, "rec": None}

    def cl(x):
        return x.detach().clone() if isinstance(x, torch.Tensor) else x

    def generic_bwd(*a, **k):
        a = list(a)
        dt = a[3].dtype
        a[3], a[4] = a[3].float(), a[4].float()
        dbc = k.pop("dbc_out", None)
        du, dd, dA, dB, dC, dD, dz, db = real_bwd(*a, **k)
        dB, dC = dB.to(dt), dC.to(dt)
        if dbc is not None:
            dbc[0].copy_(dB)
            dbc[1].copy_(dC)
            dB, dC = dbc
        return du, dd, dA, dB, dC, dD, dz, db

    call_bwd = generic_bwd if args.generic else real_bwd
    dbg = {}
    if args.debug:
        import ctypes
        from mamba_clip_amd import _lib
        lib = _lib.load()
        lib.mc_debug_alloc.argtypes = [ctypes.c_size_t]
        lib.mc_debug_copy.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        D_, L_ = 1536, 80
        nblk, nch = (D_ + 127) // 128, (L_ + 31) // 32
        dbg["shape"] = (args.batch * nblk, 4, nch, 4, 64, 32)
        dbg["bytes"] = 4 * args.batch * nblk * 4 * nch * 4 * 64 * 32
        assert lib.mc_debug_alloc(dbg["bytes"]) == 0
        torch.cuda.synchronize()

        def snap_dbg():
            t = torch.empty(dbg["shape"], device=dev, dtype=torch.float32)
            assert lib.mc_debug_copy(t.data_ptr(), dbg["bytes"], torch.cuda.current_stream().cuda_stream) == 0
            return t
        dbg["snap"] = snap_dbg

    def wrapped(*a, **k):
        i = state["n"]
        state["n"] += 1
        if i != args.call:
            return call_bwd(*a, **k)
        pre = tuple(cl(x) for x in a) if args.pre_clone else None
        out = call_bwd(*a, **k)
        state["rec"] = {"ins": tuple(cl(x) for x in a), "outs": tuple(cl(x) for x in out), "pre": pre,
                        "stream": torch.cuda.current_stream().cuda_stream,
                        "dbg": dbg["snap"]() if args.debug else None}
        return out

    ssi.scan_bwd = wrapped
    L23 = model.text.layers[-1].mixer
    runs = []
    for r in range(args.runs):
        model.load_state_dict(init)
        model.zero_grad(set_to_none=True)
        state["n"], state["rec"] = 0, None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(images, texts)
            loss = loss_fn(**out)["contrastive_loss"]
        loss.backward()
        torch.cuda.synchronize()
        rec = state["rec"]
        ins = rec["ins"]
        solo = [call_bwd(*ins) for _ in range(2)]
        torch.cuda.synchronize()
        if args.debug:
            sd = dbg["snap"]()
            torch.cuda.synchronize()
            x = rec["dbg"]
            bad = (x != sd)                                   # (blk, wave, c, s, lane, val)
            if bool(bad.any()):
                nb, nw, nc, ns = bad.shape[:4]
                # processing order: chunks and sub-tiles descending
                order = [(c, s_) for c in range(nc - 1, -1, -1) for s_ in range(ns - 1, -1, -1)]
                firsts, lanes_first, vals_first = collections.Counter(), collections.Counter(), collections.Counter()
                per_wave = bad.any(dim=5).any(dim=4)            # (blk, wave, c, s)
                idx = per_wave.nonzero().tolist()
                seen = {}
                rank = {cs: i for i, cs in enumerate(order)}
                for blk, w, c, s_ in idx:
                    key = (blk, w)
                    if key not in seen or rank[(c, s_)] < rank[seen[key]]:
                        seen[key] = (c, s_)
                for (blk, w), (c, s_) in seen.items():
                    firsts[(c, s_)] += 1
                    lb = bad[blk, w, c, s_]                     # (lane, val)
                    for ln in lb.any(dim=1).nonzero().flatten().tolist():
                        lanes_first[ln] += 1
                    for v in lb.any(dim=0).nonzero().flatten().tolist():
                        vals_first[v] += 1
                waves_idx = collections.Counter(w for (blk, w) in seen)
                blocks = sorted({blk for (blk, w) in seen})
                # which quantities differ anywhere (not only at the first sub-tile): hcar 0-7, dA 8-15, A2 16-23, entry 24-31
                anyv = bad.reshape(-1, 32).any(dim=0).nonzero().flatten().tolist()
                line_dbg_extra = {"wave_index": dict(sorted(waves_idx.items())), "n_blocks": len(blocks),
                                  "blocks_head": blocks[:24], "vals_anywhere": anyv}
                line_dbg = {"waves_affected": len(seen), "first_cs": {f"{c},{s_}": n for (c, s_), n in sorted(firsts.items())},
                            "first_lanes": dict(sorted(lanes_first.items())), "first_vals": dict(sorted(vals_first.items()))}
                ex = next(iter(seen.items()))
                (blk, w), (c, s_) = ex
                ln = bad[blk, w, c, s_].any(dim=1).nonzero().flatten()[0].item()
                line_dbg.update(line_dbg_extra)
                line_dbg["example"] = {"blk": blk, "wave": w, "c": c, "s": s_, "lane": ln,
                                       "instep": x[blk, w, c, s_, ln].tolist(), "solo": sd[blk, w, c, s_, ln].tolist()}
            else:
                line_dbg = {"waves_affected": 0}
            rec["dbg_line"] = line_dbg
        rec["solo"] = [tuple(cl(x) for x in s) for s in solo]
        rec["grads"] = {"dt_proj.bias": L23.dt_proj.bias.grad.clone(), "dt_proj.weight": L23.dt_proj.weight.grad.clone(),
                        "D": L23.D.grad.clone(), "A_log": L23.A_log.grad.clone(),
                        "x_proj.weight": L23.x_proj.weight.grad.clone(), "out_proj.weight": L23.out_proj.weight.grad.clone()}
        rec["loss"] = float(loss.detach())
        runs.append(rec)
        line = {"run": r, "loss": rec["loss"], "n_scan_bwd": state["n"]}
        if args.debug:
            line["dbg"] = rec.pop("dbg_line")
            rec["dbg"] = None

        def eqt(x, y):
            if isinstance(x, torch.Tensor):
                return bool(isinstance(y, torch.Tensor) and x.shape == y.shape and torch.equal(x, y))
            return x == y
        line["solo_repeat_equal"] = all(eqt(x, y) for x, y in zip(rec["solo"][0], rec["solo"][1]))
        line["instep_vs_solo_differ"] = {}
        for j, nm in enumerate(OUT_NAMES):
            x, y = rec["outs"][j], rec["solo"][0][j]
            if isinstance(x, torch.Tensor) and not eqt(x, y):
                line["instep_vs_solo_differ"][nm] = {"n": int((x != y).sum()), "numel": x.numel(),
                                                     "max_abs": float((x.float() - y.float()).abs().max())}
        if args.pre_clone:
            line["inputs_changed_during_call"] = [IN_NAMES[j] for j, (x, y) in enumerate(zip(rec["pre"], ins))
                                                  if isinstance(x, torch.Tensor) and not eqt(x, y)]
        cnt = lambda t: dict(sorted(collections.Counter(t.tolist()).items())[:40])
        for j, nm in ((0, "du"), (6, "dz")):
            x, y = rec["outs"][j], rec["solo"][0][j]
            if isinstance(x, torch.Tensor) and not eqt(x, y):
                idx = (x != y).nonzero()
                line[nm + "_diff_channel_in_wave"] = cnt(idx[:, 1] % 32)
                line[nm + "_diff_chunk"] = cnt(idx[:, 2] // 32)
        x, y = rec["outs"][2], rec["solo"][0][2]
        if not eqt(x, y):   # dA (dim, N)
            idx = (x != y).nonzero()
            line["dA_diff_channel_in_wave"] = cnt(idx[:, 0] % 32)
            line["dA_diff_state"] = cnt(idx[:, 1])
        dd_x, dd_y = rec["outs"][1], rec["solo"][0][1]
        if not eqt(dd_x, dd_y):
            idx = (dd_x != dd_y).nonzero()
            b, d, l = idx[:, 0], idx[:, 1], idx[:, 2]
            cnt = lambda t: dict(sorted(collections.Counter(t.tolist()).items())[:40])
            line["ddelta_diff_where"] = {"batch": cnt(b), "wblk": cnt(d // 128), "wave": cnt((d % 128) // 32),
                                         "chunk": cnt(l // 32), "subtile": cnt((l % 32) // 8), "half": cnt((l % 8) // 4),
                                         "channel_in_wave": cnt(d % 32), "first": idx[:8].tolist()}
        if r > 0:
            r0 = runs[0]
            line["inputs_vs_run0_differ"] = [IN_NAMES[j] for j, (x, y) in enumerate(zip(r0["ins"], ins))
                                             if isinstance(x, torch.Tensor) and not eqt(x, y)]
            line["instep_outs_vs_run0_differ"] = [OUT_NAMES[j] for j, (x, y) in enumerate(zip(r0["outs"], rec["outs"]))
                                                  if isinstance(x, torch.Tensor) and not eqt(x, y)]
            line["solo_outs_vs_run0_solo_differ"] = [OUT_NAMES[j] for j, (x, y) in
                                                     enumerate(zip(r0["solo"][0], rec["solo"][0]))
                                                     if isinstance(x, torch.Tensor) and not eqt(x, y)]
            line["layer23_grads_vs_run0_differ"] = [k for k in rec["grads"] if not eqt(r0["grads"][k], rec["grads"][k])]
            line["loss_equal_run0"] = rec["loss"] == r0["loss"]
        # keep memory bounded: only run 0's record and the current one
        if r > 0:
            runs[-1] = {k: v for k, v in rec.items() if k in ()}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
