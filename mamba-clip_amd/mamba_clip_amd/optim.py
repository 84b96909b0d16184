"""AdamW whose step is one HIP launch over every parameter (include/mc_ops.h mc_adamw_step).

Drop-in for the reference's optimizer (torch.optim.AdamW built in create_optimizer, reference
train.py / main.py): the same param_groups (lr, betas, eps, weight_decay), the
same update rule (decoupled weight decay, bias-corrected moments, no amsgrad), and torch AdamW's
state layout (`step`, `exp_avg`, `exp_avg_sq` per parameter), so state dicts move between the two.

Why: torch's fused AdamW runs the C2 step's 216 M fp32 parameters as ~17 multi-tensor launches at
~4 TB/s (1.46 ms per step); one launch over a device chunk table streams them at the HBM rate.
The chunk table (tensor index, group, offset, length) is built once per parameter set; the
per-tensor pointer table is rewritten each step because gradients may be re-allocated
(zero_grad(set_to_none=True)).  Step counts are per group (every parameter of a group steps
together); each parameter's state['step'] is a view of its group's counter.
"""
import math

import torch

from . import _lib


class HipAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"HipAdamW: invalid hyper-parameters lr={lr} betas={betas} eps={eps}")
        # torch AdamW's group keys too, so a state dict loads into either optimizer unchanged
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=False, differentiable=False,
                                      fused=None, decoupled_weight_decay=True))
        if len(self.param_groups) > _lib.MC_ADAMW_MAX_GROUPS:
            raise ValueError(f"HipAdamW: at most {_lib.MC_ADAMW_MAX_GROUPS} parameter groups")
        self._plan = None

    # ---- state
    def _group_step(self, gi, group):
        """The group's step counter (a CPU float tensor shared by its parameters' state['step'])."""
        st = group.get("_step_t")
        if st is None:
            steps = [float(self.state[p]["step"]) for p in group["params"] if "step" in self.state.get(p, {})]
            if steps and min(steps) != max(steps):
                raise RuntimeError("HipAdamW: parameters of one group have different step counts")
            st = torch.tensor(steps[0] if steps else 0.0, dtype=torch.float32)
            group["_step_t"] = st
        return st

    def _init_state(self, p, st):
        s = self.state[p]
        if "exp_avg" not in s:
            s["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            s["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        s["step"] = st
        return s

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        for group in self.param_groups:
            group.pop("_step_t", None)
        self._plan = None

    def state_dict(self):
        sd = super().state_dict()
        for g in sd["param_groups"]:
            g.pop("_step_t", None)
        # one step tensor per parameter, as torch's AdamW saves it (the live state keeps the shared one)
        sd["state"] = {k: dict(v, step=v["step"].clone()) if "step" in v else v for k, v in sd["state"].items()}
        return sd

    # ---- step
    def _build_plan(self, live):
        chunks, tensors = [], []
        for ti, (gi, p, s) in enumerate(live):
            n = p.numel()
            for off in range(0, n, _lib.MC_ADAMW_CHUNK):
                chunks.append((ti | (gi << 32), off, min(_lib.MC_ADAMW_CHUNK, n - off)))
            tensors.append((p.data_ptr(), s["exp_avg"].data_ptr(), s["exp_avg_sq"].data_ptr()))
        dev = live[0][1].device
        key = tuple((id(p), p.data_ptr(), id(s["exp_avg"])) for _, p, s in live)
        return dict(key=key, n=len(chunks), chunks=torch.tensor(chunks, dtype=torch.int64).to(dev),
                    base=tensors, dev=dev)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        live, hyper = [], _lib.AdamWHyper()
        hyper.n_groups = len(self.param_groups)
        for gi, group in enumerate(self.param_groups):
            if group.get("amsgrad") or group.get("maximize") or not group.get("decoupled_weight_decay", True):
                raise RuntimeError("HipAdamW: amsgrad / maximize / coupled weight decay are not supported")
            ps = [p for p in group["params"] if p.grad is not None]
            st = self._group_step(gi, group)
            if ps:
                st += 1.0
            t = float(st)
            b1, b2 = group["betas"]
            h = hyper.group[gi]
            h.beta1, h.beta2, h.eps = b1, b2, group["eps"]
            h.decay = 1.0 - group["lr"] * group["weight_decay"]
            h.step_size = group["lr"] / (1.0 - b1 ** t) if t > 0 else 0.0
            h.bc2_sqrt = math.sqrt(1.0 - b2 ** t) if t > 0 else 1.0
            for p in ps:
                if p.grad.is_sparse:
                    raise RuntimeError("HipAdamW does not support sparse gradients")
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()
                        and p.grad.dtype == torch.float32 and p.grad.is_contiguous()):
                    raise RuntimeError("HipAdamW: fp32 contiguous CUDA parameters and gradients only")
                live.append((gi, p, self._init_state(p, st)))
        if not live:
            return loss
        key = tuple((id(p), p.data_ptr(), id(s["exp_avg"])) for _, p, s in live)
        if self._plan is None or self._plan["key"] != key:
            self._plan = self._build_plan(live)
        plan = self._plan
        rows = [b + (p.grad.data_ptr(),) for b, (_, p, _) in zip(plan["base"], live)]
        tens = torch.tensor(rows, dtype=torch.int64).pin_memory().to(plan["dev"], non_blocking=True)
        _lib.check(_lib.load().mc_adamw_step(plan["n"], plan["chunks"].data_ptr(), tens.data_ptr(), hyper,
                                             _lib.stream_handle(plan["dev"])), "mc_adamw_step")
        plan["tens"] = tens     # kept until the next step (the launch reads it asynchronously)
        return loss
