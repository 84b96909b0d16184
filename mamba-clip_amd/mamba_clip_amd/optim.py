"""AdamW whose step is one HIP launch over every parameter (include/mc_ops.h mc_adamw_step).

Drop-in for the reference's optimizer (torch.optim.AdamW built in create_optimizer, reference
train.py / main.py): the same param_groups (lr, betas, eps, weight_decay), the
same update rule (decoupled weight decay, bias-corrected moments, no amsgrad), and torch AdamW's
state layout (`step`, `exp_avg`, `exp_avg_sq` per parameter), so state dicts move between the two.

Why: torch's fused AdamW runs the C2 step's 216 M fp32 parameters as ~17 multi-tensor launches at
~4 TB/s (1.46 ms per step); one launch over a device chunk table streams them at the HBM rate.
The chunk table (tensor index, bucket, offset, length) is built once per parameter set; the
per-tensor pointer table is rewritten each step because gradients may be re-allocated
(zero_grad(set_to_none=True)).

Step counts are per parameter, as in torch's AdamW: a parameter without a gradient keeps its count
(and so its bias corrections), one whose first gradient comes late starts at 1.  The launch carries
its hyper-parameters per *bucket* = (param group, step count); when every parameter of a group steps
together -- the normal case -- there is one bucket per group.  Parameters that step together share
one CPU step tensor (one in-place increment per bucket, not one per parameter); a bucket whose
members diverge is split.  More than MC_ADAMW_MAX_GROUPS buckets take several launches.
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
        self._plans = {}

    # ---- state
    def _share_steps(self):
        """Parameters of one group with equal step counts share one step tensor (after a state-dict
        load every parameter has its own)."""
        for group in self.param_groups:
            shared = {}
            for p in group["params"]:
                s = self.state.get(p)
                if s is None or "step" not in s:
                    continue
                t = float(s["step"])
                if t not in shared:
                    shared[t] = torch.tensor(t, dtype=torch.float32)
                s["step"] = shared[t]

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._share_steps()
        self._plans = {}

    def state_dict(self):
        sd = super().state_dict()
        # one step tensor per parameter, as torch's AdamW saves it (the live state shares them)
        sd["state"] = {k: dict(v, step=v["step"].clone()) if "step" in v else v for k, v in sd["state"].items()}
        return sd

    def _advance_steps(self, group, ps):
        """Increment the step count of every parameter in ps (those with a gradient), per parameter."""
        movers = {}
        fresh = []
        for p in ps:
            s = self.state[p]
            if "exp_avg" not in s:
                s["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                s["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st = s.get("step")
            if st is None:
                fresh.append(s)
            else:
                movers.setdefault(id(st), (st, []))[1].append(s)
        if fresh:
            one = torch.tensor(1.0, dtype=torch.float32)
            for s in fresh:
                s["step"] = one
        if not movers:
            return
        # how many parameters of the group hold each moving step tensor (tensors are shared only
        # within a group; the fresh parameters' new tensor is not among them)
        holders = {}
        for p in group["params"]:
            st = self.state.get(p, {}).get("step")
            if st is not None and id(st) in movers:
                holders[id(st)] = holders.get(id(st), 0) + 1
        for key, (st, states) in movers.items():
            if len(states) == holders[key]:
                st += 1.0                              # the whole bucket steps: one shared increment
            else:
                nxt = st + 1.0                         # the bucket splits: movers get their own tensor
                for s in states:
                    s["step"] = nxt

    # ---- step
    @staticmethod
    def _build_plan(live, dev):
        chunks, tensors = [], []
        for ti, (bi, p, s) in enumerate(live):
            n = p.numel()
            for off in range(0, n, _lib.MC_ADAMW_CHUNK):
                chunks.append((ti | (bi << 32), off, min(_lib.MC_ADAMW_CHUNK, n - off)))
            tensors.append((p.data_ptr(), s["exp_avg"].data_ptr(), s["exp_avg_sq"].data_ptr()))
        return dict(n=len(chunks), chunks=torch.tensor(chunks, dtype=torch.int64).to(dev), base=tensors)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        buckets = {}          # (group index, step count) -> [(p, state)]
        for gi, group in enumerate(self.param_groups):
            if group.get("amsgrad") or group.get("maximize") or not group.get("decoupled_weight_decay", True):
                raise RuntimeError("HipAdamW: amsgrad / maximize / coupled weight decay are not supported")
            ps = [p for p in group["params"] if p.grad is not None]
            for p in ps:
                if p.grad.is_sparse:
                    raise RuntimeError("HipAdamW does not support sparse gradients")
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()
                        and p.grad.dtype == torch.float32 and p.grad.is_contiguous()):
                    raise RuntimeError("HipAdamW: fp32 contiguous CUDA parameters and gradients only")
            self._advance_steps(group, ps)
            for p in ps:
                s = self.state[p]
                buckets.setdefault((gi, float(s["step"])), []).append((p, s))
        if not buckets:
            return loss
        keys = list(buckets)
        per = _lib.MC_ADAMW_MAX_GROUPS
        for b0 in range(0, len(keys), per):
            self._launch([(k, buckets[k]) for k in keys[b0:b0 + per]])
        return loss

    def _launch(self, bucket_list):
        hyper = _lib.AdamWHyper()
        hyper.n_groups = len(bucket_list)
        live = []
        for bi, ((gi, t), members) in enumerate(bucket_list):
            group = self.param_groups[gi]
            b1, b2 = group["betas"]
            h = hyper.group[bi]
            h.beta1, h.beta2, h.eps = b1, b2, group["eps"]
            h.decay = 1.0 - group["lr"] * group["weight_decay"]
            h.step_size = group["lr"] / (1.0 - b1 ** t)
            h.bc2_sqrt = math.sqrt(1.0 - b2 ** t)
            live.extend((bi, p, s) for p, s in members)
        dev = live[0][1].device
        key = tuple((bi, id(p), p.data_ptr(), id(s["exp_avg"])) for bi, p, s in live)
        plan = self._plans.get(key)
        if plan is None:
            if len(self._plans) > 16:
                self._plans.clear()
            plan = self._plans[key] = self._build_plan(live, dev)
        rows = [b + (p.grad.data_ptr(),) for b, (_, p, _) in zip(plan["base"], live)]
        tens = torch.tensor(rows, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
        _lib.check(_lib.load().mc_adamw_step(plan["n"], plan["chunks"].data_ptr(), tens.data_ptr(), hyper,
                                             _lib.stream_handle(dev)), "mc_adamw_step")
        plan["tens"] = tens     # kept until this plan's next launch (the kernel reads it asynchronously)
