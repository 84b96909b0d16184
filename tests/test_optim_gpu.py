"""optim.HipAdamW (mc_adamw_step: one launch over every parameter) against torch.optim.AdamW's
reference (single-tensor) path: same groups, same hyper-parameters, several steps, odd sizes and
unaligned views; plus state-dict exchange with torch's AdamW and a learning-rate change mid-run."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    shapes = [(3072, 768), (768,), (5,), (1,), (37, 53), (70001,), (2, 65536 + 3)]
    return [torch.randn(s, device=DEV, generator=g).requires_grad_(True) for s in shapes]


def _grads(ps, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return [torch.randn(p.shape, device=DEV, generator=g) for p in ps]


def _groups(ps):
    return [{"params": ps[:3], "weight_decay": 0.0}, {"params": ps[3:], "weight_decay": 0.2}]


def test_hip_adamw_matches_torch_adamw():
    from mamba_clip_amd.optim import HipAdamW
    a, b = _params(0), _params(0)
    oa = HipAdamW(_groups(a), lr=1e-3, betas=(0.9, 0.98), eps=1e-6)
    ob = torch.optim.AdamW(_groups(b), lr=1e-3, betas=(0.9, 0.98), eps=1e-6, foreach=False)
    for step in range(5):
        if step == 3:
            for o in (oa, ob):
                for grp in o.param_groups:
                    grp["lr"] = 5e-4
        for ps in (a, b):
            for p, gr in zip(ps, _grads(ps, 100 + step)):
                p.grad = gr
        oa.step()
        ob.step()
    for pa, pb in zip(a, b):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)
        sa, sb = oa.state[pa], ob.state[pb]
        torch.testing.assert_close(sa["exp_avg"], sb["exp_avg"], rtol=1e-5, atol=1e-7)   # b1 m + (1-b1) g vs lerp: 1-ulp differences
        torch.testing.assert_close(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-5, atol=1e-8)
        assert float(sa["step"]) == float(sb["step"]) == 5.0


def test_hip_adamw_state_dict_roundtrip_with_torch():
    from mamba_clip_amd.optim import HipAdamW
    a, b = _params(1), _params(1)
    oa = HipAdamW(_groups(a), lr=2e-3)
    for p, gr in zip(a, _grads(a, 7)):
        p.grad = gr
    oa.step()
    # HipAdamW state -> torch AdamW, one more step each: identical trajectories
    ob = torch.optim.AdamW(_groups(b), lr=2e-3, foreach=False)
    with torch.no_grad():
        for pa, pb in zip(a, b):
            pb.copy_(pa)
    ob.load_state_dict(copy.deepcopy(oa.state_dict()))   # load_state_dict keeps same-device tensors as is
    oc = HipAdamW(_groups(_params(1)), lr=2e-3)
    oc.load_state_dict(copy.deepcopy(ob.state_dict()))   # and back into a fresh HipAdamW
    c = [p for grp in oc.param_groups for p in grp["params"]]
    with torch.no_grad():
        for pc, pa in zip(c, a):
            pc.copy_(pa)
    for ps in (a, b, c):
        for p, gr in zip(ps, _grads(ps, 8)):
            p.grad = gr
    oa.step()
    ob.step()
    oc.step()
    for pa, pb, pc in zip(a, b, c):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(pc, pa, rtol=0, atol=0)


def test_hip_adamw_skips_params_without_grad_and_rejects_fp16():
    from mamba_clip_amd.optim import HipAdamW
    ps = _params(2)
    before = [p.detach().clone() for p in ps]
    o = HipAdamW(_groups(ps), lr=1e-2)
    ps[0].grad = torch.ones_like(ps[0])
    o.step()
    assert not torch.equal(ps[0], before[0])
    for p, q in zip(ps[1:], before[1:]):
        assert torch.equal(p, q)
    h = torch.zeros(4, device=DEV, dtype=torch.float16, requires_grad=True)
    o2 = HipAdamW([h])
    h.grad = torch.ones_like(h)
    with pytest.raises(RuntimeError, match="fp32"):
        o2.step()


def test_hip_adamw_per_parameter_steps_match_torch():
    """step counts are per parameter.  A parameter that skips a step keeps its count and
    bias corrections, one whose first gradient comes late starts at 1, and a torch state dict whose
    parameters of one group have different counts loads and resumes (torch AdamW, single-tensor path,
    as the oracle)."""
    from mamba_clip_amd.optim import HipAdamW
    a, b = _params(3), _params(3)
    oa = HipAdamW(_groups(a), lr=1e-3, betas=(0.9, 0.98), eps=1e-6)
    ob = torch.optim.AdamW(_groups(b), lr=1e-3, betas=(0.9, 0.98), eps=1e-6, foreach=False)
    # step k: which parameters get a gradient (param 1 skips step 1, param 4 starts at step 2, ...)
    plan = [{0, 1, 3, 5}, {0, 3, 5, 6}, {0, 1, 3, 4, 5, 6}, {1, 2, 4}, set(range(7))]
    for k, have in enumerate(plan):
        for ps in (a, b):
            grads = _grads(ps, 300 + k)
            for i, p in enumerate(ps):
                p.grad = grads[i] if i in have else None
        oa.step()
        ob.step()
    for i, (pa, pb) in enumerate(zip(a, b)):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6, msg=f"param {i}")
        assert float(oa.state[pa]["step"]) == float(ob.state[pb]["step"]), i
    # torch's state (different step counts inside each group) -> a fresh HipAdamW, two more steps
    c = _params(3)
    with torch.no_grad():
        for pc, pb in zip(c, b):
            pc.copy_(pb)
    oc = HipAdamW(_groups(c), lr=1e-3, betas=(0.9, 0.98), eps=1e-6)
    oc.load_state_dict(copy.deepcopy(ob.state_dict()))
    for k in range(2):
        for ps in (b, c):
            for p, gr in zip(ps, _grads(ps, 400 + k)):
                p.grad = gr
        ob.step()
        oc.step()
    for i, (pc, pb) in enumerate(zip(c, b)):
        torch.testing.assert_close(pc, pb, rtol=1e-5, atol=1e-6, msg=f"param {i}")
        assert float(oc.state[pc]["step"]) == float(ob.state[pb]["step"]), i
    # the saved form is torch's: one step tensor per parameter
    sd = oc.state_dict()
    steps = [v["step"] for v in sd["state"].values()]
    assert len({id(t) for t in steps}) == len(steps)


def test_hip_adamw_many_buckets_split_launches():
    """More (group, step) buckets than MC_ADAMW_MAX_GROUPS: several launches, same result as torch."""
    from mamba_clip_amd import _lib
    from mamba_clip_amd.optim import HipAdamW
    n = _lib.MC_ADAMW_MAX_GROUPS + 3
    g = torch.Generator(device=DEV).manual_seed(9)
    a = [torch.randn(1000 + 7 * i, device=DEV, generator=g).requires_grad_(True) for i in range(n)]
    b = [p.detach().clone().requires_grad_(True) for p in a]
    oa = HipAdamW([{"params": [p]} for p in a], lr=1e-3)
    ob = torch.optim.AdamW([{"params": [p]} for p in b], lr=1e-3, foreach=False)
    for k in range(n):            # parameter i starts at step i: n distinct step counts at the end
        for ps in (a, b):
            grads = _grads(ps, 500 + k)
            for i, p in enumerate(ps):
                p.grad = grads[i] if i <= k else None
        oa.step()
        ob.step()
    for pa, pb in zip(a, b):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)
