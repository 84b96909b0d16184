"""``selective_scan_fn`` -- drop-in for mamba_ssm's op, backed by HIP kernels.

Reference boundary: /root/reference/src/mamba_clip/model.py:27-28 imports
``mamba_ssm.ops.selective_scan_interface.selective_scan_fn`` and calls it at
model.py:539-550 (keyword style).  Same signature, same argument meaning, same
outputs (``out`` or ``(out, last_state)``), autograd-capable, errors surface as
``RuntimeError`` like upstream's TORCH_CHECKs.  Semantics: model.py:83-169.

The forward runs ``mc_scan_fwd`` and, when a gradient will be needed, saves
fp32 chunk states (one per MC_SCAN_CHUNK positions); the backward runs
``mc_scan_bwd`` from them.  Both launch on the current HIP stream and never
synchronise.  There is no CPU / eager fallback.
"""
import contextlib
import os
import threading

import torch

from . import _lib


def _prep_bc(M, name):
    """(B, N, L) -> (B, 1, N, L); (B, G, N, L) kept.  Unit stride along L."""
    if M.dim() == 3:
        M = M.unsqueeze(1)
    elif M.dim() != 4:
        raise RuntimeError(f"selective_scan_fn: {name} must be (B, N, L) or (B, G, N, L) (variable {name}); "
                           f"constant (D, N) {name} is not supported")
    if M.stride(-1) != 1:
        M = M.contiguous()
    return M


def _last_dim_contig(x):
    return x if x is None or x.stride(-1) == 1 else x.contiguous()


def _check_inputs(u, delta, A, B, C, D, z, delta_bias):
    if not u.is_cuda:
        raise RuntimeError("selective_scan_fn: inputs must be on the GPU (no CPU path)")
    if A.is_complex():
        raise RuntimeError("selective_scan_fn: complex A is not supported")
    if delta.dtype != u.dtype or (z is not None and z.dtype != u.dtype):
        raise RuntimeError("selective_scan_fn: u, delta and z must share a dtype")
    if C.dtype != B.dtype:
        raise RuntimeError("selective_scan_fn: B and C must share a dtype")
    batch, dim, L = u.shape
    if delta.shape != u.shape or (z is not None and z.shape != u.shape):
        raise RuntimeError("selective_scan_fn: u, delta, z shape mismatch")
    if A.shape[0] != dim:
        raise RuntimeError("selective_scan_fn: A must be (D, N)")
    dstate = A.shape[1]
    if dstate > _lib.MC_SCAN_MAX_DSTATE:
        raise RuntimeError(f"selective_scan_fn: dstate {dstate} > {_lib.MC_SCAN_MAX_DSTATE}")
    for M in (B, C):
        if M.shape[0] != batch or M.shape[2] != dstate or M.shape[3] != L:
            raise RuntimeError("selective_scan_fn: B/C must be (B, G, N, L)")
    if dim % B.shape[1] != 0:
        raise RuntimeError("selective_scan_fn: dim must be divisible by n_groups")


def fine_states_max_bytes():
    """Budget (bytes) for the fine saved states of one step's scan calls.  The fine interval costs 4x
    the default interval's memory and buys the backward's recompute pass: a C2 layer holds 252 MB of
    fine states instead of 63 MB, 6.0 GB instead of 1.5 GB for the 24 layers; a C4 layer (L 4096) would
    need 6.4 GB.  MAMBA_CLIP_AMD_FINE_STATES_MB sets it (default 8192 MB = C2 at batch 256 plus margin;
    0 = never)."""
    return int(float(os.environ.get("MAMBA_CLIP_AMD_FINE_STATES_MB", "8192")) * (1 << 20))


_FINE_SCOPE = threading.local()   # .calls: scan calls per step declared by the innermost fine_state_scope


@contextlib.contextmanager
def fine_state_scope(n_calls):
    """Declare that the enclosed forward makes ``n_calls`` training scan calls (a tower's layer count):
    each call may then take the fine interval when its own fine states fit ``budget / n_calls``.

    The choice is a function of the call's shapes, the budget and the declared count only -- never of
    what other autograd graphs happen to be alive (round 5 counted live bytes released by finalizers,
    so eval passes, checkpoint recompute or graph warm-up changed which interval, hence which bits, a
    layer produced: ADVICE r05).  Outside any scope a call counts as the step's only one."""
    prev = getattr(_FINE_SCOPE, "calls", None)
    _FINE_SCOPE.calls = max(1, int(n_calls))
    try:
        yield
    finally:
        _FINE_SCOPE.calls = prev


def fine_states_allowance():
    """Bytes of fine saved states one scan call may take (budget / declared calls per step)."""
    return fine_states_max_bytes() // (getattr(_FINE_SCOPE, "calls", None) or 1)


def states_interval(L, dim, states):
    """The interval a forward saved `states` with: default (B, dim, ceil(L / 32), N), or fine and
    position-major (B, ceil(L / 8), dim, N)."""
    fine = _lib.MC_SCAN_STATE_INTERVAL_FINE
    n_fine, n_def = -(-L // fine), -(-L // _lib.MC_SCAN_CHUNK)
    if states.shape[1] == dim and states.shape[2] == n_def:
        return 0
    if states.shape[1] == n_fine and states.shape[2] == dim:
        return fine
    raise RuntimeError(f"scan states of shape {tuple(states.shape)} match neither interval (L {L}, dim {dim})")


def scan_fwd(u, delta, A, B, C, D, z, delta_bias, delta_softplus, want_states, want_last, want_y=False,
             dirs=None, proj=None):
    """Run mc_scan_fwd.  Returns (out, chunk_states or None, last_state or None[, out_y]).

    ``dirs=(reverse_groups, u_groups)``: grouped directions (include/mc_scan.h):
    mirrored positions for the reversed groups, u shared in u_groups blocks.

    ``want_y`` (with z): also return the pre-gate output y + D u -- upstream's
    forward returns it as ``out`` next to ``out_z``.  Training does not need it:
    the backward recomputes y from the chunk states (saving it measured slower:
    +1.6 GB of forward writes at C4 for less backward work).

    ``proj=(dpx, dpw, delta_out)``: projected delta (include/mc_scan.h) -- delta is
    None and the kernel forms delta[b, d, l] = dpw[d] . dpx[b, l] itself; dpx is
    (batch, L, R) with unit stride along R, dpw (dim, R); ``delta_out`` (nullable,
    u's layout) receives the formed delta for the backward.
    """
    lib = _lib.load()
    batch, dim, L = (delta if delta is not None else u).shape
    dstate = A.shape[1]
    G = B.shape[1]
    # same (dense) layout as u: channel-major callers stay channel-major
    out = torch.empty_like(u) if dirs is None else torch.empty_like(delta)
    last = (torch.empty(batch, dim, dstate, device=u.device, dtype=torch.float32)
            if want_last and not want_states else None)
    p = _lib.ScanFwdParams()
    p.batch, p.dim, p.seqlen, p.dstate, p.n_groups = batch, dim, L, dstate, G
    p.itype, p.wtype = _lib.dtype_code(u.dtype), _lib.dtype_code(B.dtype)
    p.delta_softplus = int(bool(delta_softplus))
    p.u_batch_stride, p.u_dim_stride = u.stride(0), u.stride(1)
    if delta is not None:
        p.delta_batch_stride, p.delta_dim_stride = delta.stride(0), delta.stride(1)
    if z is not None:
        p.z_batch_stride, p.z_dim_stride = z.stride(0), z.stride(1)
    p.out_batch_stride, p.out_dim_stride = out.stride(0), out.stride(1)
    p.B_batch_stride, p.B_group_stride, p.B_dstate_stride = B.stride(0), B.stride(1), B.stride(2)
    p.C_batch_stride, p.C_group_stride, p.C_dstate_stride = C.stride(0), C.stride(1), C.stride(2)
    p.u, p.delta, p.A, p.B, p.C = u.data_ptr(), _lib.ptr(delta), A.data_ptr(), B.data_ptr(), C.data_ptr()
    p.D, p.z, p.delta_bias = _lib.ptr(D), _lib.ptr(z), _lib.ptr(delta_bias)
    p.out, p.last_state = out.data_ptr(), _lib.ptr(last)
    if proj is not None:
        dpx, dpw, delta_out = proj
        p.delta_proj_x, p.delta_proj_w, p.delta_rank = dpx.data_ptr(), dpw.data_ptr(), dpw.shape[1]
        p.dpx_batch_stride, p.dpx_token_stride, p.dpw_dim_stride = dpx.stride(0), dpx.stride(1), dpw.stride(0)
        if delta_out is not None:
            p.delta_out = delta_out.data_ptr()
            p.delta_batch_stride, p.delta_dim_stride = delta_out.stride(0), delta_out.stride(1)
    ws_bytes = lib.mc_scan_fwd_workspace_bytes(batch, L, dstate, G)
    ws = torch.empty(max(ws_bytes, 1), device=u.device, dtype=torch.uint8)
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws_bytes
    if dirs is not None:
        p.reverse_groups, p.u_groups = int(dirs[0]), int(dirs[1])
    out_y = torch.empty_like(u) if (want_y and z is not None) else None
    if out_y is not None:
        p.out_y, p.out_y_batch_stride, p.out_y_dim_stride = out_y.data_ptr(), out_y.stride(0), out_y.stride(1)
    states, nch = None, 0
    if want_states:
        # the fine saved-state interval where the pair kernel runs and the states fit the budget:
        # the backward then reads each sub-tile's entry state instead of recomputing it
        fine = _lib.MC_SCAN_STATE_INTERVAL_FINE
        fine_bytes = batch * dim * lib.mc_scan_n_states(L, fine) * dstate * 4
        if fine_bytes <= fine_states_allowance():
            p.state_interval = fine
            p.state_interval = lib.mc_scan_fwd_state_interval(p)
        nch = lib.mc_scan_n_states(L, p.state_interval)
        shape = (batch, nch, dim, dstate) if p.state_interval == fine else (batch, dim, nch, dstate)
        states = torch.empty(shape, device=u.device, dtype=torch.float32)
        p.chunk_states = states.data_ptr()
    if RECORD_DISPATCH:
        DISPATCH.append(("fwd", int(lib.mc_scan_fwd_kernel(p))))
    _lib.check(lib.mc_scan_fwd(p, _lib.stream_handle(u.device)), "mc_scan_fwd")
    if want_last and states is not None:
        if nch == 0:
            last = torch.zeros(batch, dim, dstate, device=u.device)
        else:
            last = states[:, -1] if p.state_interval == _lib.MC_SCAN_STATE_INTERVAL_FINE else states[:, :, -1, :]
    if want_y:
        return out, states, last, out_y
    return out, states, last


# Tests set RECORD_DISPATCH to see which kernel family (_lib.MC_SCAN_KERNEL_*) each call ran:
# DISPATCH collects ("fwd" | "bwd", code) per launch (mc_scan_fwd_kernel / mc_scan_bwd_kernel).
RECORD_DISPATCH = False
DISPATCH = []


def scan_bwd(u, delta, A, B, C, D, z, delta_bias, delta_softplus, dout, states, dirs=None, dz_out=None, proj=None,
             dbc_out=None):
    """Run mc_scan_bwd.  With ``dirs``, du comes back per group, (B, dim, L): the caller sums the
    groups that share a u block.  ``proj=(dpx, dpw)``: projected delta (delta None), as scan_fwd.
    ``dbc_out=(dB, dC)``: (batch, G, dstate, L) views (seqlen stride 1) the gradients are written into."""
    lib = _lib.load()
    if delta is None:
        delta = u   # shape / layout template only: with proj the kernel re-forms delta, never reads it
    batch, dim, L = delta.shape
    dstate = A.shape[1]
    G = B.shape[1]
    dout = _last_dim_contig(dout)
    du = torch.empty_like(u) if dirs is None else torch.empty_like(delta)
    ddelta = torch.empty_like(delta)
    dz = (dz_out if dz_out is not None else torch.empty_like(z)) if z is not None else None
    if dbc_out is not None:
        dB, dC = dbc_out
        if dB.shape != B.shape or dC.shape != C.shape or dB.dtype != B.dtype or dC.dtype != C.dtype \
                or dB.stride(-1) != 1 or dC.stride(-1) != 1:
            raise ValueError("scan_bwd: dbc_out views must match B / C (shape, dtype, seqlen stride 1)")
    else:
        dB = torch.empty(B.shape, device=u.device, dtype=B.dtype)
        dC = torch.empty(C.shape, device=u.device, dtype=C.dtype)
    dA = torch.empty(dim, dstate, device=u.device, dtype=torch.float32)
    dD = torch.empty(dim, device=u.device, dtype=torch.float32) if D is not None else None
    dbias = torch.empty(dim, device=u.device, dtype=torch.float32) if delta_bias is not None else None
    ws_bytes = lib.mc_scan_bwd_workspace_bytes(batch, dim, L, dstate, G)
    ws = torch.empty(max(ws_bytes, 1), device=u.device, dtype=torch.uint8)
    p = _lib.ScanBwdParams()
    p.batch, p.dim, p.seqlen, p.dstate, p.n_groups = batch, dim, L, dstate, G
    p.itype, p.wtype = _lib.dtype_code(u.dtype), _lib.dtype_code(B.dtype)
    p.delta_softplus = int(bool(delta_softplus))
    p.u_batch_stride, p.u_dim_stride = u.stride(0), u.stride(1)
    p.delta_batch_stride, p.delta_dim_stride = delta.stride(0), delta.stride(1)
    if z is not None:
        p.z_batch_stride, p.z_dim_stride = z.stride(0), z.stride(1)
    p.dout_batch_stride, p.dout_dim_stride = dout.stride(0), dout.stride(1)
    p.du_batch_stride, p.du_dim_stride = du.stride(0), du.stride(1)
    p.ddelta_batch_stride, p.ddelta_dim_stride = ddelta.stride(0), ddelta.stride(1)
    if dz is not None:
        p.dz_batch_stride, p.dz_dim_stride = dz.stride(0), dz.stride(1)
    p.B_batch_stride, p.B_group_stride, p.B_dstate_stride = B.stride(0), B.stride(1), B.stride(2)
    p.C_batch_stride, p.C_group_stride, p.C_dstate_stride = C.stride(0), C.stride(1), C.stride(2)
    p.u, p.delta, p.A, p.B, p.C = (u.data_ptr(), 0 if proj is not None else delta.data_ptr(), A.data_ptr(),
                                   B.data_ptr(), C.data_ptr())
    p.D, p.z, p.delta_bias = _lib.ptr(D), _lib.ptr(z), _lib.ptr(delta_bias)
    p.dout, p.chunk_states = dout.data_ptr(), states.data_ptr()
    p.state_interval = states_interval(L, dim, states)
    if proj is not None:
        dpx, dpw = proj
        p.delta_proj_x, p.delta_proj_w, p.delta_rank = dpx.data_ptr(), dpw.data_ptr(), dpw.shape[1]
        p.dpx_batch_stride, p.dpx_token_stride, p.dpw_dim_stride = dpx.stride(0), dpx.stride(1), dpw.stride(0)
    p.du, p.ddelta, p.dz, p.dB, p.dC = du.data_ptr(), ddelta.data_ptr(), _lib.ptr(dz), dB.data_ptr(), dC.data_ptr()
    if dbc_out is not None:
        p.dB_batch_stride, p.dB_group_stride, p.dB_dstate_stride = dB.stride(0), dB.stride(1), dB.stride(2)
        p.dC_batch_stride, p.dC_group_stride, p.dC_dstate_stride = dC.stride(0), dC.stride(1), dC.stride(2)
    p.dA, p.dD, p.ddelta_bias = dA.data_ptr(), _lib.ptr(dD), _lib.ptr(dbias)
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws_bytes
    if dirs is not None:
        p.reverse_groups, p.u_groups = int(dirs[0]), int(dirs[1])
    if RECORD_DISPATCH:
        DISPATCH.append(("bwd", int(lib.mc_scan_bwd_kernel(p))))
    _lib.check(lib.mc_scan_bwd(p, _lib.stream_handle(u.device)), "mc_scan_bwd")
    return du, ddelta, dA, dB, dC, dD, dz, dbias


class SelectiveScanFn(torch.autograd.Function):
    """Autograd wrapper; mirrors mamba_ssm's SelectiveScanFn contract."""

    @staticmethod
    def forward(ctx, u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                return_last_state=False, dz_slab=None, du_handoff=None, dbc_slab=None):
        u, delta, z = _last_dim_contig(u), _last_dim_contig(delta), _last_dim_contig(z)
        squeeze_B, squeeze_C = B.dim() == 3, C.dim() == 3
        B, C = _prep_bc(B, "B"), _prep_bc(C, "C")
        A32 = A.float().contiguous()
        D32 = D.float().contiguous() if D is not None else None
        bias32 = delta_bias.float().contiguous() if delta_bias is not None else None
        _check_inputs(u, delta, A32, B, C, D32, z, bias32)
        need_grad = any(ctx.needs_input_grad[:8])
        out, states, last = scan_fwd(u, delta, A32, B, C, D32, z, bias32, delta_softplus,
                                     want_states=need_grad, want_last=return_last_state)
        if need_grad:
            ctx.save_for_backward(u, delta, A32, B, C, D32, z, bias32, states)
        ctx.delta_softplus = delta_softplus
        ctx.squeeze = (squeeze_B, squeeze_C)
        ctx.dtypes = (A.dtype, D.dtype if D is not None else None,
                      delta_bias.dtype if delta_bias is not None else None)
        ctx.has = (D is not None, z is not None, delta_bias is not None)
        ctx.dz_slab = dz_slab   # (GradSlab, first row): dz written into that slab (ops.GradSlab)
        ctx.du_handoff = du_handoff   # ops.GradHandoff: du parked for x_proj's backward (no u gradient here)
        ctx.dbc_slab = dbc_slab       # (GradSlab, B's first row, C's first row): dB / dC written there
        return (out, last) if return_last_state else out

    @staticmethod
    def backward(ctx, dout, *args):
        u, delta, A32, B, C, D32, z, bias32, states = ctx.saved_tensors
        dz_out = None
        if ctx.dz_slab is not None and z is not None:
            slab, r0 = ctx.dz_slab
            dz_out = slab.block(r0, r0 + z.shape[1], z.shape[0])
        dbc_out = None
        if ctx.dbc_slab is not None and B.shape[1] == 1 and C.shape[1] == 1:
            slab, rb, rc = ctx.dbc_slab
            n, bsz = B.shape[2], B.shape[0]
            dbc_out = (slab.block(rb, rb + n, bsz).unsqueeze(1), slab.block(rc, rc + n, bsz).unsqueeze(1))
        du, ddelta, dA, dB, dC, dD, dz, dbias = scan_bwd(u, delta, A32, B, C, D32, z, bias32,
                                                         ctx.delta_softplus, dout, states, dz_out=dz_out,
                                                         dbc_out=dbc_out)
        if ctx.squeeze[0]:
            dB = dB.squeeze(1)
        if ctx.squeeze[1]:
            dC = dC.squeeze(1)
        a_dt, d_dt, b_dt = ctx.dtypes
        if ctx.du_handoff is not None:
            ctx.du_handoff.du, du = du, None
        return (du, ddelta, dA.to(a_dt), dB, dC,
                dD.to(d_dt) if dD is not None else None,
                dz,
                dbias.to(b_dt) if dbias is not None else None,
                None, None, None, None, None)


class ProjectedScanFn(torch.autograd.Function):
    """The Mamba mixer's dt_proj + selective scan as one op (upstream mamba_inner_fn's fusion of
    the delta projection; reference model.py:519-528, 630-647):

        delta = dt_proj.weight @ dt_raw   (per token, rank R)
        out   = selective_scan(u, delta, A, B, C, D, z, delta_bias, softplus)

    ``dt_raw`` arrives token-major, (batch * L, R); both scan kernels form delta per chunk on the
    matrix cores (the ``delta_proj_*`` fields of mc_scan.h), so the (batch, dim, L) delta never
    touches HBM: no dt_proj GEMM output, no forward or backward read of it.  The backward's ddelta
    then gives dt_raw's and the weight's gradients as GEMMs.
    """

    @staticmethod
    def forward(ctx, u, dt_raw, weight, A, B, C, D, z, delta_bias, delta_softplus, dz_slab=None):
        batch, dim, L = u.shape
        R = weight.shape[1]
        w = weight.to(u.dtype).contiguous()
        dpx = dt_raw.view(batch, L, R)
        squeeze_B, squeeze_C = B.dim() == 3, C.dim() == 3
        B, C = _prep_bc(B, "B"), _prep_bc(C, "C")
        A32 = A.float().contiguous()
        D32 = D.float().contiguous() if D is not None else None
        bias32 = delta_bias.float().contiguous() if delta_bias is not None else None
        _check_inputs(u, u, A32, B, C, D32, z, bias32)
        need_grad = any(ctx.needs_input_grad[:9])
        out, states, _ = scan_fwd(u, None, A32, B, C, D32, z, bias32, delta_softplus,
                                  want_states=need_grad, want_last=False, proj=(dpx, w, None))
        if need_grad:
            ctx.save_for_backward(u, A32, B, C, D32, z, bias32, states, dt_raw, w)
        ctx.delta_softplus = delta_softplus
        ctx.squeeze = (squeeze_B, squeeze_C)
        ctx.dtypes = (weight.dtype, A.dtype, D.dtype if D is not None else None,
                      delta_bias.dtype if delta_bias is not None else None)
        ctx.dz_slab = dz_slab
        return out

    @staticmethod
    def backward(ctx, dout):
        u, A32, B, C, D32, z, bias32, states, dt_raw, w = ctx.saved_tensors
        dz_out = None
        if ctx.dz_slab is not None and z is not None:
            slab, r0 = ctx.dz_slab
            dz_out = slab.block(r0, r0 + z.shape[1], z.shape[0])
        batch, dim, L = u.shape
        du, ddelta, dA, dB, dC, dD, dz, dbias = scan_bwd(u, None, A32, B, C, D32, z, bias32, ctx.delta_softplus,
                                                         dout, states, dz_out=dz_out,
                                                         proj=(dt_raw.view(batch, L, w.shape[1]), w))
        # ddelta has u's layout; as a (dim, batch * L) matrix it is channel-major rows
        g = ddelta.transpose(0, 1).reshape(dim, batch * L)
        from .ops import wgrad
        d_raw = torch.mm(g.t(), w) if ctx.needs_input_grad[1] else None
        d_w = wgrad(g, dt_raw) if ctx.needs_input_grad[2] else None
        if ctx.squeeze[0]:
            dB = dB.squeeze(1)
        if ctx.squeeze[1]:
            dC = dC.squeeze(1)
        w_dt, a_dt, d_dt, b_dt = ctx.dtypes
        return (du, d_raw, d_w.to(w_dt) if d_w is not None else None, dA.to(a_dt), dB, dC,
                dD.to(d_dt) if dD is not None else None, dz,
                dbias.to(b_dt) if dbias is not None else None, None, None)


def projected_scan_ok(u, rank, dstate):
    """Shapes the projected-delta scan takes (the pair kernel's: mc_scan.h)."""
    return (u.is_cuda and u.dtype in (torch.bfloat16, torch.float16) and dstate == 16 and u.shape[2] % 8 == 0
            and rank % 16 == 0 and 16 <= rank <= 256)


def selective_scan_fn(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                      return_last_state=False):
    """out = selective_scan(u, delta, A, B, C, D, z, delta_bias, softplus) [, last_state].

    u, delta, z: (B, D, L);  A: (D, N) real;  B, C: (B, N, L) or (B, G, N, L);
    D, delta_bias: (D,).  ``last_state`` is the fp32 (B, D, N) state after the
    last position.  Output dtype = u.dtype.
    """
    return SelectiveScanFn.apply(u, delta, A, B, C, D, z, delta_bias, delta_softplus, return_last_state)


class GroupedScanFn(torch.autograd.Function):
    """Scan whose n_groups groups are independent directions: group g reads u block
    g % u_groups and, if bit g of reverse_groups is set, walks its sequence backwards
    at mirrored positions (mc_scan_*_params.reverse_groups / u_groups).  SS2D's four
    cross-scan directions are ONE call per pass on u = [x, x^T]: no flipped copies
    of the inputs, no un-flip of the outputs (reference model.py:510-517, 553-565)."""

    @staticmethod
    def forward(ctx, u, delta, A, B, C, D, delta_bias, delta_softplus, reverse_groups, u_groups):
        u, delta = _last_dim_contig(u), _last_dim_contig(delta)
        B, C = _prep_bc(B, "B"), _prep_bc(C, "C")
        A32 = A.float().contiguous()
        D32 = D.float().contiguous() if D is not None else None
        bias32 = delta_bias.float().contiguous() if delta_bias is not None else None
        batch, dim, L = delta.shape
        G = B.shape[1]
        if not (1 <= u_groups <= G and G % u_groups == 0):
            # the backward sums the G / u_groups groups sharing a u block (du.view(b, G // k, k, ...))
            raise RuntimeError(f"grouped_scan_fn: u_groups={u_groups} must divide n_groups={G}")
        if (dim % G or u.shape != (batch, u_groups * (dim // G), L) or B.shape[0] != batch
                or B.shape[3] != L or C.shape != B.shape):
            raise RuntimeError("grouped_scan_fn: u (B, u_groups*dim/G, L), delta (B, dim, L), B/C (B, G, N, L) expected")
        if not u.is_cuda or delta.dtype != u.dtype or C.dtype != B.dtype:
            raise RuntimeError("grouped_scan_fn: GPU tensors; u / delta and B / C must share dtypes")
        need_grad = any(ctx.needs_input_grad[:7])
        dirs = (int(reverse_groups), int(u_groups))
        out, states, _ = scan_fwd(u, delta, A32, B, C, D32, None, bias32, delta_softplus, want_states=need_grad,
                                  want_last=False, dirs=dirs)
        if need_grad:
            ctx.save_for_backward(u, delta, A32, B, C, D32, bias32, states)
        ctx.cfg = (delta_softplus, dirs, A.dtype, D.dtype if D is not None else None,
                   delta_bias.dtype if delta_bias is not None else None)
        return out

    @staticmethod
    def backward(ctx, dout):
        u, delta, A32, B, C, D32, bias32, states = ctx.saved_tensors
        softplus, dirs, a_dt, d_dt, b_dt = ctx.cfg
        du, ddelta, dA, dB, dC, dD, _, dbias = scan_bwd(u, delta, A32, B, C, D32, None, bias32, softplus, dout,
                                                        states, dirs=dirs)
        G, k = B.shape[1], dirs[1]
        # u block j's gradient: sum of the groups g = j (mod k) that read it (fp32 accumulate;
        # with 16-bit I/O each group's part was rounded once to the I/O dtype by the kernel)
        batch, dim, L = du.shape
        du_u = du.view(batch, G // k, k, dim // G, L).sum(1, dtype=torch.float32).to(u.dtype).view(u.shape)
        return (du_u, ddelta, dA.to(a_dt), dB, dC, dD.to(d_dt) if dD is not None else None,
                dbias.to(b_dt) if dbias is not None else None, None, None, None)


def grouped_scan_fn(u, delta, A, B, C, D=None, delta_bias=None, delta_softplus=False, reverse_groups=0,
                    u_groups=1):
    """out (B, dim, L) = selective scan of each of the n_groups = B.shape[1] groups, where group g
    reads u block g % u_groups (u: (B, u_groups * dim / n_groups, L)) and runs backwards over
    mirrored positions if bit g of reverse_groups is set (its output lands at the positions it
    read).  delta (B, dim, L); B, C (B, n_groups, N, L); A (dim, N); D, delta_bias (dim,)."""
    return GroupedScanFn.apply(u, delta, A, B, C, D, delta_bias, delta_softplus, reverse_groups, u_groups)


# SS2D's four cross-scan directions over u = [x, x^T]: 0 = x, 1 = x^T, 2 = flip(x), 3 = flip(x^T)
SS2D_REVERSE_GROUPS = 0b1100
SS2D_U_GROUPS = 2
