"""Selective-scan CPU oracle (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Restates the reference semantics the reference repo embeds as text at
/root/reference/src/mamba_clip/model.py:83-169 (the ``selective_scan_ref``
body quoted inside ``flops_selective_scan_ref``), which is what the third-party
``mamba_ssm.ops.selective_scan_interface.selective_scan_fn`` computes
(call site model.py:539-550):

    delta = softplus(delta + delta_bias[d])                       (model.py:88-91)
    x_t[b,d,n] = exp(delta_t A[d,n]) x_{t-1} + delta_t B[b,g(d),n,t] u_t
                                                                  (model.py:118-127, 141)
    y_t[b,d]   = sum_n C[b,g(d),n,t] x_t[b,d,n]                   (model.py:142-148)
    out = y + D[d] u  ; out *= silu(z)  ; out.to(dtype_in)        (model.py:163-168)
    last_state = x_{L-1}                                          (model.py:149-150)

Only real A and variable (3-D ``(B,N,L)`` or grouped 4-D ``(B,G,N,L)``) B/C
are supported -- the shapes every call site in the reference uses.  The
restatement is written independently (a per-step loop over a (B,D,N) state,
group index g(d) = d // (D/G)); tests pin it against vectors generated from
the reference's own text (tests/golden/make_golden.py).
"""
import torch
import torch.nn.functional as F


def _expand_groups(M, dim):
    """(B,N,L) or (B,G,N,L) -> (B,D,N,L) with channel d reading group d // (D/G)."""
    if M.dim() == 3:
        return M.unsqueeze(1).expand(M.shape[0], dim, M.shape[1], M.shape[2])
    G = M.shape[1]
    if dim % G != 0:
        raise ValueError(f"dim {dim} not divisible by n_groups {G}")
    return M.repeat_interleave(dim // G, dim=1)


def selective_scan_ref(u, delta, A, B, C, D=None, z=None, delta_bias=None,
                       delta_softplus=False, return_last_state=False,
                       compute_dtype=torch.float32):
    """Oracle forward.  Differentiable (autograd gives the backward oracle).

    u, delta, z: (B, D, L);  A: (D, N) real;  B, C: (B, N, L) or (B, G, N, L);
    D, delta_bias: (D,).  Computes in ``compute_dtype`` (fp32 like the
    reference, or fp64 for a tighter check) and returns ``out`` cast back to
    ``u.dtype`` (and the fp32/fp64 last state if requested).
    """
    if A.is_complex():
        raise NotImplementedError("complex A is not on the reference hot path")
    if B.dim() < 3 or C.dim() < 3:
        raise NotImplementedError("constant (D,N) B/C is not on the reference hot path")
    dtype_in = u.dtype
    cd = compute_dtype
    batch, dim, L = u.shape
    uf = u.to(cd)
    dt = delta.to(cd)
    if delta_bias is not None:
        dt = dt + delta_bias.to(cd)[:, None]
    if delta_softplus:
        dt = F.softplus(dt)          # threshold 20, as F.softplus in the reference
    Af = A.to(cd)
    Bf = _expand_groups(B.to(cd), dim)   # (B, D, N, L)
    Cf = _expand_groups(C.to(cd), dim)
    state = uf.new_zeros(batch, dim, A.shape[1])
    ys = []
    # per-position views via unbind: its backward is one stack, where indexing [..., t] would
    # build a full-size zero gradient per step (minutes at L = 4096 under autograd)
    dts, us, Bts, Cts = dt.unbind(-1), uf.unbind(-1), Bf.unbind(-1), Cf.unbind(-1)
    for t in range(L):
        d_t = dts[t].unsqueeze(-1)                            # (B, D, 1)
        decay = torch.exp(d_t * Af)                           # (B, D, N)
        drive = d_t * Bts[t] * us[t].unsqueeze(-1)
        state = decay * state + drive
        ys.append((state * Cts[t]).sum(-1))
    y = torch.stack(ys, dim=-1) if L > 0 else uf.new_zeros(batch, dim, 0)
    if D is not None:
        y = y + uf * D.to(cd)[:, None]
    if z is not None:
        y = y * F.silu(z.to(cd))
    out = y.to(dtype_in)
    if return_last_state:
        return out, state
    return out


def selective_scan_ref_grads(u, delta, A, B, C, D=None, z=None, delta_bias=None,
                             delta_softplus=False, dout=None,
                             compute_dtype=torch.float64):
    """Backward oracle: autograd of ``selective_scan_ref`` w.r.t. every input.

    Returns a dict of gradients (same names as the inputs) computed in
    ``compute_dtype`` for the given upstream gradient ``dout``.
    """
    leaves = {}

    def leaf(name, t):
        if t is None:
            return None
        x = t.detach().to(compute_dtype).requires_grad_(True)
        leaves[name] = x
        return x

    args = dict(u=leaf("u", u), delta=leaf("delta", delta), A=leaf("A", A),
                B=leaf("B", B), C=leaf("C", C), D=leaf("D", D), z=leaf("z", z),
                delta_bias=leaf("delta_bias", delta_bias))
    out = selective_scan_ref(**args, delta_softplus=delta_softplus,
                             compute_dtype=compute_dtype)
    out.backward(dout.to(compute_dtype))
    return {k: v.grad for k, v in leaves.items()}
