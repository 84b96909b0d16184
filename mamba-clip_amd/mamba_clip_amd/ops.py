"""Thin torch-facing wrappers of the contrastive kernels (include/mc_contrastive.h).

``gemm_nt(A, B, alpha)``  C = alpha * A @ B.T on the matrix cores (bf16, fp32 or fp8 e4m3fn in).
``quant_rows_fp8(X)``     row-wise amax-scaled e4m3fn quantisation (K padded to 16).
``similarity_fp8(I, T, scale)``  scale * I @ T.T through the fp8 MFMA path (config 5).
``clip_loss_fp8(I, T, scale)``   the symmetric CLIP loss on that fp8 path, logits never stored.
``scaled_logits_ce``      autograd op: logits = scale * X @ Y.T, then a weighted
                          sum of row- and/or column-softmax cross-entropies --
                          the dense part of ClipLoss (loss.py:89-147) -- fused:
                          the logits never exist in memory (mc_ce_fused_*).
``ce_stats`` / ``ce_grad`` the unfused statistics / gradient kernels over a
                          materialised S (kept for logits the caller needs anyway).
All launches go on the current HIP stream; nothing synchronises.
"""
import ctypes
import os
import weakref

import torch

from . import _lib


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


def gemm_nt(A, B, alpha=1.0, alpha_dev=None, out_dtype=torch.float32, scale_a=None, scale_b=None, out=None):
    """C[m, n] = alpha * scale_a[m] * scale_b[n] * sum_k A[m, k] * B[n, k]  (A, B row-major, K contiguous).

    scale_a / scale_b (fp32 per-row factors, optional) are the dequantisation
    factors of fp8 operands from ``quant_rows_fp8``.
    """
    lib = _lib.load()
    if A.dtype != B.dtype or A.dtype not in (torch.bfloat16, torch.float32, torch.float8_e4m3fn):
        raise RuntimeError("gemm_nt: A and B must both be bf16, both fp32 or both float8_e4m3fn")
    if A.stride(-1) != 1:
        A = A.contiguous()
    if B.stride(-1) != 1:
        B = B.contiguous()
    M, K = A.shape
    N, K2 = B.shape
    if K != K2:
        raise RuntimeError("gemm_nt: inner dimensions differ")
    if out is None:
        C = torch.empty(M, N, device=A.device, dtype=out_dtype)
    else:
        if out.shape != (M, N) or out.dtype != out_dtype or out.stride(-1) != 1:
            raise RuntimeError("gemm_nt: out must be (M, N) of out_dtype with unit column stride")
        C = out
    p = _lib.GemmNTParams()
    p.M, p.N, p.K = M, N, K
    p.in_dtype, p.out_dtype = _lib.dtype_code(A.dtype), _lib.dtype_code(out_dtype)
    p.A, p.lda, p.B, p.ldb, p.C, p.ldc = A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0)
    p.alpha = float(alpha)
    p.alpha_dev = alpha_dev.data_ptr() if alpha_dev is not None else None
    for name, sc, n in (("row_scale_a", scale_a, M), ("row_scale_b", scale_b, N)):
        if sc is not None:
            if sc.dtype != torch.float32 or sc.numel() != n or not sc.is_contiguous():
                raise RuntimeError(f"gemm_nt: {name} must be a contiguous fp32 vector of {n} entries")
            setattr(p, name, sc.data_ptr())
    if GEMM_NT_RECORD is not None:
        GEMM_NT_RECORD.append(int(lib.mc_gemm_nt_kernel(p)))
    _lib.check(lib.mc_gemm_nt(p, _lib.stream_handle(A.device)), "mc_gemm_nt")
    return C


# Tests set GEMM_NT_RECORD = [] to see which kernel each gemm_nt call ran (_lib.MC_GEMM_KERNEL_*).
GEMM_NT_RECORD = None


def quant_rows_fp8(X):
    """(Q, inv_scale): Q (rows, round_up(cols, 16)) float8_e4m3fn, zero-padded; X[i] ~= Q[i] * inv_scale[i].

    Row scale s_i = 448 / max_j |X[i, j]| (include/mc_contrastive.h, mc_quant_rows_fp8).
    """
    lib = _lib.load()
    if not X.is_cuda:
        raise RuntimeError("quant_rows_fp8: X must be a HIP (cuda) tensor")
    if X.dim() != 2:
        raise RuntimeError("quant_rows_fp8: X must be 2-D")
    if X.stride(-1) != 1:
        X = X.contiguous()
    rows, cols = X.shape
    ldq = (cols + 15) // 16 * 16
    Q = torch.empty(rows, ldq, device=X.device, dtype=torch.float8_e4m3fn)
    inv = torch.empty(rows, device=X.device, dtype=torch.float32)
    _lib.check(lib.mc_quant_rows_fp8(rows, cols, _lib.dtype_code(X.dtype), X.data_ptr(), X.stride(0) if rows else cols,
                                     Q.data_ptr(), ldq, inv.data_ptr(), _lib.stream_handle(X.device)),
               "mc_quant_rows_fp8")
    return Q, inv


def similarity_fp8(image_features, text_features, logit_scale, out_dtype=torch.float32):
    """logit_scale * I @ T.T with both operands quantised row-wise to e4m3fn (fp32 accumulate).

    The similarity matmul of ClipModel.get_logits (model.py:1104-1112) on
    frozen features, fp8 MFMA (BASELINE config 5).  ``logit_scale`` is the
    already-exponentiated scale (a 0-d device tensor or a float).  fp32 or bf16
    logits, both on the library's own kernels (mc_gemm_nt: the register-panel fp8
    kernel for K <= 512); no vendor GEMM.
    """
    qi, si = quant_rows_fp8(image_features)
    qt, st = quant_rows_fp8(text_features)
    if torch.is_tensor(logit_scale):
        return gemm_nt(qi, qt, alpha_dev=logit_scale.reshape(()).float().contiguous(), out_dtype=out_dtype,
                       scale_a=si, scale_b=st)
    return gemm_nt(qi, qt, alpha=float(logit_scale), out_dtype=out_dtype, scale_a=si, scale_b=st)


def clip_loss_fp8(image_features, text_features, logit_scale):
    """Symmetric CLIP loss (loss.py:124-147, single process) on fp8 e4m3fn operands, without logits
    in memory: row-quantised features -> mc_ce_fused_fwd on the fp8 MFMA path (config 5 features,
    evaluation / frozen-feature scoring; no backward)."""
    qi, si = quant_rows_fp8(image_features)
    qt, st = quant_rows_fp8(text_features)
    n = qi.shape[0]
    sc = (logit_scale.reshape(()).float() if torch.is_tensor(logit_scale)
          else torch.tensor(float(logit_scale), device=qi.device)).contiguous()
    loss, _, _ = ce_fused_fwd(qi, qt, sc, 0, 0.5 / n, 0, 0.5 / n, sx=si, sy=st)
    return loss


def ce_stats(S, axis, label_offset, coef):
    """(lse, weighted NLL sum as a device scalar) along rows (axis 0) or columns (1)."""
    lib = _lib.load()
    rows, cols = S.shape
    n = rows if axis == 0 else cols
    lse = torch.empty(n, device=S.device, dtype=torch.float32)
    loss = torch.empty((), device=S.device, dtype=torch.float32)
    ws_b = lib.mc_ce_stats_workspace_bytes(rows, cols, axis)
    ws = _ws(ws_b, S.device)
    _lib.check(lib.mc_ce_stats(rows, cols, S.data_ptr(), S.stride(0), axis, int(label_offset), lse.data_ptr(),
                               None, float(coef), loss.data_ptr(), ws.data_ptr(), ws_b,
                               _lib.stream_handle(S.device)), "mc_ce_stats")
    return lse, loss


def ce_grad(S, lse_r, off_r, coef_r, lse_c, off_c, coef_c, gout, out_dtype, scale):
    """G = gout * d(loss)/dS (fp32 or bf16) and d(loss)/d(scale) (device scalar)."""
    lib = _lib.load()
    rows, cols = S.shape
    G = torch.empty(rows, cols, device=S.device, dtype=out_dtype)
    dscale = torch.empty((), device=S.device, dtype=torch.float32)
    ws_b = lib.mc_ce_grad_workspace_bytes(rows, cols)
    ws = _ws(ws_b, S.device)
    gout = gout.reshape(()).float().contiguous()
    _lib.check(lib.mc_ce_grad(rows, cols, S.data_ptr(), S.stride(0), lse_r.data_ptr(), int(off_r), float(coef_r),
                              lse_c.data_ptr() if lse_c is not None else None, int(off_c), float(coef_c),
                              gout.data_ptr(), _lib.dtype_code(out_dtype), G.data_ptr(), cols, scale.data_ptr(),
                              dscale.data_ptr(), ws.data_ptr(), ws_b, _lib.stream_handle(S.device)), "mc_ce_grad")
    return G, dscale


# G blocks of the fused backward hold at most this many elements (32 MiB bf16):
# the backward never materialises the full M x N matrix once M * N exceeds it.
CE_GRAD_BLOCK_ELEMS = 1 << 24


def _ce_params(X, Y, sc, row_off, coef_r, col_off, coef_c, sx=None, sy=None):
    p = _lib.CEFusedParams()
    p.M, p.K = X.shape
    p.N = Y.shape[0]
    p.in_dtype = _lib.dtype_code(X.dtype)
    p.X, p.ldx, p.Y, p.ldy = X.data_ptr(), X.stride(0), Y.data_ptr(), Y.stride(0)
    p.row_scale_x, p.row_scale_y = _lib.ptr(sx), _lib.ptr(sy)
    p.scale_dev = sc.data_ptr()
    p.row_off, p.coef_r, p.col_off, p.coef_c = int(row_off), float(coef_r), int(col_off), float(coef_c)
    return p


def ce_fused_fwd(X, Y, sc, row_off=0, coef_r=1.0, col_off=0, coef_c=0.0, sx=None, sy=None):
    """(loss, lse_r, lse_c) of  coef_r * sum_i CE_row_i + coef_c * sum_j CE_col_j,  S = sc * X @ Y^T,
    computed tile-wise on the matrix cores without storing S (mc_ce_fused_fwd).

    X, Y: row-major (K contiguous) bf16 / fp32, or fp8 e4m3fn with per-row
    dequantisation factors sx / sy (``quant_rows_fp8``).  sc: 0-d fp32 device
    tensor.  lse_c is None when coef_c == 0 (no column term)."""
    lib = _lib.load()
    M, N = X.shape[0], Y.shape[0]
    cols = coef_c != 0.0
    lse_r = torch.empty(M, device=X.device, dtype=torch.float32)
    lse_c = torch.empty(N, device=X.device, dtype=torch.float32) if cols else None
    loss = torch.empty((), device=X.device, dtype=torch.float32)
    p = _ce_params(X, Y, sc, row_off, coef_r, col_off, coef_c, sx, sy)
    ws_b = lib.mc_ce_fused_fwd_workspace_bytes(M, N, int(cols))
    ws = _ws(ws_b, X.device)
    p.lse_r, p.lse_c, p.loss_out = lse_r.data_ptr(), _lib.ptr(lse_c), loss.data_ptr()
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws_b
    _lib.check(lib.mc_ce_fused_fwd(p, _lib.stream_handle(X.device)), "mc_ce_fused_fwd")
    return loss, lse_r, lse_c


def ce_fused_grad(X, Y, sc, lse_r, lse_c, row_off, coef_r, col_off, coef_c, gout, g_dtype, want_dscale=False):
    """(sc * G, dscale): one block of dloss/dS recomputed from (lse_r, lse_c), S = sc * X @ Y^T
    (mc_ce_fused_grad); ``G @ Y`` is then dX directly.  dscale is sum(G S) / sc or None."""
    lib = _lib.load()
    M, N = X.shape[0], Y.shape[0]
    G = torch.empty(M, N, device=X.device, dtype=g_dtype)
    p = _ce_params(X, Y, sc, row_off, coef_r, col_off, coef_c)
    p.lse_r, p.lse_c = _lib.ptr(lse_r), _lib.ptr(lse_c)
    p.gout_dev = gout.data_ptr()
    p.g_dtype, p.g_times_scale, p.G, p.ldg = _lib.dtype_code(g_dtype), 1, G.data_ptr(), N
    dscale = None
    ws = None
    if want_dscale:
        dscale = torch.empty((), device=X.device, dtype=torch.float32)
        ws_b = lib.mc_ce_fused_grad_workspace_bytes(M, N)
        ws = _ws(ws_b, X.device)
        p.dscale_out, p.workspace, p.workspace_bytes = dscale.data_ptr(), ws.data_ptr(), ws_b
    _lib.check(lib.mc_ce_fused_grad(p, _lib.stream_handle(X.device)), "mc_ce_fused_grad")
    return G, dscale


def _mm_nt(a, b_t, out):
    """out = a @ b_t^T.  fp32 operands run the library's exact-fp32 MFMA GEMM (mc_gemm_nt, b_t
    K-contiguous): a library fp32 GEMM follows the process-wide allow_tf32 flag, which init_device
    turns on like the reference (utils/dist_utils.py:41-43) -- flipping that flag here would race
    with other threads.  bf16 operands run the library GEMM (no reduced-precision variant)."""
    if a.dtype == torch.float32:
        return gemm_nt(a, b_t, out=out)
    return torch.mm(a, b_t.t(), out=out)


def _block_rows(other):
    return max(128, CE_GRAD_BLOCK_ELEMS // max(other, 1) // 128 * 128)


class ScaledLogitsCE(torch.autograd.Function):
    """loss = coef_r * sum_i CE_row_i(S) + coef_c * sum_j CE_col_j(S),  S = scale * X @ Y^T.

    Row i's label is column i + row_off; column j's label is row j + col_off.
    coef_c == 0 drops the column term (local-loss halves).  X and Y are the
    (gathered) feature matrices; bf16 inputs run the bf16 MFMA path, fp32
    inputs the exact-fp32 MFMA path; logits and statistics are fp32.

    Neither pass stores S.  Forward: mc_ce_fused_fwd (logit tiles reduced to
    LSE partials in registers).  Backward: dX in row blocks -- G_blk (recomputed
    by mc_ce_fused_grad, already times scale) @ Y -- and dY in column blocks
    from the transposed problem (roles of X/Y, rows/columns, offsets and
    coefficients swapped) -- G^T_blk @ X; both products are plain NN GEMMs
    (hipBLASLt), so no operand is ever transposed in memory.  Blocks hold at
    most CE_GRAD_BLOCK_ELEMS elements.
    """

    @staticmethod
    def forward(ctx, X, Y, scale, row_off, coef_r, col_off, coef_c):
        dt = X.dtype if X.dtype in (torch.bfloat16, torch.float32) else torch.float32
        Xc = X.to(dt).contiguous()
        Yc = Y.to(dt).contiguous()
        sc = scale.reshape(()).float().contiguous()
        loss, lse_r, lse_c = ce_fused_fwd(Xc, Yc, sc, row_off, coef_r, col_off, coef_c)
        ctx.save_for_backward(Xc, Yc, sc, lse_r, lse_c if lse_c is not None else lse_r)
        ctx.cfg = (row_off, coef_r, col_off, coef_c, lse_c is not None, X.dtype, Y.dtype, scale.dtype, scale.shape)
        return loss

    @staticmethod
    def backward(ctx, gout):
        Xc, Yc, sc, lse_r, lse_c = ctx.saved_tensors
        row_off, coef_r, col_off, coef_c, has_c, xdt, ydt, sdt, sshape = ctx.cfg
        lse_c = lse_c if has_c else None
        gout = gout.reshape(()).float().contiguous()
        gdt = Xc.dtype  # G feeds the GEMMs in the operands' dtype
        M, N = Xc.shape[0], Yc.shape[0]
        want_ds = ctx.needs_input_grad[2]
        dX = dY = dscale = None
        # second operands of dX = G @ Y and dY = G^T @ X as (K-contiguous) row-major transposes
        Yt = Yc.t().contiguous() if Yc.dtype == torch.float32 else Yc.t()
        Xt = Xc.t().contiguous() if Xc.dtype == torch.float32 else Xc.t()
        if ctx.needs_input_grad[0] or want_ds:
            dX = torch.empty_like(Xc) if ctx.needs_input_grad[0] else None
            R = _block_rows(N)
            parts = []
            for r0 in range(0, M, R):
                r1 = min(M, r0 + R)
                G, ds = ce_fused_grad(Xc[r0:r1], Yc, sc, lse_r[r0:r1], lse_c, row_off + r0, coef_r, col_off - r0,
                                      coef_c, gout, gdt, want_ds)
                if dX is not None:
                    _mm_nt(G, Yt, dX[r0:r1])
                if ds is not None:
                    parts.append(ds)
            if want_ds:
                dscale = parts[0] if len(parts) == 1 else torch.stack(parts).sum()
            dX = dX.to(xdt) if dX is not None else None
        if ctx.needs_input_grad[1]:
            dY = torch.empty_like(Yc)
            R = _block_rows(M)
            for c0 in range(0, N, R):
                c1 = min(N, c0 + R)
                # transposed problem: rows = columns c0..c1 of S, columns = rows of S
                GT, _ = ce_fused_grad(Yc[c0:c1], Xc, sc, lse_c[c0:c1] if has_c else None, lse_r, col_off + c0,
                                      coef_c, row_off - c0, coef_r, gout, gdt)
                _mm_nt(GT, Xt, dY[c0:c1])
            dY = dY.to(ydt)
        dS = dscale.to(sdt).reshape(sshape) if want_ds else None
        return dX, dY, dS, None, None, None, None


def scaled_logits_ce(X, Y, scale, row_off=0, coef_r=1.0, col_off=0, coef_c=0.0):
    return ScaledLogitsCE.apply(X, Y, scale, row_off, coef_r, col_off, coef_c)


# ---------------------------------------------------------------------------- encoder ops (include/mc_ops.h)
class AddRMSNormFn(torch.autograd.Function):
    """(y, h) = (rmsnorm(x + res) * w, x + res); h is the fp32 residual stream."""

    @staticmethod
    def forward(ctx, x, res, weight, eps):
        lib = _lib.load()
        x = x.contiguous()
        rows = x.numel() // x.shape[-1]
        cols = x.shape[-1]
        y = torch.empty_like(x)
        h = torch.empty(x.shape, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        w = weight.float().contiguous()
        r = res.float().contiguous() if res is not None else None
        _lib.check(lib.mc_add_rmsnorm_fwd(rows, cols, _lib.dtype_code(x.dtype), x.data_ptr(), _lib.ptr(r),
                                          w.data_ptr(), float(eps), y.data_ptr(), h.data_ptr(), rstd.data_ptr(),
                                          _lib.stream_handle(x.device)), "mc_add_rmsnorm_fwd")
        ctx.save_for_backward(h, w, rstd)
        ctx.meta = (x.dtype, res is not None, weight.dtype)
        return y, h

    @staticmethod
    def backward(ctx, dy, dh_out):
        lib = _lib.load()
        h, w, rstd = ctx.saved_tensors
        xdt, has_res, wdt = ctx.meta
        cols = h.shape[-1]
        rows = h.numel() // cols
        dy = (dy if dy is not None else torch.zeros(h.shape, device=h.device, dtype=xdt)).to(xdt).contiguous()
        dres = dh_out.float().contiguous() if dh_out is not None else None
        dx = torch.empty(h.shape, device=h.device, dtype=xdt)
        dres_in = torch.empty_like(h) if has_res else None
        dw = torch.empty(cols, device=h.device, dtype=torch.float32)
        ws_b = lib.mc_add_rmsnorm_bwd_workspace_bytes(rows, cols)
        ws = _ws(ws_b, h.device)
        _lib.check(lib.mc_add_rmsnorm_bwd(rows, cols, _lib.dtype_code(xdt), dy.data_ptr(), _lib.ptr(dres),
                                          h.data_ptr(), w.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                                          _lib.ptr(dres_in), dw.data_ptr(), ws.data_ptr(), ws_b,
                                          _lib.stream_handle(h.device)), "mc_add_rmsnorm_bwd")
        return dx, dres_in, dw.to(wdt), None


def add_rmsnorm(x, residual, weight, eps=1e-5):
    return AddRMSNormFn.apply(x, residual, weight, eps)


class AddLayerNormFn(torch.autograd.Function):
    """(y, h) = (LayerNorm(x + res) * w + b, x + res); h in the activation dtype (pre-LN residual stream)."""

    @staticmethod
    def forward(ctx, x, res, weight, bias, eps):
        lib = _lib.load()
        x = x.contiguous()
        res = res.to(x.dtype).contiguous()
        cols = x.shape[-1]
        rows = x.numel() // cols
        y = torch.empty_like(x)
        h = torch.empty_like(x)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        w = weight.float().contiguous()
        b = bias.float().contiguous() if bias is not None else None
        _lib.check(lib.mc_add_layernorm_fwd(rows, cols, _lib.dtype_code(x.dtype), x.data_ptr(), res.data_ptr(),
                                            w.data_ptr(), _lib.ptr(b), float(eps), y.data_ptr(), h.data_ptr(),
                                            mean.data_ptr(), rstd.data_ptr(), _lib.stream_handle(x.device)),
                   "mc_add_layernorm_fwd")
        ctx.save_for_backward(h, w, mean, rstd)
        ctx.meta = (weight.dtype, bias.dtype if bias is not None else None)
        return y, h

    @staticmethod
    def backward(ctx, dy, dh):
        h, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = _layernorm_bwd(h, w, mean, rstd, dy, dh, ctx.meta[1] is not None, want_colsum=True)
        wdt, bdt = ctx.meta
        return dx, dx, dw.to(wdt), (db.to(bdt) if db is not None else None), None


class LayerNormFn(torch.autograd.Function):
    """y = LayerNorm(x) * w + b with the activation dtype in and out (fp32 statistics)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        lib = _lib.load()
        x = x.contiguous()
        cols = x.shape[-1]
        rows = x.numel() // cols
        y = torch.empty_like(x)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        w = weight.float().contiguous()
        b = bias.float().contiguous() if bias is not None else None
        _lib.check(lib.mc_add_layernorm_fwd(rows, cols, _lib.dtype_code(x.dtype), x.data_ptr(), None, w.data_ptr(),
                                            _lib.ptr(b), float(eps), y.data_ptr(), None, mean.data_ptr(),
                                            rstd.data_ptr(), _lib.stream_handle(x.device)), "mc_add_layernorm_fwd")
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.meta = (weight.dtype, bias.dtype if bias is not None else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = _layernorm_bwd(x, w, mean, rstd, dy, None, ctx.meta[1] is not None, want_colsum=True)
        wdt, bdt = ctx.meta
        return dx, dw.to(wdt), (db.to(bdt) if db is not None else None), None


COLSUM_ATTR = "_mc_colsum"   # fp32 column sums riding on a gradient tensor (LinearSK picks them up)


def _layernorm_bwd(h, w, mean, rstd, dy, dh, has_bias, want_colsum=False):
    lib = _lib.load()
    cols = h.shape[-1]
    rows = h.numel() // cols
    dy = (dy if dy is not None else torch.zeros_like(h)).to(h.dtype).contiguous()
    dh = dh.to(h.dtype).contiguous() if dh is not None else None
    dx = torch.empty_like(h)
    dw = torch.empty(cols, device=h.device, dtype=torch.float32)
    db = torch.empty(cols, device=h.device, dtype=torch.float32) if has_bias else None
    csum = torch.empty(cols, device=h.device, dtype=torch.float32) if want_colsum else None
    ws_b = lib.mc_add_layernorm_bwd_workspace_bytes(rows, cols)
    ws = _ws(ws_b, h.device)
    _lib.check(lib.mc_add_layernorm_bwd(rows, cols, _lib.dtype_code(h.dtype), dy.data_ptr(), _lib.ptr(dh),
                                        h.data_ptr(), w.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                                        dw.data_ptr(), _lib.ptr(db), _lib.ptr(csum), ws.data_ptr(), ws_b,
                                        _lib.stream_handle(h.device)), "mc_add_layernorm_bwd")
    if csum is not None:
        # the bias gradient of the linear layer whose output entered this norm (fc2 / attention
        # proj): LinearSK.backward uses it instead of re-reading dx for the column sum
        # (with dx's version counter: an in-place accumulation into dx invalidates the sums)
        setattr(dx, COLSUM_ATTR, (csum, dx._version))
    return dx, dw, db


def add_layernorm(x, residual, weight, bias, eps=1e-6):
    """Pre-LN block entry: returns (LN(x + residual), x + residual); residual None -> (LN(x), x)."""
    if residual is None:
        return LayerNormFn.apply(x, weight, bias, eps), x
    return AddLayerNormFn.apply(x, residual, weight, bias, eps)


class GradSlab:
    """One gradient buffer shared by the backward passes of ops that read row blocks of the
    same channel-major activation.  The Mamba mixer splits in_proj's (2*d_inner, B*L) output
    into x (-> conv1d) and z (-> the scan's gate); the scan backward writes dz and the conv
    backward writes dx straight into their halves of one (2*d_inner, B*L) buffer, so the
    split's backward is the buffer itself instead of a concatenating copy."""

    def __init__(self, rows, cols, dtype, device):
        self.rows, self.cols, self.dtype, self.device = rows, cols, dtype, device
        self.buf = None

    def get(self):
        if self.buf is None:
            self.buf = torch.empty(self.rows, self.cols, dtype=self.dtype, device=self.device)
        return self.buf

    def block(self, r0, r1, batch):
        """rows [r0, r1) as the (batch, r1 - r0, L) channel-major view the kernels take."""
        return self.get()[r0:r1].view(r1 - r0, batch, self.cols // batch).transpose(0, 1)


class SplitRowsFn(torch.autograd.Function):
    """(X[:k], X[k:]) of a 2-D activation; backward returns the slab when both gradients
    already live in it (written there by the consumers' backward kernels), else concatenates."""

    @staticmethod
    def forward(ctx, X, k, slab):
        ctx.k, ctx.slab, ctx.shape = k, slab, X.shape
        return X[:k], X[k:]

    @staticmethod
    def backward(ctx, ga, gb):
        k, slab = ctx.k, ctx.slab
        buf = slab.buf if slab is not None else None
        if (buf is not None and ga is not None and gb is not None and ga.data_ptr() == buf.data_ptr()
                and gb.data_ptr() == buf[k:].data_ptr() and ga.stride() == buf.stride() == gb.stride()):
            slab.shared = True   # (observable by tests: the no-copy path was taken)
            return buf, None, None
        rows, cols = ctx.shape
        ref = ga if ga is not None else gb
        ga = ga if ga is not None else torch.zeros(k, cols, dtype=ref.dtype, device=ref.device)
        gb = gb if gb is not None else torch.zeros(rows - k, cols, dtype=ref.dtype, device=ref.device)
        return torch.cat([ga, gb]), None, None


def split_rows(X, k, slab=None):
    return SplitRowsFn.apply(X, k, slab)


class SplitRowsNFn(torch.autograd.Function):
    """Row blocks of `sizes` of a 2-D activation (the mixer's x_proj output: dt_raw, B, C rows);
    backward returns the slab when every block's gradient already lives in it, else concatenates."""

    @staticmethod
    def forward(ctx, X, sizes, slab):
        ctx.sizes, ctx.slab, ctx.shape = sizes, slab, X.shape
        return X.split(list(sizes), dim=0)

    @staticmethod
    def backward(ctx, *grads):
        slab, sizes = ctx.slab, ctx.sizes
        buf = slab.buf if slab is not None else None
        if buf is not None and all(g is not None for g in grads):
            r0, ok = 0, True
            for g, n in zip(grads, sizes):
                blk = buf[r0:r0 + n]
                ok = ok and g.data_ptr() == blk.data_ptr() and g.shape == blk.shape and g.stride() == blk.stride()
                r0 += n
            if ok:
                slab.shared = True
                return buf, None, None
        cols = ctx.shape[1]
        ref = next(g for g in grads if g is not None)
        parts = [g.reshape(n, cols) if g is not None else torch.zeros(n, cols, dtype=ref.dtype, device=ref.device)
                 for g, n in zip(grads, sizes)]
        return torch.cat(parts), None, None


def split_rows_n(X, sizes, slab=None):
    return SplitRowsNFn.apply(X, tuple(sizes), slab)


class CausalConv1dFn(torch.autograd.Function):
    """Depthwise causal conv1d (+SiLU) over (batch, dim, seqlen); output contiguous."""

    @staticmethod
    def forward(ctx, x, weight, bias, silu, dx_slab=None):
        lib = _lib.load()
        if x.stride(-1) != 1:
            x = x.contiguous()
        Bsz, D, L = x.shape
        K = weight.shape[-1]
        w = weight.reshape(D, K).float().contiguous()
        b = bias.float().contiguous() if bias is not None else None
        y = torch.empty_like(x)          # keeps a dense channel-major layout of x
        _lib.check(lib.mc_causal_conv1d_fwd(Bsz, D, L, K, _lib.dtype_code(x.dtype), x.data_ptr(), x.stride(0),
                                            x.stride(1), w.data_ptr(), _lib.ptr(b), int(silu), y.data_ptr(),
                                            y.stride(0), y.stride(1), _lib.stream_handle(x.device)),
                   "mc_causal_conv1d_fwd")
        ctx.save_for_backward(x, w, b if b is not None else w)
        ctx.meta = (silu, bias is not None, weight.shape, weight.dtype)
        ctx.dx_slab = dx_slab
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib.load()
        x, w, b = ctx.saved_tensors
        silu, has_b, wshape, wdt = ctx.meta
        Bsz, D, L = x.shape
        K = w.shape[-1]
        dy = dy.to(x.dtype)
        if dy.stride(-1) != 1:
            dy = dy.contiguous()
        # dx into rows [0, D) of the shared slab (x was rows [0, D) of the in_proj output)
        dx = ctx.dx_slab.block(0, D, Bsz) if ctx.dx_slab is not None else torch.empty_like(x)
        dw = torch.empty(D, K, device=x.device, dtype=torch.float32)
        db = torch.empty(D, device=x.device, dtype=torch.float32) if has_b else None
        ws_b = lib.mc_causal_conv1d_bwd_workspace_bytes(Bsz, D, L, K)
        ws = _ws(ws_b, x.device)
        _lib.check(lib.mc_causal_conv1d_bwd(Bsz, D, L, K, _lib.dtype_code(x.dtype), x.data_ptr(), x.stride(0),
                                            x.stride(1), w.data_ptr(), b.data_ptr() if has_b else None, int(silu),
                                            dy.data_ptr(), dy.stride(0), dy.stride(1), dx.data_ptr(), dx.stride(0),
                                            dx.stride(1), dw.data_ptr(), _lib.ptr(db), ws.data_ptr(),
                                            ws_b, _lib.stream_handle(x.device)), "mc_causal_conv1d_bwd")
        return dx, dw.reshape(wshape).to(wdt), (db.to(wdt) if db is not None else None), None, None


def causal_conv1d(x, weight, bias=None, silu=True, dx_slab=None):
    return CausalConv1dFn.apply(x, weight, bias, silu, dx_slab)


# open_clip's OPENAI_DATASET_MEAN / _STD: the reference's default Normalize (data.py:47-53)
IMAGE_MEAN = (0.48145466, 0.4578275, 0.40821073)
IMAGE_STD = (0.26862954, 0.26130258, 0.27577711)
_NORM_CACHE = {}


def _norm_affine(device, C, mean, std):
    """scale = 1 / (255 std), shift = -mean / std per channel (ToTensor + Normalize on raw bytes)."""
    key = (device, C, tuple(mean), tuple(std))
    if key not in _NORM_CACHE:
        m = torch.tensor(mean, dtype=torch.float64)[:C]
        sd = torch.tensor(std, dtype=torch.float64)[:C]
        _NORM_CACHE[key] = ((1.0 / (255.0 * sd)).float().to(device), (-m / sd).float().to(device))
    return _NORM_CACHE[key]


class PatchIm2colFn(torch.autograd.Function):
    """Non-overlapping (k = s = P) patch rows in `out_dtype`, the input cast fused in (float NCHW), or
    the whole image input path for raw uint8 NHWC images (ToTensor + Normalize + patchify,
    mc_patch_embed_input).  For a float image the map is a permutation, so the backward is the inverse
    permutation (one strided copy): VSSM's input gradient (model.py:189-201) flows through it."""

    @staticmethod
    def forward(ctx, img, patch, out_dtype, mean, std):
        lib = _lib.load()
        u8 = img.dtype == torch.uint8
        img = img.contiguous()
        if u8:
            Bsz, H, W, C = img.shape
        else:
            Bsz, C, H, W = img.shape
        out_dtype = out_dtype or (torch.float32 if u8 else img.dtype)
        out = torch.empty(Bsz * (H // patch) * (W // patch), C * patch * patch, device=img.device, dtype=out_dtype)
        if patch % 4 == 0:
            p = _lib.PatchInputParams()
            p.batch, p.channels, p.height, p.width, p.patch = Bsz, C, H, W, patch
            p.layout = _lib.MC_LAYOUT_NHWC if u8 else _lib.MC_LAYOUT_NCHW
            p.in_dtype, p.out_dtype = _lib.dtype_code(img.dtype), _lib.dtype_code(out_dtype)
            if u8:
                sc, sh = _norm_affine(img.device, C, mean or IMAGE_MEAN, std or IMAGE_STD)
                p.scale, p.shift = sc.data_ptr(), sh.data_ptr()
            p.img, p.out = img.data_ptr(), out.data_ptr()
            _lib.check(lib.mc_patch_embed_input(ctypes.byref(p), _lib.stream_handle(img.device)), "mc_patch_embed_input")
        else:   # VSSM's P = 4 goes here too; other P (not a multiple of 4): element-wise kernel, same dtype
            if u8:
                raise RuntimeError("patch_im2col: uint8 images need a patch size that is a multiple of 4")
            src = img if img.dtype == out_dtype else img.to(out_dtype)
            _lib.check(lib.mc_patch_im2col(Bsz, C, H, W, patch, _lib.dtype_code(out_dtype), src.data_ptr(),
                                           out.data_ptr(), _lib.stream_handle(img.device)), "mc_patch_im2col")
        ctx.meta = (Bsz, C, H, W, patch, img.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        Bsz, C, H, W, P, in_dt = ctx.meta
        if in_dt == torch.uint8:
            return None, None, None, None, None
        gi = g.reshape(Bsz, H // P, W // P, C, P, P).permute(0, 3, 1, 4, 2, 5).reshape(Bsz, C, H, W)
        return gi.to(in_dt), None, None, None, None


def patch_im2col(img, patch, out_dtype=None, mean=None, std=None):
    """(B, C, H, W) float -> (B * H/P * W/P, C * P * P) patch rows (row = (b, h/P, w/P), col = (c, ph, pw)),
    cast to out_dtype on the way; or (B, H, W, C) uint8 raw images -> the same rows normalised with
    mean / std (default open_clip's OPENAI_DATASET_MEAN / _STD, the reference's transform)."""
    return PatchIm2colFn.apply(img, patch, out_dtype, mean, std)


# ---------------------------------------------------------------------------- projections with split-K weight grads
# The towers' weight gradients are GEMMs with a short output (N x K <= 3072 x
# 3072) and a very long reduction (M = batch * tokens = 50432 at C2): one
# library GEMM tiles the output into too few workgroups for 256 CUs (measured
# on MI355X, tools/gemm_wgrad_ab.py: 231-610 TF/s).  Splitting M into s slabs
# and summing the fp32 partials (one strided-batched GEMM + one reduction)
# runs 1.3-1.8x faster and keeps the sum in fp32.
def _split_factor(M, N, K):
    """Slabs for the token-dim split, from a sweep of the C2 shapes (tools/wgrad_sweep.py,
    profiles/r03/wgrad_split_sweep.txt): large outputs 4; small outputs (dt_proj, x_proj) and the
    ViT's long-M medium outputs (qkv, proj, patch embed) 16; Mamba out_proj (M = 20480) 8."""
    if N * K >= 2_000_000:
        s = 4
    elif N * K < 250_000 or M >= 40_000:
        s = 16
    else:
        s = 8
    while s > 1 and M % s:
        s //= 2
    return s


def _wgrad_layout(t, rows_are_tokens):
    """(layout, leading dim) of a 2-D operand for mc_gemm_wgrad, or None when neither dim is unit-stride.
    rows_are_tokens: t is (T, features) (X); else (features, T) (G)."""
    st_tok, st_feat = (t.stride(0), t.stride(1)) if rows_are_tokens else (t.stride(1), t.stride(0))
    if st_feat == 1 and t.shape[1 if rows_are_tokens else 0] > 0:
        return _lib.MC_WGRAD_TOKEN_MAJOR, st_tok
    if st_tok == 1:
        return _lib.MC_WGRAD_FEATURE_MAJOR, st_feat
    return None


def wgrad_hip(G, X, splits=0):
    """G @ X in fp32 on the hand-written long-reduction GEMM (csrc/gemm_wgrad.hip, mc_gemm_wgrad):
    G (N, T) and X (T, K), 16-bit, each with one unit-stride dim; returns None when the shape or
    layout is outside the kernel's (T % 64, 16-B aligned rows), so the caller takes the library path."""
    if not (G.is_cuda and G.dtype == X.dtype and G.dtype in (torch.bfloat16, torch.float16)):
        return None
    N, T = G.shape
    K = X.shape[1]
    la, lb = _wgrad_layout(G, False), _wgrad_layout(X, True)
    if la is None or lb is None or T % 64 or T == 0 or G.data_ptr() % 16 or X.data_ptr() % 16:
        return None
    if la[1] % 8 or lb[1] % 8 or (la[0] == _lib.MC_WGRAD_TOKEN_MAJOR and N % 8) or \
            (lb[0] == _lib.MC_WGRAD_TOKEN_MAJOR and K % 8):
        return None
    out = torch.empty(N, K, device=G.device, dtype=torch.float32)
    p = _lib.WgradParams()
    p.M, p.N, p.T, p.dtype = N, K, T, _lib.dtype_code(G.dtype)
    p.a_layout, p.lda, p.b_layout, p.ldb = la[0], la[1], lb[0], lb[1]
    p.A, p.B, p.C, p.ldc, p.splits = G.data_ptr(), X.data_ptr(), out.data_ptr(), K, int(splits)
    lib = _lib.load()
    ws_b = lib.mc_gemm_wgrad_workspace_bytes(ctypes.byref(p))
    ws = _ws(ws_b, G.device) if ws_b else None
    if ws is not None:
        p.workspace, p.workspace_bytes = ws.data_ptr(), ws_b
    _lib.check(lib.mc_gemm_wgrad(ctypes.byref(p), _lib.stream_handle(G.device)), "mc_gemm_wgrad")
    return out


# The towers' long-K weight gradients on mc_gemm_wgrad (csrc/gemm_wgrad.hip, on by default since round 5:
# 1.0-1.1 PFLOP/s vs the library split-K slabs' 0.75-0.91 at the ViT / Mamba shapes, same-box step
# C2 69.96 -> 68.5 ms, C3 25.4 -> 25.0 ms, profiles/r05/wgrad/); 0 = the library slabs (A/B)
WGRAD_HIP = os.environ.get("MAMBA_CLIP_AMD_WGRAD_HIP", "1") != "0"


def wgrad(G, X):
    """G @ X in fp32 for G (N, M), X (M, K), any strides, M the long reduction dim."""
    N, M = G.shape
    K = X.shape[1]
    if WGRAD_HIP and G.is_cuda and M >= 8192 and min(N, K) >= 256:
        # (the skinny x_proj / dt_proj outputs, 80 and 48 wide, stay on the library: 25 vs 47 us at C2)
        out = wgrad_hip(G, X)
        if out is not None:
            return out
    s = _split_factor(M, N, K) if (G.is_cuda and M >= 8192) else 1
    if s == 1:
        return torch.mm(G, X).float()
    Gs = G.unflatten(1, (s, M // s)).transpose(0, 1)        # (s, N, M/s)
    Xs = X.unflatten(0, (s, M // s))                        # (s, M/s, K)
    part = torch.bmm(Gs, Xs, out_dtype=torch.float32).contiguous()   # (s, N, K) fp32 slab partials
    out = torch.empty(N, K, device=part.device, dtype=torch.float32)
    # one coalesced pass over the slabs in a fixed order (torch's dim-0 sum ran at ~3 TB/s)
    _lib.check(_lib.load().mc_sum_slabs(s, N * K, part.data_ptr(), part.stride(0), out.data_ptr(),
                                        _lib.stream_handle(part.device)), "mc_sum_slabs")
    return out


def colsum(x):
    """(R, C) fp32 / bf16 / fp16 with unit column stride -> (C,) fp32 column sums (mc_colsum): fixed row
    slices, folded in order -- deterministic, no cross-workgroup hand-off inside the launch (torch's
    reduction of the same shape combines workgroups through a staging buffer and returned wrong sums
    beside concurrent library GEMMs: DESIGN.md 4.9)."""
    if x.stride(-1) != 1:
        x = x.contiguous()
    R, C = x.shape
    out = torch.empty(C, device=x.device, dtype=torch.float32)
    lib = _lib.load()
    ws_b = lib.mc_colsum_workspace_bytes(R, C)
    ws = _ws(ws_b, x.device)
    _lib.check(lib.mc_colsum(R, C, _lib.dtype_code(x.dtype), x.data_ptr(), x.stride(0), out.data_ptr(), ws.data_ptr(),
                             ws_b, _lib.stream_handle(x.device)), "mc_colsum")
    return out


class L2NormalizeFn(torch.autograd.Function):
    """torch.nn.functional.normalize(x, dim=-1) for 2-D x (the towers' output features, reference
    model.py:1011-1017): fp32 out; one wave per row each way (mc_l2norm_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, x, eps):
        x2 = x if x.stride(-1) == 1 else x.contiguous()
        R, C = x2.shape
        y = torch.empty(R, C, device=x.device, dtype=torch.float32)
        norm = torch.empty(R, device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().mc_l2norm_fwd(R, C, _lib.dtype_code(x2.dtype), x2.data_ptr(), x2.stride(0), eps,
                                             y.data_ptr(), C, norm.data_ptr(), _lib.stream_handle(x.device)),
                   "mc_l2norm_fwd")
        ctx.save_for_backward(x2, norm)
        ctx.eps = eps
        return y

    @staticmethod
    def backward(ctx, g):
        x2, norm = ctx.saved_tensors
        g = g.float()
        if g.stride(-1) != 1:
            g = g.contiguous()
        R, C = x2.shape
        dx = torch.empty(R, C, device=x2.device, dtype=x2.dtype)
        _lib.check(_lib.load().mc_l2norm_bwd(R, C, _lib.dtype_code(x2.dtype), x2.data_ptr(), x2.stride(0),
                                             norm.data_ptr(), ctx.eps, g.data_ptr(), g.stride(0), dx.data_ptr(), C,
                                             _lib.stream_handle(x2.device)), "mc_l2norm_bwd")
        return dx, None


def l2_normalize(x, eps=1e-12):
    """F.normalize(x, dim=-1) on the GPU kernels for 2-D CUDA tensors; torch elsewhere.  Result dtype as
    torch's: fp32 under CUDA autocast (norm runs in fp32 there and the division promotes), the input's
    dtype otherwise (pure_bf16 / pure_fp16 precisions)."""
    if x.is_cuda and x.dim() == 2 and x.dtype in (torch.float32, torch.bfloat16, torch.float16) and x.shape[1] > 0:
        y = L2NormalizeFn.apply(x, eps)
        if x.dtype != torch.float32 and not torch.is_autocast_enabled("cuda"):
            y = y.to(x.dtype)
        return y
    return torch.nn.functional.normalize(x, dim=-1, eps=eps)


class TokenEmbedFn(torch.autograd.Function):
    """ViT token embedding: m = cat([cls, x], 1) + pos, cls / pos cast to x's dtype (reference
    model.py:232-358 via open_clip / timm's _pos_embed).  Same forward values as the torch ops; the
    backward's batch reductions (d pos = sum_b dm, d cls = sum_b dm[:, 0] = d pos[0]) run as one
    deterministic mc_colsum in fp32 instead of two torch reductions."""

    @staticmethod
    def forward(ctx, cls, x, pos):
        B, N, C = x.shape
        m = torch.cat([cls.to(x.dtype).expand(B, -1, -1), x], dim=1) + pos.to(x.dtype)
        ctx.meta = (cls.dtype, pos.dtype, N)
        return m

    @staticmethod
    def backward(ctx, dm):
        cls_dt, pos_dt, N = ctx.meta
        B, _, C = dm.shape
        dpos = colsum(dm.reshape(B, (N + 1) * C)).view(1, N + 1, C)
        dcls = dpos[:, :1].clone()
        return dcls.to(cls_dt), dm[:, 1:], dpos.to(pos_dt)


def token_embed(cls, x, pos):
    if x.is_cuda and cls.requires_grad and pos.requires_grad:
        return TokenEmbedFn.apply(cls, x, pos)
    return torch.cat([cls.to(x.dtype).expand(x.shape[0], -1, -1), x], dim=1) + pos.to(x.dtype)


class AddPosFn(torch.autograd.Function):
    """h + pos[:, :T] for (B, T, C) h and a (1, Tmax, C) position table (BERT's position embedding):
    the table's gradient is a deterministic batch column sum (mc_colsum), rows >= T zero."""

    @staticmethod
    def forward(ctx, h, pos):
        T = h.shape[1]
        ctx.meta = (pos.shape, pos.dtype, h.dtype)
        return h + pos[:, :T]

    @staticmethod
    def backward(ctx, g):
        pshape, pdt, hdt = ctx.meta
        B, T, C = g.shape
        dpos = torch.zeros(pshape, device=g.device, dtype=pdt)
        dpos[:, :T] = colsum(g.reshape(B, T * C)).view(1, T, C).to(pdt)
        return g, dpos


def add_pos(h, pos):
    if h.is_cuda and pos.requires_grad:
        return AddPosFn.apply(h, pos)
    return h + pos[:, : h.shape[1]]


def sum_rows(t):
    """(R, n) fp32 contiguous -> (n,) column sums in a fixed order: two mc_sum_slabs passes (R -> R/16
    -> 1) when R is a multiple of 16, so each pass has enough workgroups (one pass over R = 256 rows
    of 2304 -- the attention backward's per-batch sums -- would run 3 workgroups)."""
    R, n = t.shape
    lib, st = _lib.load(), _lib.stream_handle(t.device)
    if R >= 64 and R % 16 == 0:
        mid = torch.empty(R // 16, n, device=t.device, dtype=torch.float32)
        _lib.check(lib.mc_sum_slabs(16, (R // 16) * n, t.data_ptr(), (R // 16) * n, mid.data_ptr(), st), "mc_sum_slabs")
        t, R = mid, R // 16
    out = torch.empty(n, device=t.device, dtype=torch.float32)
    _lib.check(lib.mc_sum_slabs(R, n, t.data_ptr(), n, out.data_ptr(), st), "mc_sum_slabs")
    return out


class NegExpManyFn(torch.autograd.Function):
    """A_i = -exp(A_log_i) for every mixer of a tower in one multi-tensor launch (plus one in-place
    negation); backward dA_log_i = dA_i * A_i in one launch.  Per mixer this was 4 single-tensor
    launches (exp, neg; neg, mul) -- reference mixer: A = -torch.exp(self.A_log.float())
    (model.py:519-528).  Bitwise the same values: negation is exact."""

    @staticmethod
    def forward(ctx, *logs):
        outs = torch._foreach_exp([t.float() for t in logs])
        torch._foreach_neg_(outs)
        ctx.save_for_backward(*outs)
        ctx.set_materialize_grads(False)   # an A without a gradient gets none (not a zero pass)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        outs = ctx.saved_tensors
        idx = [i for i, g in enumerate(gs) if g is not None]
        res = [None] * len(gs)
        if idx:
            for i, v in zip(idx, torch._foreach_mul([gs[i].float() for i in idx], [outs[i] for i in idx])):
                res[i] = v
        return tuple(res)


def neg_exp_many(logs):
    return list(NegExpManyFn.apply(*logs))


class GradHandoff:
    """The Mamba mixer's x (conv output) feeds both x_proj and the scan, so its gradient is the sum of
    x_proj's dX and the scan's du.  The scan backward (which always runs first: x_proj's output
    gradient needs its ddelta / dB / dC) parks du here and returns no gradient for u; x_proj's
    backward then accumulates dX onto du in its GEMM epilogue (addmm_, beta = 1), so the separate
    bf16 add of the two producers -- and its extra pass over the (d_inner, B*L) gradient -- goes."""

    def __init__(self):
        self.du = None

    def take(self):
        du, self.du = self.du, None
        return du


# ---------------------------------------------------------------------------- per-forward weight casts (mc_cast_f32_many)
# Under autocast every projection casts its fp32 weight (and bias) to bf16 on each use: ~230
# single-tensor cast launches per C2 step.  weight_cast_scope(model, dt) casts all of a model's
# Linear parameters in ONE launch into a fresh buffer at the start of its forward; the autograd
# functions below take their 16-bit weights from it (_wcast).  The scope ends with the forward, so
# a copy is never served for a later forward (parameters may have changed); the backward uses the
# copies its forward saved, exactly as with per-use casts.
_WCAST = None   # {id(param): (param, 16-bit copy)} while a scope is active
_WCAST_T = None  # {id(param): (param, 16-bit TRANSPOSED copy)} for the weights _T_WANTED names
_T_WANTED = weakref.WeakValueDictionary()   # id -> weight whose input gradient asked for a transposed copy
_CAST_PLANS = {}


def _wcast(t, dt):
    """t.to(dt), served from the active weight_cast_scope when t is one of its parameters."""
    if t.dtype == dt:
        return t
    if _WCAST is not None:
        e = _WCAST.get(id(t))
        if e is not None and e[0] is t and e[1].dtype == dt:
            return e[1]
    return t.to(dt)


class _CastPlan:
    """Chunk table (device) and buffer layout for one parameter set."""

    def __init__(self, params, dt, device):
        offs, off = [], 0
        rows = []
        for p in params:
            offs.append(off)
            n = p.numel()
            for s0 in range(0, n, _lib.MC_CAST_CHUNK):
                rows.append((p.data_ptr() + 4 * s0, off + s0, min(_lib.MC_CAST_CHUNK, n - s0)))
            off += (n + 7) // 8 * 8                     # 16-B aligned slices
        self.offs, self.total, self.dt = offs, off, dt
        self.nchunks = len(rows)
        self.table = torch.tensor(rows, dtype=torch.int64).to(device)   # mc_cast_chunk = 3 x 8 B

    def run(self, params):
        buf = torch.empty(self.total, device=self.table.device, dtype=self.dt)
        _lib.check(_lib.load().mc_cast_f32_many(self.nchunks, self.table.data_ptr(), buf.data_ptr(),
                                                _lib.dtype_code(self.dt), _lib.stream_handle(buf.device)),
                   "mc_cast_f32_many")
        return [buf[o:o + p.numel()].view(p.shape) for o, p in zip(self.offs, params)]


def _wcast_t(weight, x, dt):
    """The 16-bit transposed copy of `weight` for the "tn" input gradient (_dgrad) when that form
    applies to x @ weight^T, served from the active weight_cast_scope; None when the form does not
    apply or the scope has no copy yet (the weight is then registered, and the next scope casts it)."""
    if not (DGRAD_TN and WCAST_T and x.is_cuda and weight.dim() == 2 and weight.numel() >= 1 << 19
            and x.numel() // max(x.shape[-1], 1) >= 8192):
        return None
    if _WCAST_T is not None:
        e = _WCAST_T.get(id(weight))
        if e is not None and e[0] is weight and e[1].dtype == dt:
            return e[1]
    if _WCAST is not None and weight.dtype == torch.float32:
        _T_WANTED[id(weight)] = weight
    return None


class _TransposePlan:
    """Tile table (device, mc_cast_t_tile = 4 x 8 B) and buffer layout for the transposed copies."""

    def __init__(self, params, dt, device):
        offs, off, rows = [], 0, []
        for p in params:
            R, C = p.shape
            offs.append(off)
            for r0 in range(0, R, 64):
                for c0 in range(0, C, 64):
                    rows.append((p.data_ptr() + 4 * (r0 * C + c0), off + c0 * R + r0,
                                 C | (R << 32), min(64, R - r0) | (min(64, C - c0) << 32)))
            off += (R * C + 7) // 8 * 8
        self.offs, self.total, self.dt = offs, off, dt
        self.ntiles = len(rows)
        self.table = torch.tensor(rows, dtype=torch.int64).to(device)

    def run(self, params):
        buf = torch.empty(self.total, device=self.table.device, dtype=self.dt)
        _lib.check(_lib.load().mc_cast_transpose_f32_many(self.ntiles, self.table.data_ptr(), buf.data_ptr(),
                                                          _lib.dtype_code(self.dt), _lib.stream_handle(buf.device)),
                   "mc_cast_transpose_f32_many")
        return [buf[o:o + p.numel()].view(p.shape[1], p.shape[0]) for o, p in zip(self.offs, params)]


class weight_cast_scope:
    """Context manager: one-launch 16-bit copies of `module`'s Linear weights / biases for one forward
    (no-op off the GPU, outside autocast, or when nested)."""

    def __init__(self, module, dt):
        self.module, self.dt, self.active = module, dt, False
        self.buf = self.buf_t = None

    def record_stream(self, stream):
        """The copies are used on another stream too (ClipModel's concurrent towers)."""
        for b in (self.buf, self.buf_t):
            if b is not None:
                b.record_stream(stream)

    def __enter__(self):
        global _WCAST, _WCAST_T
        if _WCAST is not None or self.dt not in (torch.bfloat16, torch.float16):
            return self
        params = [p for m in self.module.modules() if isinstance(m, torch.nn.Linear)
                  for p in (m.weight, m.bias)
                  if p is not None and p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()]
        if not params:
            return self
        key = (id(self.module), self.dt, tuple((p.data_ptr(), p.numel()) for p in params))
        plan = _CAST_PLANS.get(key[:2])
        if plan is None or plan[0] != key:
            plan = (key, _CastPlan(params, self.dt, params[0].device))
            _CAST_PLANS[key[:2]] = plan
        copies = plan[1].run(params)
        self.buf = copies[0]
        _WCAST = {id(p): (p, c) for p, c in zip(params, copies)}
        tparams = [p for p in params if p.dim() == 2 and _T_WANTED.get(id(p)) is p]
        if tparams:
            tkey = (id(self.module), self.dt, "t", tuple((p.data_ptr(), p.shape) for p in tparams))
            tplan = _CAST_PLANS.get(tkey[:3])
            if tplan is None or tplan[0] != tkey:
                tplan = (tkey, _TransposePlan(tparams, self.dt, params[0].device))
                _CAST_PLANS[tkey[:3]] = tplan
            tcopies = tplan[1].run(tparams)
            self.buf_t = tcopies[0]
            _WCAST_T = {id(p): (p, c) for p, c in zip(tparams, tcopies)}
        self.active = True
        return self

    def __exit__(self, *exc):
        global _WCAST, _WCAST_T
        if self.active:
            _WCAST = _WCAST_T = None
        return False


# Input gradients dx = g @ w of the towers' projections with the weight TRANSPOSED first: hipBLASLt
# runs the "tn" form of these shapes (the forward's) faster than the "nn" form torch picks for a
# row-major w -- e.g. the ViT fc2 input gradient (50432 x 3072 x 768): 0.246 ms nn vs 0.188 ms tn in
# the tuning file (tuning/gemm_gfx950_dp.csv).  The transposed 16-bit copies come from the forward's
# weight_cast_scope (mc_cast_transpose_f32_many, one launch for all of them: _wcast_t); a per-call
# transpose of the 16-bit copy (~40 us each for the ViT's fc weights) is only the first step's
# fallback.  A/B toggle.
DGRAD_TN = os.environ.get("MAMBA_CLIP_AMD_DGRAD_TN", "1") != "0"
WCAST_T = os.environ.get("MAMBA_CLIP_AMD_WCAST_T", "1") != "0"     # A/B: scope copies vs per-call transposes


# The remaining towers' Linear forward / input-gradient GEMMs (qkv, proj, patch embedding, the MLP's
# fc1 input gradient) on mc_linear instead of the library: A/B toggles.
LINEAR_HIP_FWD = os.environ.get("MAMBA_CLIP_AMD_LINEAR_HIP_FWD", "0") == "1"
LINEAR_HIP_DGRAD = os.environ.get("MAMBA_CLIP_AMD_LINEAR_HIP_DGRAD", "0") == "1"


def _fwd_gemm(xc, wc, bc):
    """F.linear(xc, wc, bc), on mc_linear (bias epilogue) when LINEAR_HIP_FWD and the shapes qualify."""
    if LINEAR_HIP_FWD and xc.is_cuda and xc.dim() >= 2 and (bc is None or bc.dtype == xc.dtype):
        x2 = xc.reshape(-1, xc.shape[-1])
        if x2.shape[0] >= 8192 and linear_hip_ok(x2, wc):
            return linear_hip(x2, wc, bc).view(*xc.shape[:-1], wc.shape[0])
    return torch.nn.functional.linear(xc, wc, bc)


def _dgrad(g2, wc, wt=None):
    """g2 (M, N) @ wc (N, K) for a row-major weight copy wc (wt: its transposed copy, or None)."""
    if LINEAR_HIP_DGRAD and wt is not None and g2.shape[0] >= 8192 and linear_hip_ok(g2, wt):
        return linear_hip(g2, wt)
    if wt is not None:
        return torch.mm(g2, wt.t())
    if DGRAD_TN and g2.is_cuda and g2.shape[0] >= 8192 and wc.shape[0] * wc.shape[1] >= 1 << 19:
        return torch.mm(g2, wc.t().contiguous().t())
    return torch.mm(g2, wc)


def _compute_dtype(t):
    if t.is_cuda and torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return t.dtype


class LinearSK(torch.autograd.Function):
    """y = x @ w^T (+ b), autocast-aware; backward: dx = g @ w, dw = split-K g^T x (fp32), db = sum g."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        dt = _compute_dtype(x)
        xc, wc = x.to(dt), _wcast(weight, dt)
        bc = _wcast(bias, dt) if bias is not None else None
        with torch.autocast("cuda", enabled=False):
            y = _fwd_gemm(xc, wc, bc)
        ctx.save_for_backward(xc, wc)
        ctx.has_bias = bias is not None
        colmajor = xc.dim() == 2 and xc.stride(0) == 1 and xc.stride(1) != 1
        ctx.wt = None if colmajor else _wcast_t(weight, xc, dt)
        return y

    @staticmethod
    def backward(ctx, gy):
        xc, wc = ctx.saved_tensors
        K = xc.shape[-1]
        g2 = gy.reshape(-1, gy.shape[-1]).to(wc.dtype)
        x2 = xc.reshape(-1, K)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if xc.dim() == 2 and xc.stride(0) == 1 and xc.stride(1) != 1:
                # x is a transposed (column-major) view, e.g. the mixer's channel-major
                # scan output: produce dx in the same layout so the producer's
                # backward needs no transpose copy
                dx = torch.mm(wc.t(), g2.t()).t()
            else:
                dx = _dgrad(g2, wc, ctx.wt).view(xc.shape)
        if ctx.needs_input_grad[1]:
            dw = wgrad(g2.t(), x2)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            pre = getattr(gy, COLSUM_ATTR, None)   # column sums taken by the producer of gy (LayerNorm bwd)
            if pre is not None and pre[1] == gy._version and pre[0].shape[0] == g2.shape[1]:
                db = pre[0]
            elif g2.is_cuda:
                db = colsum(g2)
            else:
                db = torch.sum(g2, 0, dtype=torch.float32)
        return dx, dw, db


def linear_sk(x, weight, bias=None):
    return LinearSK.apply(x, weight, bias)


# w @ X with a short reduction (the mixer's dt_proj forward, K = dt_rank) on mc_gemm_small_k instead of
# the library GEMM.  A/B toggle.
SMALL_K_HIP = os.environ.get("MAMBA_CLIP_AMD_SMALL_K_HIP", "1") != "0"


def small_k_ok(wc, Xc):
    K = wc.shape[1]
    return (SMALL_K_HIP and Xc.is_cuda and wc.dtype == Xc.dtype and Xc.dtype in (torch.bfloat16, torch.float16)
            and K in (16, 32, 48, 64) and Xc.shape[1] % 8 == 0 and Xc.stride(1) == 1 and Xc.stride(0) % 8 == 0
            and Xc.data_ptr() % 16 == 0 and wc.stride(1) == 1 and wc.stride(0) % 4 == 0 and wc.data_ptr() % 8 == 0)


def gemm_small_k(wc, Xc):
    """wc (M, K) @ Xc (K, T) on mc_gemm_small_k (caller checks small_k_ok)."""
    M, K = wc.shape
    T = Xc.shape[1]
    y = torch.empty(M, T, device=Xc.device, dtype=Xc.dtype)
    _lib.check(_lib.load().mc_gemm_small_k(M, K, T, _lib.dtype_code(Xc.dtype), wc.data_ptr(), wc.stride(0),
                                           Xc.data_ptr(), Xc.stride(0), y.data_ptr(), T,
                                           _lib.stream_handle(Xc.device)), "mc_gemm_small_k")
    return y


# w @ X with few output rows and a long reduction (the mixer's x_proj forward, 80 x 1536) on
# mc_gemm_skinny_m.  A/B toggle, off: as built it streams X at 1.7 TB/s (38.3 vs the library's 25.7 us at
# C2; step +0.1-0.25 ms, profiles/r05/mixer/) -- one 8 KB chunk in flight per wave, latency-bound.
SKINNY_M_HIP = os.environ.get("MAMBA_CLIP_AMD_SKINNY_M_HIP", "0") == "1"


def skinny_m_ok(wc, Xc):
    M, K = wc.shape
    return (SKINNY_M_HIP and Xc.is_cuda and wc.dtype == Xc.dtype and Xc.dtype in (torch.bfloat16, torch.float16)
            and 0 < M <= 96 and K % 256 == 0 and Xc.shape[1] % 8 == 0 and Xc.stride(1) == 1
            and Xc.stride(0) % 8 == 0 and Xc.data_ptr() % 16 == 0 and wc.stride(1) == 1 and wc.stride(0) % 4 == 0
            and wc.data_ptr() % 8 == 0)


def gemm_skinny_m(wc, Xc):
    """wc (M, K) @ Xc (K, T) on mc_gemm_skinny_m (caller checks skinny_m_ok)."""
    M, K = wc.shape
    T = Xc.shape[1]
    y = torch.empty(M, T, device=Xc.device, dtype=Xc.dtype)
    _lib.check(_lib.load().mc_gemm_skinny_m(M, K, T, _lib.dtype_code(Xc.dtype), wc.data_ptr(), wc.stride(0),
                                            Xc.data_ptr(), Xc.stride(0), y.data_ptr(), T,
                                            _lib.stream_handle(Xc.device)), "mc_gemm_skinny_m")
    return y


class WeightLeftMM(torch.autograd.Function):
    """y = w @ X for a weight w (N, K) and activations X (K, M) (channel-major GEMMs of the Mamba mixer)."""

    @staticmethod
    def forward(ctx, weight, X, handoff=None, out_slab=None):
        dt = _compute_dtype(X)
        wc, Xc = _wcast(weight, dt), X.to(dt)
        with torch.autocast("cuda", enabled=False):
            if small_k_ok(wc, Xc):
                y = gemm_small_k(wc, Xc)
            elif skinny_m_ok(wc, Xc):
                y = gemm_skinny_m(wc, Xc)
            else:
                y = torch.mm(wc, Xc)
        ctx.save_for_backward(wc, Xc)
        ctx.handoff = handoff
        ctx.out_slab = out_slab   # (GradSlab, first row): dX written into those rows (ops.GradSlab)
        return y

    @staticmethod
    def backward(ctx, gy):
        wc, Xc = ctx.saved_tensors
        g = gy.to(wc.dtype)
        dw = dX = None
        if ctx.needs_input_grad[0]:
            dw = wgrad(g, Xc.t())
        acc = ctx.handoff.take() if ctx.handoff is not None else None
        if ctx.needs_input_grad[1]:
            accv = acc.transpose(0, 1) if (acc is not None and Xc.is_contiguous()) else None
            accv = accv.view(Xc.shape) if (accv is not None and accv.is_contiguous()
                                           and accv.numel() == Xc.numel()) else None
            if accv is not None:
                # the other consumer's gradient (GradHandoff), in X's layout: dX += w^T g in the epilogue
                dX = accv
                dX.addmm_(wc.t(), g)
                acc = None
            elif Xc.stride(0) == 1 and Xc.stride(1) != 1:
                dX = torch.mm(g.t(), wc).t()      # X is a transposed view: keep its layout (no copy downstream)
            elif ctx.out_slab is not None and acc is None and Xc.is_contiguous():
                slab, r0 = ctx.out_slab
                dX = slab.get()[r0:r0 + Xc.shape[0]]
                torch.mm(wc.t(), g, out=dX)
            else:
                dX = torch.mm(wc.t(), g)
            if acc is not None:   # handed-off gradient in another layout: summed after the GEMM
                dX = dX + acc.transpose(0, 1).reshape(Xc.shape)
        return dw, dX, None, None


def wleft_mm(weight, X, handoff=None, out_slab=None):
    return WeightLeftMM.apply(weight, X, handoff, out_slab)


def mixer_proj_ok(x_cm, rank, dstate):
    """Shapes mc_mixer_proj_* take: 16-bit (D, T) rows with unit token stride, D % 64, T % 8, rank % 16
    in [16, 96], dstate 16 (every reference config)."""
    dt = _compute_dtype(x_cm)
    D, T = x_cm.shape
    return (x_cm.is_cuda and dt in (torch.bfloat16, torch.float16) and x_cm.stride(1) == 1 and D % 64 == 0
            and T % 8 == 0 and T > 0 and rank % 16 == 0 and 16 <= rank <= 96 and dstate == 16
            and x_cm.stride(0) % 8 == 0 and x_cm.data_ptr() % 16 == 0)


class MixerProjFn(torch.autograd.Function):
    """x_dbl = x_proj(x), delta = dt_proj.weight @ x_dbl[:R] for the Mamba mixer's channel-major
    activations (D, T), in one HIP pass (mc_mixer_proj_fwd); backward: d_x_dbl and dx = x_proj^T d_x_dbl
    + du (the scan's gradient, handed over by ops.GradHandoff) in one pass (mc_mixer_proj_bwd), the two
    weight gradients as split-K GEMMs (ops.wgrad).  Same roundings as the library-GEMM chain:
    x_dbl, delta, d_dtraw and dx stored once in the activation dtype."""

    @staticmethod
    def forward(ctx, x, w_x, w_dt, handoff):
        dt = _compute_dtype(x)
        lib = _lib.load()
        xc = x if x.dtype == dt else x.to(dt)
        wx, wdt = _wcast(w_x, dt).contiguous(), _wcast(w_dt, dt).contiguous()
        D, T = xc.shape
        P, R = wx.shape[0], wdt.shape[1]
        xd = torch.empty(P, T, device=xc.device, dtype=dt)
        delta = torch.empty(D, T, device=xc.device, dtype=dt)
        p = _lib.MixerProjParams()
        p.dim, p.tokens, p.rank, p.proj_rows, p.dtype = D, T, R, P, _lib.dtype_code(dt)
        p.x_ld, p.x_dbl_ld, p.delta_ld = xc.stride(0), T, T
        p.x, p.w_x, p.w_dt, p.x_dbl, p.delta = xc.data_ptr(), wx.data_ptr(), wdt.data_ptr(), xd.data_ptr(), delta.data_ptr()
        _lib.check(lib.mc_mixer_proj_fwd(ctypes.byref(p), _lib.stream_handle(xc.device)), "mc_mixer_proj_fwd")
        ctx.save_for_backward(xc, wx, wdt, xd)
        ctx.handoff = handoff
        # B and C rows as their own outputs (views of x_dbl): their gradients arrive separately, so
        # autograd never builds a zero-filled (P, T) gradient of x_dbl
        return xd[R:P - 16], xd[P - 16:], delta

    @staticmethod
    def backward(ctx, g_b, g_c, g_delta):
        xc, wx, wdt, xd = ctx.saved_tensors
        lib = _lib.load()
        D, T = xc.shape
        P, R = wx.shape[0], wdt.shape[1]
        dt = xc.dtype
        if g_delta is None:
            g_delta = torch.zeros(D, T, device=xc.device, dtype=dt)
        g_delta = _hip_rows(g_delta.to(dt), 8, "MixerProjFn")
        g_b = _hip_rows(g_b.to(dt), 8, "MixerProjFn") if g_b is not None else None
        g_c = _hip_rows(g_c.to(dt), 8, "MixerProjFn") if g_c is not None else None
        du = ctx.handoff.take() if ctx.handoff is not None else None
        if du is not None:
            du = du.transpose(0, 1)                          # (B, D, L) channel-major -> (D, B, L)
            du = du.reshape(D, T) if du.is_contiguous() else du.reshape(D, T).contiguous()
            du = du.to(dt)
        dxd = torch.empty(P, T, device=xc.device, dtype=dt)
        dx = torch.empty(D, T, device=xc.device, dtype=dt)
        p = _lib.MixerProjBwdParams()
        p.dim, p.tokens, p.rank, p.proj_rows, p.dtype = D, T, R, P, _lib.dtype_code(dt)
        p.g_delta_ld, p.d_x_dbl_ld, p.dx_ld = g_delta.stride(0), T, T
        p.g_delta, p.w_x, p.w_dt, p.d_x_dbl, p.dx = g_delta.data_ptr(), wx.data_ptr(), wdt.data_ptr(), dxd.data_ptr(), dx.data_ptr()
        if g_b is not None:
            p.g_b, p.g_b_ld = g_b.data_ptr(), g_b.stride(0)
        if g_c is not None:
            p.g_c, p.g_c_ld = g_c.data_ptr(), g_c.stride(0)
        if du is not None:
            p.du, p.du_ld = du.data_ptr(), du.stride(0)
        _lib.check(lib.mc_mixer_proj_bwd(ctypes.byref(p), _lib.stream_handle(xc.device)), "mc_mixer_proj_bwd")
        dw_x = wgrad(dxd, xc.t()) if ctx.needs_input_grad[1] else None
        dw_dt = wgrad(g_delta, xd[:R].t()) if ctx.needs_input_grad[2] else None
        return (dx if ctx.needs_input_grad[0] else None), dw_x, dw_dt, None


def mixer_proj(x_cm, w_x, w_dt, handoff=None):
    """(B rows (16, T), C rows (16, T), delta (D, T)) for the mixer's channel-major x (D, T): the
    x_dbl = [dt_raw; B; C] split of x_proj with dt_raw consumed by dt_proj inside; see MixerProjFn."""
    return MixerProjFn.apply(x_cm, w_x, w_dt, handoff)


# ---------------------------------------------------------------------------- fused bias-gradient passes (mc_ops.h)
def _aligned_rows(t, V):
    return t.stride(-1) == 1 and t.data_ptr() % 16 == 0 and t.stride(0) % V == 0


def _hip_rows(t, V, who):
    """t with 16-B aligned rows for a HIP kernel: a fresh dense copy when t's layout does not
    qualify.  There is no torch fallback on the GPU: a width the kernel cannot tile raises."""
    if t.shape[-1] % V:
        raise RuntimeError(f"{who}: row width {t.shape[-1]} must be a multiple of {V} elements")
    return t if _aligned_rows(t, V) else t.clone(memory_format=torch.contiguous_format)


# ---------------------------------------------------------------------------- towers' Linears on mc_linear
# The forward / input-gradient GEMMs of the ViT Linears on the hand-written 256 x 256 kernel
# (csrc/gemm_wgrad.hip, mc_linear) with the epilogues the library cannot fuse: bias + exact-erf GELU
# for fc1 (one pass writes h and gelu(h)) and GELU' for fc2's input gradient (one pass writes
# gh = ga * gelu'(h) and fc1's bias gradient).


def linear_hip_ok(x2, w):
    """x2 (rows, K) and w (cols, K) qualify for mc_linear: 16-bit, same dtype, unit stride along K,
    K % 64, cols % 8, 16-B aligned rows."""
    return (x2.is_cuda and x2.dim() == 2 and w.dim() == 2 and x2.dtype == w.dtype
            and x2.dtype in (torch.bfloat16, torch.float16) and x2.shape[1] == w.shape[1]
            and x2.shape[1] % 64 == 0 and x2.shape[1] > 0 and w.shape[0] % 8 == 0
            and x2.stride(1) == 1 and w.stride(1) == 1 and x2.stride(0) % 8 == 0 and w.stride(0) % 8 == 0
            and x2.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


def linear_hip(x2, w, bias=None, epilogue=None, h=None, want_colsum=False):
    """x2 @ w^T on mc_linear with a fused epilogue (include/mc_gemm.h):
    NONE / BIAS -> y; BIAS_GELU -> (h, gelu(h)); GELU_GRAD (h = the pre-activation) -> (gh, colsum or None).
    The caller checks linear_hip_ok; a launch error raises (no library fallback inside)."""
    if epilogue is None:
        epilogue = _lib.MC_LINEAR_EPI_BIAS if bias is not None else _lib.MC_LINEAR_EPI_NONE
    rows, K = x2.shape
    cols = w.shape[0]
    y = torch.empty(rows, cols, device=x2.device, dtype=x2.dtype)
    p = _lib.LinearParams()
    p.rows, p.cols, p.K, p.dtype, p.epilogue = rows, cols, K, _lib.dtype_code(x2.dtype), epilogue
    p.X, p.ldx, p.W, p.ldw, p.Y, p.ldy = x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0), y.data_ptr(), cols
    y2 = colsum_out = None
    if bias is not None:
        if bias.dtype != x2.dtype or bias.stride(0) != 1 or bias.data_ptr() % 8:
            bias = bias.to(x2.dtype).contiguous()
        p.bias = bias.data_ptr()
    if epilogue == _lib.MC_LINEAR_EPI_BIAS_GELU:
        y2 = torch.empty_like(y)
        p.Y2, p.ldy2 = y2.data_ptr(), cols
    ws = None
    if epilogue == _lib.MC_LINEAR_EPI_GELU_GRAD:
        h = _hip_rows(h, 8, "linear_hip GELU_GRAD")
        p.H, p.ldh = h.data_ptr(), h.stride(0)
        if want_colsum:
            colsum_out = torch.empty(cols, device=x2.device, dtype=torch.float32)
            p.colsum = colsum_out.data_ptr()
    lib = _lib.load()
    ws_b = lib.mc_linear_workspace_bytes(ctypes.byref(p))
    if ws_b:
        ws = _ws(ws_b, x2.device)
        p.workspace, p.workspace_bytes = ws.data_ptr(), ws_b
    _lib.check(lib.mc_linear(ctypes.byref(p), _lib.stream_handle(x2.device)), "mc_linear")
    if epilogue == _lib.MC_LINEAR_EPI_BIAS_GELU:
        return y, y2
    if epilogue == _lib.MC_LINEAR_EPI_GELU_GRAD:
        return y, colsum_out
    return y


# which MLP passes run on mc_linear (A/B toggles, tools/ab_step.py --toggle ops.MLP_HIP_FC1 ...):
#   FC1: fc1 + bias + GELU in one epilogue; FC2: fc2 + bias; BWD: fc2's input gradient times GELU' with
#   fc1's bias gradient in one epilogue, and fc1's input gradient.  Off: the library GEMM of that pass
#   (+ the standalone GELU / mc_gelu_bwd passes).  Measured in DESIGN 4.3 (round 5, same-box C2 step
#   A/B, profiles/r05/linear/): BWD -0.35..-0.52 ms (4 of 4 reps), FC2 -0.04..-0.35 ms (3 of 3) -- on;
#   FC1 +0.07..+0.44 ms (its un-overlapped GELU epilogue costs more than the pass it saves) -- off.
MLP_HIP_FC1 = os.environ.get("MAMBA_CLIP_AMD_MLP_HIP_FC1", "0") == "1"
MLP_HIP_FC2 = os.environ.get("MAMBA_CLIP_AMD_MLP_HIP_FC2", "1") == "1"
MLP_HIP_BWD = os.environ.get("MAMBA_CLIP_AMD_MLP_HIP_BWD", "1") == "1"


def _gelu_bwd(h2, g2):
    """(gh, db) = (g2 * gelu'(h2), column sums of gh) in one pass (mc_gelu_bwd)."""
    lib = _lib.load()
    V = 16 // h2.element_size()
    cols = h2.shape[1]
    h2, g2 = _hip_rows(h2, V, "gelu backward"), _hip_rows(g2, V, "gelu backward")
    gh = torch.empty_like(h2)
    db = torch.empty(cols, device=h2.device, dtype=torch.float32)
    ws_b = lib.mc_grad_colsum_workspace_bytes(h2.shape[0], cols)
    ws = _ws(ws_b, h2.device)
    _lib.check(lib.mc_gelu_bwd(h2.shape[0], cols, _lib.dtype_code(h2.dtype), h2.data_ptr(), h2.stride(0),
                               g2.data_ptr(), g2.stride(0), gh.data_ptr(), gh.stride(0), db.data_ptr(),
                               ws.data_ptr(), ws_b, _lib.stream_handle(h2.device)), "mc_gelu_bwd")
    return gh, db


class MlpFn(torch.autograd.Function):
    """y = fc2(gelu(fc1(x))) -- the ViT block's MLP (timm Mlp: fc1 -> nn.GELU() exact erf -> fc2; the
    reference's image tower, model.py:1011-1017), each pass on mc_linear or the library per the
    MLP_HIP_* toggles:
      forward:  (h, a) = fc1 + bias + GELU in one epilogue;  y = a @ w2^T + b2
      backward: gh = (gy @ w2) * gelu'(h) with fc1's bias gradient in one epilogue (no standalone
                GELU-backward pass, no stored fc2 input gradient);  dx = gh @ w1;  dW1, dW2 on
                mc_gemm_wgrad;  db2 = column sums of gy.
    Same roundings as the unfused chain: h, a, y, ga (inside the epilogue) and gh once each in the
    activation dtype."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        dt = _compute_dtype(x)
        xc = x.to(dt)
        w1c, b1c, w2c, b2c = _wcast(w1, dt), _wcast(b1, dt), _wcast(w2, dt), _wcast(b2, dt)
        x2 = xc.reshape(-1, xc.shape[-1])
        with torch.autocast("cuda", enabled=False):
            # each mc_linear call is guarded by linear_hip_ok (strides / 16-B alignment the kernel needs);
            # an ineligible operand takes the library GEMM instead of failing the step
            if MLP_HIP_FC1 and linear_hip_ok(x2, w1c):
                h, a = linear_hip(x2, w1c, b1c, _lib.MC_LINEAR_EPI_BIAS_GELU)
            else:
                h = torch.nn.functional.linear(x2, w1c, b1c)
                a = torch.nn.functional.gelu(h)
            y = (linear_hip(a, w2c, b2c) if MLP_HIP_FC2 and linear_hip_ok(a, w2c)
                 else torch.nn.functional.linear(a, w2c, b2c))
        ctx.save_for_backward(x2, h, a, w1c, w2c)
        ctx.wt1, ctx.wt2 = _wcast_t(w1, xc, dt), _wcast_t(w2, a, dt)
        ctx.xshape = xc.shape
        return y.view(*xc.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, h, a, w1c, w2c = ctx.saved_tensors
        g2 = gy.reshape(-1, gy.shape[-1]).to(h.dtype)
        if not _aligned_rows(g2, 8):
            g2 = g2.contiguous()
        pre = getattr(gy, COLSUM_ATTR, None)   # gy's column sums taken by its producer (LayerNorm bwd)
        if pre is not None and pre[1] == gy._version and pre[0].shape[0] == g2.shape[1]:
            db2 = pre[0]
        else:
            db2 = colsum(g2)
        dw2 = wgrad(g2.t(), a)
        wt2 = (ctx.wt2 if ctx.wt2 is not None else w2c.t().contiguous()) if MLP_HIP_BWD else None
        if MLP_HIP_BWD and linear_hip_ok(g2, wt2) and _aligned_rows(h, 8):
            gh, db1 = linear_hip(g2, wt2, None, _lib.MC_LINEAR_EPI_GELU_GRAD, h=h, want_colsum=True)
        else:
            gh, db1 = _gelu_bwd(h, _dgrad(g2, w2c, ctx.wt2))
        dw1 = wgrad(gh.t(), x2)
        dx = None
        if ctx.needs_input_grad[0]:
            wt1 = (ctx.wt1 if ctx.wt1 is not None else w1c.t().contiguous()) if MLP_HIP_BWD else None
            if MLP_HIP_BWD and linear_hip_ok(gh, wt1):
                dx = linear_hip(gh, wt1)
            else:
                dx = _dgrad(gh, w1c, ctx.wt1)
            dx = dx.view(ctx.xshape)
        return dx, dw1, db1, dw2, db2


def mlp_hip_ok(x, w1, b1, w2, b2):
    """The ViT MLP qualifies for MlpFn: on the GPU, 16-bit compute, biases, widths % 64 (both GEMMs' K)."""
    dt = _compute_dtype(x)
    return (x.is_cuda and b1 is not None and b2 is not None and dt in (torch.bfloat16, torch.float16) and w1.dim() == 2 and w2.dim() == 2
            and x.shape[-1] % 64 == 0 and w1.shape[0] % 64 == 0 and w2.shape[0] % 64 == 0
            and x.numel() // max(x.shape[-1], 1) >= 1)


def mlp(x, w1, b1, w2, b2):
    """ViT MLP y = fc2(gelu(fc1(x))): MlpFn on the GPU, else fc1_gelu + linear_sk."""
    if (MLP_HIP_FC1 or MLP_HIP_FC2 or MLP_HIP_BWD) and mlp_hip_ok(x, w1, b1, w2, b2):
        return MlpFn.apply(x, w1, b1, w2, b2)
    return linear_sk(fc1_gelu(x, w1, b1), w2, b2)


class FC1GeluFn(torch.autograd.Function):
    """a = gelu(x @ w^T + b) -- the MLP's first projection and activation (timm Mlp fc1 + GELU).

    Backward on the GPU: one pass (mc_gelu_bwd) forms gh = ga * gelu'(h) AND the fc1 bias
    gradient; then dx = gh @ w and the split-K weight gradient.  Elsewhere (CPU tests) the
    same math in torch."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        dt = _compute_dtype(x)
        xc, wc, bc = x.to(dt), _wcast(weight, dt), _wcast(bias, dt)
        with torch.autocast("cuda", enabled=False):
            h = torch.nn.functional.linear(xc, wc, bc)
            a = torch.nn.functional.gelu(h)
        ctx.save_for_backward(xc, wc, h)
        ctx.wt = _wcast_t(weight, xc, dt)
        return a

    @staticmethod
    def backward(ctx, ga):
        xc, wc, h = ctx.saved_tensors
        cols = h.shape[-1]
        h2 = h.reshape(-1, cols)
        g2 = ga.reshape(-1, cols).to(h.dtype)
        V = 16 // h.element_size()
        if h.is_cuda:
            lib = _lib.load()
            h2, g2 = _hip_rows(h2, V, "fc1_gelu backward"), _hip_rows(g2, V, "fc1_gelu backward")
            gh = torch.empty_like(h2)
            db = torch.empty(cols, device=h.device, dtype=torch.float32)
            ws_b = lib.mc_grad_colsum_workspace_bytes(h2.shape[0], cols)
            ws = _ws(ws_b, h.device)
            _lib.check(lib.mc_gelu_bwd(h2.shape[0], cols, _lib.dtype_code(h.dtype), h2.data_ptr(), h2.stride(0),
                                       g2.data_ptr(), g2.stride(0), gh.data_ptr(), gh.stride(0), db.data_ptr(),
                                       ws.data_ptr(), ws_b, _lib.stream_handle(h.device)), "mc_gelu_bwd")
        else:   # CPU tensors (the CPU restatement tests): the same math in torch
            gh = torch.ops.aten.gelu_backward(g2, h2)
            db = gh.sum(0, dtype=torch.float32)
        x2 = xc.reshape(-1, xc.shape[-1])
        dx = _dgrad(gh, wc, ctx.wt).view(xc.shape) if ctx.needs_input_grad[0] else None
        dw = wgrad(gh.t(), x2) if ctx.needs_input_grad[1] else None
        return dx, dw, db if ctx.needs_input_grad[2] else None


def fc1_gelu(x, weight, bias):
    return FC1GeluFn.apply(x, weight, bias)


class QKVProjFn(torch.autograd.Function):
    """(q, k, v) = heads of x @ w^T + b, each (B, H, N, D) -- a view of the (B, N, 3, H, D) output.

    Backward on the GPU: mc_qkv_grad_pack writes dq / dk / dv straight into the packed
    (B*N, 3C) output gradient and sums its columns (the qkv bias gradient) in the same pass --
    no stack copy, no second read; then dx and the split-K weight gradient."""

    @staticmethod
    def forward(ctx, x, weight, bias, heads):
        dt = _compute_dtype(x)
        xc, wc, bc = x.to(dt), _wcast(weight, dt), _wcast(bias, dt)
        Bsz, N, C = xc.shape
        with torch.autocast("cuda", enabled=False):
            y = _fwd_gemm(xc, wc, bc)
        ctx.save_for_backward(xc, wc)
        ctx.heads = heads
        ctx.wt = _wcast_t(weight, xc, dt)
        q, k, v = y.view(Bsz, N, 3, heads, C // heads).unbind(2)
        return q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)

    @staticmethod
    def backward(ctx, dq, dk, dv):
        xc, wc = ctx.saved_tensors
        Bsz, N, C = xc.shape
        H = ctx.heads
        D = C // H
        grads = [g if g is not None else torch.zeros(Bsz, H, N, D, device=xc.device, dtype=xc.dtype)
                 for g in (dq, dk, dv)]
        grads = [g.to(xc.dtype) for g in grads]
        V = 16 // xc.element_size()
        if xc.is_cuda:
            if D % V:
                raise RuntimeError(f"qkv_proj backward: head_dim {D} must be a multiple of {V}")
            grads = [g if (g.stride(-1) == 1 and g.data_ptr() % 16 == 0 and all(st % V == 0 for st in g.stride()[:3]))
                     else g.contiguous() if not g.is_contiguous() else g.clone() for g in grads]
            lib = _lib.load()
            g2 = torch.empty(Bsz * N, 3 * C, device=xc.device, dtype=xc.dtype)
            db = torch.empty(3 * C, device=xc.device, dtype=torch.float32)
            p = _lib.QkvPackParams()
            p.batch, p.seq, p.heads, p.head_dim, p.dtype = Bsz, N, H, D, _lib.dtype_code(xc.dtype)
            for i, g in enumerate(grads):          # g: (B, H, N, D) -> strides of batch, token, head
                p.src[i] = g.data_ptr()
                p.sb[i], p.sn[i], p.sh[i] = g.stride(0), g.stride(2), g.stride(1)
            ws_b = lib.mc_grad_colsum_workspace_bytes(Bsz * N, 3 * C)
            ws = _ws(ws_b, xc.device)
            p.out, p.ld_out, p.dbias = g2.data_ptr(), 3 * C, db.data_ptr()
            p.workspace, p.workspace_bytes = ws.data_ptr(), ws_b
            _lib.check(lib.mc_qkv_grad_pack(p, _lib.stream_handle(xc.device)), "mc_qkv_grad_pack")
        else:   # CPU tensors (the CPU restatement tests): the same math in torch
            g2 = torch.stack([g.transpose(1, 2) for g in grads], dim=2).reshape(Bsz * N, 3 * C)
            db = g2.sum(0, dtype=torch.float32)
        dx = _dgrad(g2, wc, ctx.wt).view(xc.shape) if ctx.needs_input_grad[0] else None
        dw = wgrad(g2.t(), xc.reshape(-1, C)) if ctx.needs_input_grad[1] else None
        return dx, dw, db if ctx.needs_input_grad[2] else None, None


def qkv_proj(x, weight, bias, heads):
    return QKVProjFn.apply(x, weight, bias, heads)


# ---------------------------------------------------------------------------- fused short-sequence attention (mc_attn.h)
def attn_supported(seqlen, head_dim, dtype):
    return head_dim == 64 and 1 <= seqlen <= 256 and dtype in (torch.bfloat16, torch.float16)


class PackedAttentionFn(torch.autograd.Function):
    """o = softmax(q k^T / sqrt(D)) v per head, for q / k / v the three C-wide slices of a packed
    (B, N, 3C) projection output (timm Attention's qkv Linear), o as (B, N, C) -- the layout
    the output projection reads.  Forward mc_attn_fwd, backward mc_attn_bwd writing dq / dk / dv
    straight into the packed (B, N, 3C) gradient of the projection output (no stack, no copy)."""

    @staticmethod
    def forward(ctx, qkv, heads):
        Bsz, N, C3 = qkv.shape
        C = C3 // 3
        D = C // heads
        if not (qkv.is_cuda and attn_supported(N, D, qkv.dtype)):
            raise RuntimeError(f"packed_attention: unsupported (device {qkv.device}, N {N}, head_dim {D}, "
                               f"{qkv.dtype}); bf16/f16 on the GPU, head_dim 64, N <= 256")
        lib = _lib.load()
        y = _hip_rows(qkv.reshape(Bsz * N, C3), 8, "packed_attention").view(Bsz, N, C3)
        o = torch.empty(Bsz, N, C, device=qkv.device, dtype=qkv.dtype)
        lse = torch.empty(Bsz, heads, N, device=qkv.device, dtype=torch.float32)
        p = _lib.AttnFwdParams()
        p.batch, p.heads, p.seqlen, p.head_dim, p.dtype = Bsz, heads, N, D, _lib.dtype_code(qkv.dtype)
        p.scale = D ** -0.5
        es = y.element_size()
        p.q, p.k, p.v = y.data_ptr(), y.data_ptr() + C * es, y.data_ptr() + 2 * C * es
        p.q_bs, p.q_ns, p.q_hs = y.stride(0), y.stride(1), D
        p.o, p.o_bs, p.o_ns, p.o_hs = o.data_ptr(), o.stride(0), o.stride(1), D
        p.lse = lse.data_ptr()
        _lib.check(lib.mc_attn_fwd(p, _lib.stream_handle(qkv.device)), "mc_attn_fwd")
        ctx.save_for_backward(y, o, lse)
        ctx.heads = heads
        return o

    @staticmethod
    def backward(ctx, go):
        y, o, lse = ctx.saved_tensors
        Bsz, N, C3 = y.shape
        C = C3 // 3
        D = C // ctx.heads
        lib = _lib.load()
        g = _hip_rows(go.to(o.dtype).reshape(Bsz * N, C), 8, "packed_attention backward").view(Bsz, N, C)
        dy = torch.empty_like(y)
        p = _lib.AttnBwdParams()
        p.batch, p.heads, p.seqlen, p.head_dim, p.dtype = Bsz, ctx.heads, N, D, _lib.dtype_code(y.dtype)
        p.scale = D ** -0.5
        es = y.element_size()
        p.q, p.k, p.v = y.data_ptr(), y.data_ptr() + C * es, y.data_ptr() + 2 * C * es
        p.q_bs, p.q_ns, p.q_hs = y.stride(0), y.stride(1), D
        if g.stride() != o.stride():
            raise RuntimeError("packed_attention backward: dout and o layouts differ")
        p.o, p.dout, p.o_bs, p.o_ns, p.o_hs = o.data_ptr(), g.data_ptr(), o.stride(0), o.stride(1), D
        p.lse = lse.data_ptr()
        p.dq, p.dk, p.dv = dy.data_ptr(), dy.data_ptr() + C * es, dy.data_ptr() + 2 * C * es
        p.dq_bs, p.dq_ns, p.dq_hs = dy.stride(0), dy.stride(1), D
        # per-batch column sums of dq | dk | dv, taken in the kernel: the qkv bias gradient rides on dy
        # (LinearSK picks it up instead of a second pass over the (B*N, 3C) gradient)
        dsum = torch.empty(Bsz, 3 * C, device=y.device, dtype=torch.float32)
        p.dsum = dsum.data_ptr()
        _lib.check(lib.mc_attn_bwd(p, _lib.stream_handle(y.device)), "mc_attn_bwd")
        setattr(dy, COLSUM_ATTR, (sum_rows(dsum), dy._version))
        return dy, None


def packed_attention(qkv, heads):
    return PackedAttentionFn.apply(qkv, heads)


# ---------------------------------------------------------------------------- SS2D cross-scan glue (mc_ss2d.h)
def _cl_ok(t):
    """Channels-last view the SS2D kernels take as is: unit channel stride, 4-element aligned."""
    return (t.stride(-1) == 1 and t.shape[-1] % 4 == 0 and all(s % 4 == 0 for s in t.stride()[:3])
            and t.data_ptr() % (4 * t.element_size()) == 0)


class SS2DConvStackFn(torch.autograd.Function):
    """u = [x, x^T] of SS2D's cross-scan, fp32 (B, 2, C, H*W), from the channels-last in_proj half:
    silu(depthwise conv3x3(x) + b) written in both frames by one kernel (reference model.py:636-637
    permute + conv2d + SiLU, 510-517 stack / transpose, 531-537 fp32 cast)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        if not x.is_cuda:
            raise RuntimeError("ss2d_conv_stack: CUDA tensors only (the CPU restatement lives in oracle/)")
        Bsz, H, W, C = x.shape
        k = weight.shape[-1]
        xs = x if _cl_ok(x) else x.contiguous()
        w32 = weight.float().contiguous()
        b32 = bias.float().contiguous() if bias is not None else None
        u = torch.empty(Bsz, 2, C, H * W, device=x.device, dtype=torch.float32)
        p = _lib.SS2DConvParams()
        p.batch, p.height, p.width, p.channels, p.ksize = Bsz, H, W, C, k
        p.xtype = _lib.dtype_code(xs.dtype)
        p.x_batch_stride, p.x_row_stride, p.x_col_stride = xs.stride(0), xs.stride(1), xs.stride(2)
        p.x, p.weight, p.bias, p.u = xs.data_ptr(), w32.data_ptr(), _lib.ptr(b32), u.data_ptr()
        _lib.check(_lib.load().mc_ss2d_conv_stack_fwd(ctypes.byref(p), _lib.stream_handle(x.device)),
                   "mc_ss2d_conv_stack_fwd")
        ctx.save_for_backward(xs, w32, b32)
        ctx.dtypes = (weight.dtype, bias.dtype if bias is not None else None)
        return u

    @staticmethod
    def backward(ctx, du):
        xs, w32, b32 = ctx.saved_tensors
        Bsz, H, W, C = xs.shape
        k = w32.shape[-1]
        du = du.float().contiguous()
        dx = torch.empty(Bsz, H, W, C, device=xs.device, dtype=xs.dtype)
        dw = torch.empty_like(w32)
        db = torch.empty(C, device=xs.device, dtype=torch.float32) if b32 is not None else None
        lib = _lib.load()
        ws_b = lib.mc_ss2d_conv_bwd_workspace_bytes(Bsz, H, W, C, k)
        ws = _ws(ws_b, xs.device)
        p = _lib.SS2DConvBwdParams()
        f = p.fwd
        f.batch, f.height, f.width, f.channels, f.ksize = Bsz, H, W, C, k
        f.xtype = _lib.dtype_code(xs.dtype)
        f.x_batch_stride, f.x_row_stride, f.x_col_stride = xs.stride(0), xs.stride(1), xs.stride(2)
        f.x, f.weight, f.bias = xs.data_ptr(), w32.data_ptr(), _lib.ptr(b32)
        p.du, p.dx, p.dweight, p.dbias = du.data_ptr(), dx.data_ptr(), dw.data_ptr(), _lib.ptr(db)
        p.workspace, p.workspace_bytes = ws.data_ptr(), ws_b
        _lib.check(lib.mc_ss2d_conv_stack_bwd(ctypes.byref(p), _lib.stream_handle(xs.device)), "mc_ss2d_conv_stack_bwd")
        wdt, bdt = ctx.dtypes
        return dx, dw.to(wdt), db.to(bdt) if db is not None else None


def ss2d_conv_stack(x, weight, bias):
    return SS2DConvStackFn.apply(x, weight, bias)


def _group_proj(w, wstr, x, xstr, y, ystr, B, G, M, Nn, L, mod=None, acc=None, astr=None):
    """One mc_ss2d_group_proj launch: Y[b,g,m,l] = A + sum_n W[g,m,n] X[b,g % mod,n,l] (fp32).
    wstr = (g, m, n) strides of W; xstr = (b, g, n) of X; ystr / astr = (b, g, m) of Y / A."""
    p = _lib.SS2DGroupProjParams()
    p.batch, p.groups, p.rows_out, p.rows_in, p.seqlen = B, G, M, Nn, L
    p.x_group_mod = mod or G
    p.w, (p.w_gs, p.w_ms, p.w_ns) = w.data_ptr(), wstr
    p.x, (p.x_bs, p.x_gs, p.x_ns) = x.data_ptr(), xstr
    if acc is not None:
        p.acc, (p.a_bs, p.a_gs, p.a_ms) = acc.data_ptr(), astr
    p.y, (p.y_bs, p.y_gs, p.y_ms) = y.data_ptr(), ystr
    _lib.check(_lib.load().mc_ss2d_group_proj(ctypes.byref(p), _lib.stream_handle(y.device)), "mc_ss2d_group_proj")


def ss2d_proj_ok(u, w_x, w_dt):
    """Shapes / dtypes SS2DProjFn takes: fp32 CUDA u (B, 2, d, L) contiguous, fp32 weights."""
    return (u.is_cuda and u.dtype == torch.float32 and u.dim() == 4 and u.shape[1] == 2 and u.is_contiguous()
            and w_x.dtype == torch.float32 and w_dt.dtype == torch.float32 and w_x.shape[0] == 4
            and w_x.shape[2] == u.shape[2] and w_dt.shape[1] == u.shape[2] and u.shape[2] <= 4096)


class SS2DProjFn(torch.autograd.Function):
    """SS2D's per-direction projections (reference model.py:519-528, in fp32 as model.py:531-537): with
    u = [x, x^T] (B, 2, d, L) holding the two frames and direction k = 2 i + j reading frame j,
        x_dbl[b,k] = x_proj[k] u[b, j]      (c = R + 2N rows: dt, B, C)
        delta[b,k] = dt_proj[k] x_dbl[b,k,:R]
    on mc_ss2d_group_proj -- no permuted operand copies (torch.einsum made ~10 elementwise copies and
    tiny-K library GEMMs around them).  Backward: d(dt rows) and du on the same kernel (du as
    two in-order passes over i), the weight gradients as batched GEMMs over L summed over the batch in a
    fixed order (ops.colsum).  Returns (delta, B rows, C rows) as (B, 4, ., L) views / tensors."""

    @staticmethod
    def forward(ctx, u, w_x, w_dt, R, N):
        Bsz, _, d, L = u.shape
        c = R + 2 * N
        wx, wdt = w_x.contiguous(), w_dt.contiguous()
        x_dbl = torch.empty(Bsz, 4, c, L, device=u.device, dtype=torch.float32)
        delta = torch.empty(Bsz, 4, d, L, device=u.device, dtype=torch.float32)
        # weights with the output row contiguous (one 64-B scalar load per n and 16 rows): [k][n][m]
        wx_t = wx.transpose(1, 2).contiguous()
        wdt_t = wdt.transpose(1, 2).contiguous()
        _group_proj(wx_t, (c * d, 1, c), u, (2 * d * L, d * L, L), x_dbl, (4 * c * L, c * L, L), Bsz, 4, c, d, L, mod=2)
        _group_proj(wdt_t, (d * R, 1, d), x_dbl, (4 * c * L, c * L, L), delta, (4 * d * L, d * L, L), Bsz, 4, d, R, L)
        ctx.save_for_backward(u, wx, wdt, x_dbl)
        ctx.rn = (R, N)
        return delta, x_dbl[:, :, R:R + N], x_dbl[:, :, R + N:]

    @staticmethod
    def backward(ctx, g_delta, g_B, g_C):
        u, wx, wdt, x_dbl = ctx.saved_tensors
        R, N = ctx.rn
        Bsz, _, d, L = u.shape
        c = R + 2 * N
        dx = torch.empty(Bsz, 4, c, L, device=u.device, dtype=torch.float32)
        wx_p, wdt_p = wx, wdt   # [k][c][d] / [k][d][R]: already output-row contiguous here
        if g_delta is None:
            dx[:, :, :R].zero_()
            g_delta = torch.zeros(Bsz, 4, d, L, device=u.device, dtype=torch.float32)
        else:
            g_delta = g_delta.float().contiguous()
            # d(dt rows)[b,k] = dt_proj[k]^T ddelta[b,k]
            _group_proj(wdt_p, (d * R, 1, R), g_delta, (4 * d * L, d * L, L), dx, (4 * c * L, c * L, L), Bsz, 4, R, d, L)
        for off, g in ((R, g_B), (R + N, g_C)):
            if g is None:
                dx[:, :, off:off + N].zero_()
            else:
                dx[:, :, off:off + N].copy_(g)
        # du[b,j] = x_proj[j]^T dx[b,j] + x_proj[2+j]^T dx[b,2+j]: two passes, the second accumulating in place
        du = torch.empty_like(u)
        _group_proj(wx_p, (c * d, 1, d), dx, (4 * c * L, c * L, L), du, (2 * d * L, d * L, L), Bsz, 2, d, c, L)
        _group_proj(wx_p[2:], (c * d, 1, d), dx[:, 2:], (4 * c * L, c * L, L), du, (2 * d * L, d * L, L), Bsz, 2,
                    d, c, L, acc=du, astr=(2 * d * L, d * L, L))
        # weight gradients: per-batch GEMMs over L, summed over the batch in a fixed order
        dwx = torch.matmul(dx.view(Bsz, 2, 2, c, L), u.transpose(-1, -2).unsqueeze(1))   # [b][i][j] (k = 2 i + j)
        dwx = colsum(dwx.reshape(Bsz, 4 * c * d)).view(4, c, d)
        dwdt = torch.matmul(g_delta, x_dbl[:, :, :R].transpose(-1, -2))          # (B, 4, d, R)
        dwdt = colsum(dwdt.reshape(Bsz, 4 * d * R)).view(4, d, R)
        return du, dwx, dwdt, None, None


def ss2d_proj(u, w_x, w_dt, R, N):
    return SS2DProjFn.apply(u, w_x, w_dt, R, N)


class SS2DMergeFn(torch.autograd.Function):
    """y = LayerNorm(((y1 + y2) + y3) + y4) * silu(z), channels-last, from the grouped scan's
    (B, 4C, H*W) fp32 output (directions 1 / 3 in the x^T frame) -- reference model.py:553-565 flips /
    transposes and 640-643 sum, transpose, out_norm, gate -- in one kernel; the backward writes each
    direction's output gradient in its own frame, dz and the LayerNorm parameter gradients."""

    @staticmethod
    def forward(ctx, out, z, ln_w, ln_b, eps, y_dtype):
        if not out.is_cuda:
            raise RuntimeError("ss2d_merge_ln_gate: CUDA tensors only (the CPU restatement lives in oracle/)")
        Bsz, H, W, C = z.shape
        o = out.float().contiguous()
        zs = z if _cl_ok(z) else z.contiguous()
        lw = ln_w.float().contiguous()
        lb = ln_b.float().contiguous() if ln_b is not None else None
        y = torch.empty(Bsz, H, W, C, device=out.device, dtype=y_dtype)
        mean = torch.empty(Bsz * H * W, device=out.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        p = _lib.SS2DMergeParams()
        _merge_params(p, o, zs, lw, lb, eps, y_dtype, mean, rstd)
        p.y = y.data_ptr()
        _lib.check(_lib.load().mc_ss2d_merge_ln_gate_fwd(ctypes.byref(p), _lib.stream_handle(out.device)),
                   "mc_ss2d_merge_ln_gate_fwd")
        ctx.save_for_backward(o, zs, lw, lb, mean, rstd)
        ctx.cfg = (eps, y_dtype, z.dtype, ln_w.dtype, ln_b.dtype if ln_b is not None else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        o, zs, lw, lb, mean, rstd = ctx.saved_tensors
        eps, y_dtype, z_dt, lw_dt, lb_dt = ctx.cfg
        Bsz, H, W, C = zs.shape
        dy = dy.to(y_dtype)
        if not _cl_ok(dy):
            dy = dy.contiguous()
        dout = torch.empty_like(o)
        dz = torch.empty(Bsz, H, W, C, device=zs.device, dtype=zs.dtype)
        dlw = torch.empty_like(lw)
        dlb = torch.empty_like(lb) if lb is not None else None
        lib = _lib.load()
        ws_b = lib.mc_ss2d_merge_bwd_workspace_bytes(Bsz, H, W, C)
        ws = _ws(ws_b, zs.device)
        p = _lib.SS2DMergeBwdParams()
        _merge_params(p.fwd, o, zs, lw, lb, eps, y_dtype, mean, rstd)
        p.dy = dy.data_ptr()
        p.dy_batch_stride, p.dy_row_stride, p.dy_col_stride = dy.stride(0), dy.stride(1), dy.stride(2)
        p.dout, p.dz, p.dln_weight, p.dln_bias = dout.data_ptr(), dz.data_ptr(), dlw.data_ptr(), _lib.ptr(dlb)
        p.workspace, p.workspace_bytes = ws.data_ptr(), ws_b
        _lib.check(lib.mc_ss2d_merge_ln_gate_bwd(ctypes.byref(p), _lib.stream_handle(zs.device)),
                   "mc_ss2d_merge_ln_gate_bwd")
        return (dout, dz.to(z_dt), dlw.to(lw_dt), dlb.to(lb_dt) if dlb is not None else None, None, None)


def _merge_params(p, o, zs, lw, lb, eps, y_dtype, mean, rstd):
    Bsz, H, W, C = zs.shape
    p.batch, p.height, p.width, p.channels = Bsz, H, W, C
    p.ztype, p.ytype, p.eps = _lib.dtype_code(zs.dtype), _lib.dtype_code(y_dtype), float(eps)
    p.out, p.z = o.data_ptr(), zs.data_ptr()
    p.z_batch_stride, p.z_row_stride, p.z_col_stride = zs.stride(0), zs.stride(1), zs.stride(2)
    p.ln_weight, p.ln_bias = lw.data_ptr(), _lib.ptr(lb)
    p.mean, p.rstd = mean.data_ptr(), rstd.data_ptr()


def ss2d_merge_ln_gate(out, z, ln_weight, ln_bias, eps):
    """out (B, 4C, H*W) fp32, z (B, H, W, C) channels-last -> (B, H, W, C): fp32 like the reference's
    LayerNorm output, or the autocast dtype under autocast (the value out_proj's cast would give)."""
    y_dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else torch.float32
    return SS2DMergeFn.apply(out, z, ln_weight, ln_bias, eps, y_dtype)
