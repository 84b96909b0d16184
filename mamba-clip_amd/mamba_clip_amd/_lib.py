"""ctypes binding of libmamba_clip_amd.so (the C ABI declared in include/*.h).

The product path has NO fallback: if the HIP library is missing or fails to
load, importing any op raises.  Build it with
``make -C mamba-clip_amd`` (or ``python -c "import __graft_entry__ as g; g.build()"``).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MAMBA_CLIP_AMD_LIB overrides the path (dev A/B builds only)
LIB_PATH = os.environ.get("MAMBA_CLIP_AMD_LIB") or os.path.join(_HERE, "libmamba_clip_amd.so")

MC_DTYPE_F32, MC_DTYPE_BF16, MC_DTYPE_F16, MC_DTYPE_FP8_E4M3, MC_DTYPE_U8 = 0, 1, 2, 3, 4
MC_LAYOUT_NCHW, MC_LAYOUT_NHWC = 0, 1
MC_SCAN_CHUNK = 32
MC_SCAN_STATE_INTERVAL_FINE = 8
MC_SCAN_KERNEL_NONE, MC_SCAN_KERNEL_PAIR, MC_SCAN_KERNEL_GENERIC, MC_SCAN_KERNEL_DIRS = 0, 1, 2, 3
MC_GEMM_KERNEL_TILE, MC_GEMM_KERNEL_FP8_TILE, MC_GEMM_KERNEL_FP8_PANEL = 1, 2, 3   # mc_gemm_nt_kernel
MC_SCAN_MAX_DSTATE = 32
MC_CAST_CHUNK = 16384

c_i32, c_i64, c_vp, c_fp = ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p


class ScanFwdParams(ctypes.Structure):
    """Mirror of ``mc_scan_fwd_params`` (include/mc_scan.h)."""
    _fields_ = [
        ("batch", c_i32), ("dim", c_i32), ("seqlen", c_i32), ("dstate", c_i32), ("n_groups", c_i32),
        ("itype", c_i32), ("wtype", c_i32), ("delta_softplus", c_i32),
        ("u_batch_stride", c_i64), ("u_dim_stride", c_i64),
        ("delta_batch_stride", c_i64), ("delta_dim_stride", c_i64),
        ("z_batch_stride", c_i64), ("z_dim_stride", c_i64),
        ("out_batch_stride", c_i64), ("out_dim_stride", c_i64),
        ("B_batch_stride", c_i64), ("B_group_stride", c_i64), ("B_dstate_stride", c_i64),
        ("C_batch_stride", c_i64), ("C_group_stride", c_i64), ("C_dstate_stride", c_i64),
        ("u", c_vp), ("delta", c_vp), ("A", c_fp), ("B", c_vp), ("C", c_vp),
        ("D", c_fp), ("z", c_vp), ("delta_bias", c_fp),
        ("out", c_vp), ("chunk_states", c_fp), ("last_state", c_fp),
        ("workspace", c_vp), ("workspace_bytes", ctypes.c_size_t),
        ("out_y", c_vp), ("out_y_batch_stride", c_i64), ("out_y_dim_stride", c_i64),
        ("reverse_groups", c_i32), ("u_groups", c_i32),
        ("delta_proj_x", c_vp), ("delta_proj_w", c_vp), ("delta_rank", c_i32),
        ("dpx_batch_stride", c_i64), ("dpx_token_stride", c_i64), ("dpw_dim_stride", c_i64),
        ("delta_out", c_vp), ("state_interval", c_i32),
    ]


class ScanBwdParams(ctypes.Structure):
    """Mirror of ``mc_scan_bwd_params`` (include/mc_scan.h)."""
    _fields_ = [
        ("batch", c_i32), ("dim", c_i32), ("seqlen", c_i32), ("dstate", c_i32), ("n_groups", c_i32),
        ("itype", c_i32), ("wtype", c_i32), ("delta_softplus", c_i32),
        ("u_batch_stride", c_i64), ("u_dim_stride", c_i64),
        ("delta_batch_stride", c_i64), ("delta_dim_stride", c_i64),
        ("z_batch_stride", c_i64), ("z_dim_stride", c_i64),
        ("dout_batch_stride", c_i64), ("dout_dim_stride", c_i64),
        ("du_batch_stride", c_i64), ("du_dim_stride", c_i64),
        ("ddelta_batch_stride", c_i64), ("ddelta_dim_stride", c_i64),
        ("dz_batch_stride", c_i64), ("dz_dim_stride", c_i64),
        ("B_batch_stride", c_i64), ("B_group_stride", c_i64), ("B_dstate_stride", c_i64),
        ("C_batch_stride", c_i64), ("C_group_stride", c_i64), ("C_dstate_stride", c_i64),
        ("u", c_vp), ("delta", c_vp), ("A", c_fp), ("B", c_vp), ("C", c_vp),
        ("D", c_fp), ("z", c_vp), ("delta_bias", c_fp), ("dout", c_vp), ("chunk_states", c_fp),
        ("du", c_vp), ("ddelta", c_vp), ("dz", c_vp), ("dB", c_vp), ("dC", c_vp),
        ("dA", c_fp), ("dD", c_fp), ("ddelta_bias", c_fp),
        ("workspace", c_vp), ("workspace_bytes", ctypes.c_size_t),
        ("out_y", c_vp), ("out_y_batch_stride", c_i64), ("out_y_dim_stride", c_i64),
        ("reverse_groups", c_i32), ("u_groups", c_i32),
        ("delta_proj_x", c_vp), ("delta_proj_w", c_vp), ("delta_rank", c_i32),
        ("dpx_batch_stride", c_i64), ("dpx_token_stride", c_i64), ("dpw_dim_stride", c_i64),
        ("state_interval", c_i32),
        ("dB_batch_stride", c_i64), ("dB_group_stride", c_i64), ("dB_dstate_stride", c_i64),
        ("dC_batch_stride", c_i64), ("dC_group_stride", c_i64), ("dC_dstate_stride", c_i64),
    ]


MC_ADAMW_MAX_GROUPS = 8
MC_ADAMW_CHUNK = 65536


class AdamWGroup(ctypes.Structure):
    """Mirror of ``mc_adamw_group`` (include/mc_ops.h)."""
    _fields_ = [("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float), ("decay", ctypes.c_float),
                ("step_size", ctypes.c_float), ("bc2_sqrt", ctypes.c_float)]


class AdamWHyper(ctypes.Structure):
    """Mirror of ``mc_adamw_hyper`` (include/mc_ops.h)."""
    _fields_ = [("n_groups", ctypes.c_int32), ("reserved", ctypes.c_int32), ("group", AdamWGroup * MC_ADAMW_MAX_GROUPS)]


class MixerProjParams(ctypes.Structure):
    """Mirror of ``mc_mixer_proj_params`` (include/mc_ops.h)."""
    _fields_ = [
        ("dim", c_i32), ("tokens", c_i32), ("rank", c_i32), ("proj_rows", c_i32), ("dtype", c_i32),
        ("x_ld", c_i64), ("x_dbl_ld", c_i64), ("delta_ld", c_i64),
        ("x", c_vp), ("w_x", c_vp), ("w_dt", c_vp), ("x_dbl", c_vp), ("delta", c_vp),
    ]


class MixerProjBwdParams(ctypes.Structure):
    """Mirror of ``mc_mixer_proj_bwd_params`` (include/mc_ops.h)."""
    _fields_ = [
        ("dim", c_i32), ("tokens", c_i32), ("rank", c_i32), ("proj_rows", c_i32), ("dtype", c_i32),
        ("g_delta_ld", c_i64), ("g_b_ld", c_i64), ("g_c_ld", c_i64), ("du_ld", c_i64), ("d_x_dbl_ld", c_i64),
        ("dx_ld", c_i64),
        ("g_delta", c_vp), ("g_b", c_vp), ("g_c", c_vp), ("w_x", c_vp), ("w_dt", c_vp), ("du", c_vp),
        ("d_x_dbl", c_vp), ("dx", c_vp),
    ]


class GemmNTParams(ctypes.Structure):
    """Mirror of ``mc_gemm_nt_params`` (include/mc_contrastive.h)."""
    _fields_ = [
        ("M", c_i32), ("N", c_i32), ("K", c_i32), ("in_dtype", c_i32), ("out_dtype", c_i32),
        ("A", c_vp), ("lda", c_i64), ("B", c_vp), ("ldb", c_i64), ("C", c_vp), ("ldc", c_i64),
        ("alpha", ctypes.c_float), ("alpha_dev", c_fp),
        ("row_scale_a", c_fp), ("row_scale_b", c_fp),
    ]


class CEFusedParams(ctypes.Structure):
    """Mirror of ``mc_ce_fused_params`` (include/mc_contrastive.h)."""
    _fields_ = [
        ("M", c_i32), ("N", c_i32), ("K", c_i32), ("in_dtype", c_i32),
        ("X", c_vp), ("ldx", c_i64), ("Y", c_vp), ("ldy", c_i64),
        ("row_scale_x", c_fp), ("row_scale_y", c_fp),
        ("scale", ctypes.c_float), ("scale_dev", c_fp),
        ("row_off", c_i64), ("coef_r", ctypes.c_float), ("col_off", c_i64), ("coef_c", ctypes.c_float),
        ("lse_r", c_fp), ("lse_c", c_fp), ("loss_out", c_fp), ("gout_dev", c_fp),
        ("g_dtype", c_i32), ("g_times_scale", c_i32), ("G", c_vp), ("ldg", c_i64),
        ("dscale_out", c_fp), ("workspace", c_vp), ("workspace_bytes", ctypes.c_size_t),
    ]


class QkvPackParams(ctypes.Structure):
    """Mirror of ``mc_qkv_pack_params`` (include/mc_ops.h)."""
    _fields_ = [
        ("batch", c_i32), ("seq", c_i32), ("heads", c_i32), ("head_dim", c_i32), ("dtype", c_i32),
        ("src", c_vp * 3), ("sb", c_i64 * 3), ("sn", c_i64 * 3), ("sh", c_i64 * 3),
        ("out", c_vp), ("ld_out", c_i64), ("dbias", c_fp), ("workspace", c_vp), ("workspace_bytes", ctypes.c_size_t),
    ]


class AttnFwdParams(ctypes.Structure):
    """Mirror of ``mc_attn_fwd_params`` (include/mc_attn.h)."""
    _fields_ = [
        ("batch", c_i32), ("heads", c_i32), ("seqlen", c_i32), ("head_dim", c_i32), ("dtype", c_i32),
        ("scale", ctypes.c_float),
        ("q", c_vp), ("k", c_vp), ("v", c_vp), ("q_bs", c_i64), ("q_ns", c_i64), ("q_hs", c_i64),
        ("o", c_vp), ("o_bs", c_i64), ("o_ns", c_i64), ("o_hs", c_i64), ("lse", c_fp),
    ]


class AttnBwdParams(ctypes.Structure):
    """Mirror of ``mc_attn_bwd_params`` (include/mc_attn.h)."""
    _fields_ = [
        ("batch", c_i32), ("heads", c_i32), ("seqlen", c_i32), ("head_dim", c_i32), ("dtype", c_i32),
        ("scale", ctypes.c_float),
        ("q", c_vp), ("k", c_vp), ("v", c_vp), ("q_bs", c_i64), ("q_ns", c_i64), ("q_hs", c_i64),
        ("o", c_vp), ("dout", c_vp), ("o_bs", c_i64), ("o_ns", c_i64), ("o_hs", c_i64), ("lse", c_fp),
        ("dq", c_vp), ("dk", c_vp), ("dv", c_vp), ("dq_bs", c_i64), ("dq_ns", c_i64), ("dq_hs", c_i64),
        ("dsum", c_fp),
    ]


class SS2DConvParams(ctypes.Structure):
    """Mirror of ``mc_ss2d_conv_params`` (include/mc_ss2d.h)."""
    _fields_ = [
        ("batch", c_i32), ("height", c_i32), ("width", c_i32), ("channels", c_i32), ("ksize", c_i32),
        ("xtype", c_i32), ("x_batch_stride", c_i64), ("x_row_stride", c_i64), ("x_col_stride", c_i64),
        ("x", c_vp), ("weight", c_fp), ("bias", c_fp), ("u", c_fp),
    ]


class SS2DConvBwdParams(ctypes.Structure):
    """Mirror of ``mc_ss2d_conv_bwd_params`` (include/mc_ss2d.h)."""
    _fields_ = [
        ("fwd", SS2DConvParams), ("du", c_fp), ("dx", c_vp), ("dweight", c_fp), ("dbias", c_fp),
        ("workspace", c_vp), ("workspace_bytes", ctypes.c_size_t),
    ]


class SS2DMergeParams(ctypes.Structure):
    """Mirror of ``mc_ss2d_merge_params`` (include/mc_ss2d.h)."""
    _fields_ = [
        ("batch", c_i32), ("height", c_i32), ("width", c_i32), ("channels", c_i32),
        ("ztype", c_i32), ("ytype", c_i32), ("eps", ctypes.c_float),
        ("out", c_fp), ("z", c_vp), ("z_batch_stride", c_i64), ("z_row_stride", c_i64), ("z_col_stride", c_i64),
        ("ln_weight", c_fp), ("ln_bias", c_fp), ("y", c_vp), ("mean", c_fp), ("rstd", c_fp),
    ]


class SS2DGroupProjParams(ctypes.Structure):
    """Mirror of ``mc_ss2d_group_proj_params`` (include/mc_ss2d.h)."""
    _fields_ = [
        ("batch", c_i32), ("groups", c_i32), ("rows_out", c_i32), ("rows_in", c_i32), ("seqlen", c_i32),
        ("x_group_mod", c_i32),
        ("w", c_fp), ("w_gs", c_i64), ("w_ms", c_i64), ("w_ns", c_i64),
        ("x", c_fp), ("x_bs", c_i64), ("x_gs", c_i64), ("x_ns", c_i64),
        ("acc", c_fp), ("a_bs", c_i64), ("a_gs", c_i64), ("a_ms", c_i64),
        ("y", c_fp), ("y_bs", c_i64), ("y_gs", c_i64), ("y_ms", c_i64),
    ]


class SS2DMergeBwdParams(ctypes.Structure):
    """Mirror of ``mc_ss2d_merge_bwd_params`` (include/mc_ss2d.h)."""
    _fields_ = [
        ("fwd", SS2DMergeParams), ("dy", c_vp),
        ("dy_batch_stride", c_i64), ("dy_row_stride", c_i64), ("dy_col_stride", c_i64),
        ("dout", c_fp), ("dz", c_vp), ("dln_weight", c_fp), ("dln_bias", c_fp),
        ("workspace", c_vp), ("workspace_bytes", ctypes.c_size_t),
    ]


MC_WGRAD_TOKEN_MAJOR, MC_WGRAD_FEATURE_MAJOR = 0, 1


class WgradParams(ctypes.Structure):
    """Mirror of ``mc_wgrad_params`` (include/mc_gemm.h)."""
    _fields_ = [
        ("M", c_i32), ("N", c_i32), ("T", c_i32), ("dtype", c_i32), ("a_layout", c_i32), ("b_layout", c_i32),
        ("A", c_vp), ("lda", c_i64), ("B", c_vp), ("ldb", c_i64), ("C", c_vp), ("ldc", c_i64),
        ("splits", c_i32), ("reserved", c_i32), ("workspace", c_vp), ("workspace_bytes", ctypes.c_size_t),
    ]


MC_LINEAR_EPI_NONE, MC_LINEAR_EPI_BIAS, MC_LINEAR_EPI_BIAS_GELU, MC_LINEAR_EPI_GELU_GRAD = 0, 1, 2, 3


class LinearParams(ctypes.Structure):
    """Mirror of ``mc_linear_params`` (include/mc_gemm.h)."""
    _fields_ = [
        ("rows", c_i32), ("cols", c_i32), ("K", c_i32), ("dtype", c_i32), ("epilogue", c_i32), ("reserved", c_i32),
        ("X", c_vp), ("ldx", c_i64), ("W", c_vp), ("ldw", c_i64), ("Y", c_vp), ("ldy", c_i64),
        ("Y2", c_vp), ("ldy2", c_i64), ("bias", c_vp), ("H", c_vp), ("ldh", c_i64), ("colsum", c_vp),
        ("workspace", c_vp), ("workspace_bytes", ctypes.c_size_t),
    ]


class PatchInputParams(ctypes.Structure):
    """Mirror of ``mc_patch_input_params`` (include/mc_ops.h)."""
    _fields_ = [
        ("batch", c_i32), ("channels", c_i32), ("height", c_i32), ("width", c_i32), ("patch", c_i32),
        ("layout", c_i32), ("in_dtype", c_i32), ("out_dtype", c_i32),
        ("img", c_vp), ("scale", c_fp), ("shift", c_fp), ("out", c_vp),
    ]


# symbol -> (restype, argtypes); every entry point include/*.h declares
SYMBOLS = {
    "mc_last_error": (ctypes.c_char_p, []),
    "mc_version": (ctypes.c_char_p, []),
    "mc_scan_n_chunks": (c_i32, [c_i32]),
    "mc_scan_n_states": (c_i32, [c_i32, c_i32]),
    "mc_scan_fwd_state_interval": (c_i32, [ctypes.POINTER(ScanFwdParams)]),
    "mc_scan_fwd_kernel": (c_i32, [ctypes.POINTER(ScanFwdParams)]),
    "mc_gemm_wgrad_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(WgradParams)]),
    "mc_gemm_wgrad": (ctypes.c_int, [ctypes.POINTER(WgradParams), c_vp]),
    "mc_linear_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(LinearParams)]),
    "mc_linear": (ctypes.c_int, [ctypes.POINTER(LinearParams), c_vp]),
    "mc_gemm_small_k": (ctypes.c_int, [c_i32, c_i32, c_i32, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "mc_gemm_skinny_m": (ctypes.c_int, [c_i32, c_i32, c_i32, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "mc_scan_bwd_kernel": (c_i32, [ctypes.POINTER(ScanBwdParams)]),
    "mc_scan_chunk_states_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32, c_i32]),
    "mc_scan_fwd_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32, c_i32]),
    "mc_scan_bwd_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32, c_i32, c_i32]),
    "mc_scan_fwd": (ctypes.c_int, [ctypes.POINTER(ScanFwdParams), c_vp]),
    "mc_scan_bwd": (ctypes.c_int, [ctypes.POINTER(ScanBwdParams), c_vp]),
    "mc_gemm_nt": (ctypes.c_int, [ctypes.POINTER(GemmNTParams), c_vp]),
    "mc_gemm_nt_kernel": (c_i32, [ctypes.POINTER(GemmNTParams)]),
    "mc_quant_rows_fp8": (ctypes.c_int, [c_i32, c_i32, c_i32, c_vp, c_i64, c_vp, c_i64, c_fp, c_vp]),
    "mc_ce_stats": (ctypes.c_int, [c_i32, c_i32, c_fp, c_i64, c_i32, c_i64, c_fp, c_fp, ctypes.c_float, c_fp,
                                   c_vp, ctypes.c_size_t, c_vp]),
    "mc_ce_stats_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32]),
    "mc_ce_grad": (ctypes.c_int, [c_i32, c_i32, c_fp, c_i64, c_fp, c_i64, ctypes.c_float, c_fp, c_i64,
                                  ctypes.c_float, c_fp, c_i32, c_vp, c_i64, c_fp, c_fp, c_vp, ctypes.c_size_t, c_vp]),
    "mc_ce_grad_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32]),
    "mc_ce_fused_fwd": (ctypes.c_int, [ctypes.POINTER(CEFusedParams), c_vp]),
    "mc_ce_fused_fwd_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32]),
    "mc_ce_fused_grad": (ctypes.c_int, [ctypes.POINTER(CEFusedParams), c_vp]),
    "mc_ce_fused_grad_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32]),
    "mc_add_rmsnorm_fwd": (ctypes.c_int, [c_i32, c_i32, c_i32, c_vp, c_fp, c_fp, ctypes.c_float, c_vp, c_fp, c_fp,
                                          c_vp]),
    "mc_add_rmsnorm_bwd": (ctypes.c_int, [c_i32, c_i32, c_i32, c_vp, c_fp, c_fp, c_fp, c_fp, c_vp, c_fp, c_fp, c_vp,
                                          ctypes.c_size_t, c_vp]),
    "mc_add_rmsnorm_bwd_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32]),
    "mc_add_layernorm_fwd": (ctypes.c_int, [c_i32, c_i32, c_i32, c_vp, c_vp, c_fp, c_fp, ctypes.c_float, c_vp, c_vp,
                                            c_fp, c_fp, c_vp]),
    "mc_add_layernorm_bwd": (ctypes.c_int, [c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_fp, c_fp, c_fp, c_vp, c_fp, c_fp,
                                            c_fp, c_vp, ctypes.c_size_t, c_vp]),
    "mc_add_layernorm_bwd_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32]),
    "mc_causal_conv1d_fwd": (ctypes.c_int, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_i64, c_i64, c_fp, c_fp, c_i32,
                                            c_vp, c_i64, c_i64, c_vp]),
    "mc_causal_conv1d_bwd": (ctypes.c_int, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_i64, c_i64, c_fp, c_fp, c_i32,
                                            c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_fp, c_fp, c_vp,
                                            ctypes.c_size_t, c_vp]),
    "mc_causal_conv1d_bwd_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32, c_i32]),
    "mc_patch_im2col": (ctypes.c_int, [c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp]),
    "mc_grad_colsum_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32]),
    "mc_gelu_bwd": (ctypes.c_int, [c_i32, c_i32, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_fp, c_vp,
                                   ctypes.c_size_t, c_vp]),
    "mc_qkv_grad_pack": (ctypes.c_int, [ctypes.POINTER(QkvPackParams), c_vp]),
    "mc_stream_copy": (ctypes.c_int, [c_vp, c_vp, ctypes.c_size_t, c_vp]),
    "mc_cast_f32_many": (ctypes.c_int, [c_i32, c_vp, c_vp, c_i32, c_vp]),
    "mc_cast_transpose_f32_many": (ctypes.c_int, [c_i32, c_vp, c_vp, c_i32, c_vp]),
    "mc_adamw_step": (ctypes.c_int, [c_i32, c_vp, c_vp, ctypes.POINTER(AdamWHyper), c_vp]),
    "mc_sum_slabs": (ctypes.c_int, [c_i32, c_i64, c_fp, c_i64, c_fp, c_vp]),
    "mc_colsum_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32]),
    "mc_colsum_fold": (ctypes.c_int, [c_i32, c_i32, c_fp, c_fp, c_vp]),
    "mc_colsum": (ctypes.c_int, [c_i32, c_i32, c_i32, c_vp, c_i64, c_fp, c_vp, ctypes.c_size_t, c_vp]),
    "mc_l2norm_fwd": (ctypes.c_int, [c_i32, c_i32, c_i32, c_vp, c_i64, ctypes.c_float, c_fp, c_i64, c_fp, c_vp]),
    "mc_l2norm_bwd": (ctypes.c_int, [c_i32, c_i32, c_i32, c_vp, c_i64, c_fp, ctypes.c_float, c_fp, c_i64, c_vp,
                                     c_i64, c_vp]),
    "mc_attn_fwd": (ctypes.c_int, [ctypes.POINTER(AttnFwdParams), c_vp]),
    "mc_attn_bwd": (ctypes.c_int, [ctypes.POINTER(AttnBwdParams), c_vp]),
    "mc_mixer_proj_fwd": (ctypes.c_int, [ctypes.POINTER(MixerProjParams), c_vp]),
    "mc_mixer_proj_bwd": (ctypes.c_int, [ctypes.POINTER(MixerProjBwdParams), c_vp]),
    "mc_patch_embed_input": (ctypes.c_int, [ctypes.POINTER(PatchInputParams), c_vp]),
    "mc_ss2d_conv_stack_fwd": (ctypes.c_int, [ctypes.POINTER(SS2DConvParams), c_vp]),
    "mc_ss2d_conv_stack_bwd": (ctypes.c_int, [ctypes.POINTER(SS2DConvBwdParams), c_vp]),
    "mc_ss2d_conv_bwd_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32, c_i32, c_i32]),
    "mc_ss2d_merge_ln_gate_fwd": (ctypes.c_int, [ctypes.POINTER(SS2DMergeParams), c_vp]),
    "mc_ss2d_merge_ln_gate_bwd": (ctypes.c_int, [ctypes.POINTER(SS2DMergeBwdParams), c_vp]),
    "mc_ss2d_merge_bwd_workspace_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32, c_i32]),
    "mc_ss2d_group_proj": (ctypes.c_int, [ctypes.POINTER(SS2DGroupProjParams), c_vp]),
}

_lib = None


def load():
    """Load the library (once).  Raises if it is absent -- no fallback path."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"mamba_clip_amd: HIP library not found at {LIB_PATH}; build it with "
            "`make -C mamba-clip_amd` (gfx950).  There is no CPU fallback.")
    import torch  # noqa: F401  -- load torch's libamdhip64 first: one HIP runtime per process
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().mc_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def dtype_code(dt):
    import torch
    codes = {torch.float32: MC_DTYPE_F32, torch.bfloat16: MC_DTYPE_BF16, torch.float16: MC_DTYPE_F16,
             torch.float8_e4m3fn: MC_DTYPE_FP8_E4M3, torch.uint8: MC_DTYPE_U8}
    if dt not in codes:
        raise RuntimeError(f"mamba_clip_amd: unsupported dtype {dt} (float32, bfloat16, float16, float8_e4m3fn, uint8 only)")
    return codes[dt]


def ptr(t):
    return None if t is None else t.data_ptr()


def stream_handle(device=None):
    import torch
    return torch.cuda.current_stream(device).cuda_stream
