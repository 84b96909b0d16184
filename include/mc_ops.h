/*
 * mc_ops.h -- C ABI of the MI355X encoder kernels around the scan (libmamba_clip_amd.so).
 *
 * The reference gets these from third-party packages it imports but does not
 * vendor (open_clip/timm for the ViT tower, mamba_ssm/causal_conv1d for a
 * Mamba block: SURVEY.md section 2.2); the build owns them:
 *   mc_add_rmsnorm_fwd/bwd  fused residual-add + RMSNorm (Mamba block pre-norm,
 *                           residual stream kept in fp32)
 *   mc_add_layernorm_fwd/bwd fused residual-add + LayerNorm (ViT / BERT pre-LN
 *                           blocks: timm Block norm1/norm2 + the residual add)
 *   mc_causal_conv1d_fwd/bwd depthwise causal conv1d (+ optional SiLU) over the
 *                           sequence of (batch, dim, seqlen) activations, the
 *                           short conv in front of the scan (the 2-D analogue is
 *                           SS2D's depthwise conv, model.py:331-339)
 *   mc_patch_embed_input     the image input path: float NCHW or raw uint8 NHWC images ->
 *                           normalised patch rows for the patch-embed GEMM in one pass
 *   mc_patch_im2col          ViT / VSSM patch-embed input reshuffle: stride ==
 *                           kernel conv as a GEMM (model.py:189-191 PatchEmbed2D)
 * Same conventions as mc_scan.h: device pointers, caller-owned buffers,
 * asynchronous on `stream`, MC_OK / MC_ERR_* return codes.
 */
#ifndef MAMBA_CLIP_AMD_MC_OPS_H
#define MAMBA_CLIP_AMD_MC_OPS_H

#include <stddef.h>
#include <stdint.h>

#include "mc_scan.h"

#ifdef __cplusplus
extern "C" {
#endif

/* h = x + res_in (res_in nullable);  y = h * rsqrt(mean(h^2) + eps) * w
 * x, y: rows x cols in `dtype` (bf16 / f16 / f32); res_in, res_out, w, rstd fp32.
 * res_out (rows x cols fp32) receives h; rstd (rows) the inverse RMS. */
int mc_add_rmsnorm_fwd(int32_t rows, int32_t cols, int32_t dtype, const void* x, const float* res_in, const float* w,
                       float eps, void* y, float* res_out, float* rstd, void* stream);

/* Backward of the above given dy (dtype) and dres (fp32 gradient of res_out,
 * nullable): dh = rstd * (w dy - h rstd^2 mean(h w dy)) + dres, written to
 * dx (dtype, nullable) and dres_in (fp32, nullable); dw (cols, fp32) =
 * sum_rows dy h rstd, reduced deterministically through the workspace. */
int mc_add_rmsnorm_bwd(int32_t rows, int32_t cols, int32_t dtype, const void* dy, const float* dres, const float* h,
                       const float* w, const float* rstd, void* dx, float* dres_in, float* dw, void* workspace,
                       size_t workspace_bytes, void* stream);
size_t mc_add_rmsnorm_bwd_workspace_bytes(int32_t rows, int32_t cols);

/* Residual-add + LayerNorm (ViT / BERT pre-LN blocks):
 *   h = x + res (rounded to dtype; res nullable -> h = x), y = (h - mean) * rstd * w + bias.
 * x, res, y, h_out: (rows, cols) row-major in dtype, 16-B aligned rows; w, bias (cols,) fp32
 * (bias nullable); mean, rstd (rows,) fp32 saved for the backward.  h_out nullable.
 * cols % 8 == 0 (16-bit) / % 4 (fp32) and <= 4096 / 2048. */
int mc_add_layernorm_fwd(int32_t rows, int32_t cols, int32_t dtype, const void* x, const void* res, const float* w,
                         const float* bias, float eps, void* y, void* h_out, float* mean, float* rstd, void* stream);

/* Backward of (y, h) = add_layernorm(x, res): dx = dres = dh + d(LN)/dh . dy  (dh nullable),
 * dw, dbias (cols,) fp32 (dbias nullable); dx_colsum (cols,) fp32, nullable: the column
 * sums of dx as stored -- the bias gradient of the linear layer that produced x (ViT/BERT
 * fc2 and attention proj), taken in this pass.  Deterministic reductions in workspace. */
int mc_add_layernorm_bwd(int32_t rows, int32_t cols, int32_t dtype, const void* dy, const void* dh, const void* h,
                         const float* w, const float* mean, const float* rstd, void* dx, float* dw, float* dbias,
                         float* dx_colsum, void* workspace, size_t workspace_bytes, void* stream);
size_t mc_add_layernorm_bwd_workspace_bytes(int32_t rows, int32_t cols);

/* y[b, d, t] = act( bias[d] + sum_k w[d, k] * x[b, d, t - (K-1) + k] ), zero left padding.
 * x, y: (batch, dim, seqlen) with strides (x_bs, x_ds, 1) / (y_bs, y_ds, 1) -- e.g. the
 * channel-major (dim, batch*seqlen) GEMM output viewed as (batch, dim, seqlen);
 * w (dim, K) fp32, bias (dim,) fp32 nullable; act = SiLU if silu else identity.  K <= 8. */
int mc_causal_conv1d_fwd(int32_t batch, int32_t dim, int32_t seqlen, int32_t K, int32_t dtype, const void* x,
                         int64_t x_bs, int64_t x_ds, const float* w, const float* bias, int32_t silu, void* y,
                         int64_t y_bs, int64_t y_ds, void* stream);

/* Backward: dx (dtype, strides dx_bs, dx_ds, 1), dw (dim, K) fp32, dbias (dim) fp32 (nullable). */
int mc_causal_conv1d_bwd(int32_t batch, int32_t dim, int32_t seqlen, int32_t K, int32_t dtype, const void* x,
                         int64_t x_bs, int64_t x_ds, const float* w, const float* bias, int32_t silu, const void* dy,
                         int64_t dy_bs, int64_t dy_ds, void* dx, int64_t dx_bs, int64_t dx_ds, float* dw,
                         float* dbias, void* workspace, size_t workspace_bytes, void* stream);
size_t mc_causal_conv1d_bwd_workspace_bytes(int32_t batch, int32_t dim, int32_t seqlen, int32_t K);

/* patches[(b*ph + i)*pw + j, (c*P + ky)*P + kx] = img[b, c, i*P + ky, j*P + kx]
 * img (batch, C, H, W) contiguous; H % P == W % P == 0; same dtype in and out. */
int mc_patch_im2col(int32_t batch, int32_t C, int32_t H, int32_t W, int32_t P, int32_t dtype, const void* img,
                    void* patches, void* stream);

/* The image input path of the patch embedding (reference: data.py get_transform 37-108 ToTensor +
 * Normalize, then the visual tower's k = s = P patch conv):
 *   out[(b*ph + i)*pw + j, (c*P + ky)*P + kx] = scale[c] * img(b, c, i*P + ky, j*P + kx) + shift[c]
 * img: float NCHW (f32 / bf16 / f16; scale, shift nullable -> a plain im2col with a dtype cast) or
 * uint8 NHWC decoded images (1 or 3 channels; scale = 1 / (255 std), shift = -mean / std).
 * P % 4 == 0, H % P == W % P == 0; out (B*ph*pw, C*P*P) row-major in out_dtype (f32 / bf16 / f16). */
enum { MC_LAYOUT_NCHW = 0, MC_LAYOUT_NHWC = 1 };
typedef struct mc_patch_input_params {
  int32_t batch, channels, height, width, patch;
  int32_t layout, in_dtype, out_dtype;
  const void* img;
  const float* scale;   /* (C,) fp32, nullable together with shift */
  const float* shift;
  void* out;
} mc_patch_input_params;
int mc_patch_embed_input(const mc_patch_input_params* p, void* stream);

/* Fused gradient passes that also produce the bias gradient of the GEMM in
 * front of them, in the same single stream over the (rows x cols) gradient
 * (rows 16-B aligned, cols a multiple of 8 / 4 for 16-bit / fp32):
 * mc_gelu_bwd: gh = ga * gelu'(h)  (exact erf GELU, torch approximate='none'),
 *              dbias[c] = sum_rows gh[:, c]  -- the ViT / BERT MLP's fc1 bias;
 * mc_qkv_grad_pack: the attention's q / k / v gradients (three (batch, seq,
 *              heads, head_dim) tensors, any batch / token / head strides,
 *              head_dim contiguous) packed into the qkv projection's output
 *              gradient (batch*seq, 3*heads*head_dim) -- the layout of its
 *              (B, N, 3, H, D) view -- plus its column sums (the qkv bias, nullable).
 * Column sums are fp32, of the stored (rounded) values, deterministic
 * (fixed-order slice partials in the workspace, mc_grad_colsum_workspace_bytes).
 * Replace the unfused torch sequence GELU-backward + sum(0) and
 * stack(dq, dk, dv) + sum(0) behind the towers' MLP / attention (timm Block,
 * open_clip VisionTransformer as loaded at reference model.py:1270). */
size_t mc_grad_colsum_workspace_bytes(int32_t rows, int32_t cols);
int mc_gelu_bwd(int32_t rows, int32_t cols, int32_t dtype, const void* h, int64_t ldh, const void* ga, int64_t ldga,
                void* gh, int64_t ldgh, float* dbias, void* workspace, size_t workspace_bytes, void* stream);

typedef struct mc_qkv_pack_params {
  int32_t batch, seq, heads, head_dim, dtype;
  const void* src[3];                 /* dq, dk, dv */
  int64_t sb[3], sn[3], sh[3];        /* element strides of batch, token, head per source */
  void* out; int64_t ld_out;
  float* dbias;                       /* nullable */
  void* workspace; size_t workspace_bytes;
} mc_qkv_pack_params;
int mc_qkv_grad_pack(const mc_qkv_pack_params* p, void* stream);

/* mc_stream_copy: dst[0, nbytes) = src[0, nbytes) with 16-B non-temporal vector loads / stores.
 * A measurement utility with no reference counterpart: bench.py times it as the achievable
 * HBM streaming rate next to the 8 TB/s spec.  16-B aligned, nbytes % 16 == 0. */
int mc_stream_copy(const void* src, void* dst, size_t nbytes, void* stream);

/* mc_sum_slabs: dst[i] = sum_{k < s} src[k * slab_stride + i], i < n, fp32, the slabs added in
 * order k = 0, 1, ... (deterministic).  The slab sum of the towers' split-K weight gradients
 * (ops.wgrad: s strided-batched GEMM partials over the token dimension); one coalesced pass with
 * 16-B loads when n, slab_stride and the pointers allow. */
int mc_sum_slabs(int32_t s, int64_t n, const float* src, int64_t slab_stride, float* dst, void* stream);

/* mc_cast_f32_many: dst_base[c.dst_off + i] = (dtype) c.src[i], i < c.n, for every chunk c, in ONE
 * launch (RNE: the bits of torch's .to(bfloat16 / float16)).  The towers' projection weights are
 * cast once per forward instead of one cast kernel per weight and use (~230 launches per C2 step).
 * chunks: DEVICE array of n_chunks entries, each at most MC_CAST_CHUNK elements; the table holds
 * destination OFFSETS (elements) so one table serves a fresh dst_base every forward.  dst_dtype
 * bf16 or f16.  Chunks with 16-B aligned src / dst and n % 8 == 0 move as 16-B vectors. */
#define MC_CAST_CHUNK 16384
typedef struct {
  const float* src;
  int64_t dst_off;
  int64_t n;
} mc_cast_chunk;
int mc_cast_f32_many(int32_t n_chunks, const mc_cast_chunk* chunks, void* dst_base, int32_t dst_dtype, void* stream);

/* Transposed 16-bit copies of fp32 weights in one launch (the towers' input gradients run the "tn"
 * GEMM form, which needs w^T row-major): one table entry per tile of up to 64 x 64 source elements,
 * dst[c * dst_ld + r] = src[r * src_ld + c] for r < rows, c < cols (src / dst at the tile origins).
 * tiles: DEVICE array of n_tiles entries. */
typedef struct mc_cast_t_tile {
  const float* src;       /* tile origin in the fp32 source */
  int64_t dst_off;        /* tile origin in dst_base, elements */
  int32_t src_ld, dst_ld; /* row strides, elements */
  int32_t rows, cols;     /* tile extent in the source (<= 64 each) */
} mc_cast_t_tile;
int mc_cast_transpose_f32_many(int32_t n_tiles, const mc_cast_t_tile* tiles, void* dst_base, int32_t dst_dtype,
                               void* stream);

/* AdamW step over many fp32 parameters in one launch (replaces torch.optim.AdamW's step in the
 * reference's train loop, train.py:183-198 / create_optimizer; decoupled weight decay, no amsgrad):
 *   p *= 1 - lr * wd;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2;
 *   p -= step_size * m / (sqrt(v) / bc2_sqrt + eps),  step_size = lr / (1 - b1^t), bc2_sqrt = sqrt(1 - b2^t).
 * tensors: DEVICE array, one entry per parameter (g may change every step); chunks: DEVICE array,
 * one entry per <= MC_ADAMW_CHUNK elements of a tensor (off a multiple of 4); hyper: host struct,
 * passed by value to the kernel (hyper-parameters and bias corrections of this step, per group). */
#define MC_ADAMW_MAX_GROUPS 8
#define MC_ADAMW_CHUNK 65536
typedef struct mc_adamw_tensor {
  float* p;
  float* m;
  float* v;
  const float* g;
} mc_adamw_tensor;
typedef struct mc_adamw_chunk {
  int32_t tensor, group;
  int64_t off, n;
} mc_adamw_chunk;
typedef struct mc_adamw_group {
  float beta1, beta2, eps, decay;    /* decay = 1 - lr * weight_decay */
  float step_size, bc2_sqrt;
} mc_adamw_group;
typedef struct mc_adamw_hyper {
  int32_t n_groups, reserved;
  mc_adamw_group group[MC_ADAMW_MAX_GROUPS];
} mc_adamw_hyper;
int mc_adamw_step(int32_t n_chunks, const mc_adamw_chunk* chunks, const mc_adamw_tensor* tensors,
                  const mc_adamw_hyper* hyper, void* stream);

/* ---- Mamba mixer projections (mixer_proj.hip): x_proj and dt_proj around the scan, fused.
 * Reference: the mixer's x_dbl = x_proj(x), delta = dt_proj.weight @ dt_raw (upstream
 * mamba_simple.Mamba; SS2D's analogue model.py:519-528, 630-647).  Channel-major activations
 * (dim, tokens), tokens contiguous; all 16-bit (dtype bf16 / f16), weights contiguous.
 *   forward:  x_dbl (P, T) = w_x (P, D) . x (D, T), rounded to dtype;
 *             delta (D, T) = w_dt (D, R) . x_dbl[0:R], rounded (no bias: the scan adds it)
 *   backward: d_x_dbl (P, T) = [w_dt^T . g_delta ; g_b ; g_c], rounded;
 *             dx (D, T) = w_x^T . d_x_dbl + du (du nullable), rounded once
 * The weight gradients are left to the caller (they are reductions over T).
 * Requirements: dim % 64 == 0, tokens % 8 == 0, rank % 16 == 0 in [16, 96], proj_rows = rank + 32
 * (dstate 16: every reference config); 16-B aligned rows (strides % 8 elements; du 8-B), w_dt
 * 8-B aligned. */
typedef struct mc_mixer_proj_params {
  int32_t dim, tokens, rank, proj_rows, dtype;
  int64_t x_ld, x_dbl_ld, delta_ld;      /* row strides (elements) */
  const void* x;                          /* (dim, tokens) */
  const void* w_x;                        /* (proj_rows, dim): x_proj.weight */
  const void* w_dt;                       /* (dim, rank): dt_proj.weight */
  void* x_dbl;                            /* (proj_rows, tokens) out */
  void* delta;                            /* (dim, tokens) out */
} mc_mixer_proj_params;

int mc_mixer_proj_fwd(const mc_mixer_proj_params* p, void* stream);

typedef struct mc_mixer_proj_bwd_params {
  int32_t dim, tokens, rank, proj_rows, dtype;
  int64_t g_delta_ld, g_b_ld, g_c_ld, du_ld, d_x_dbl_ld, dx_ld;
  const void* g_delta;                    /* (dim, tokens): gradient of delta */
  const void* g_b;                        /* nullable (16, tokens): gradient of x_dbl's B rows (the scan's dB) */
  const void* g_c;                        /* nullable (16, tokens): gradient of the C rows (dC) */
  const void* w_x;
  const void* w_dt;
  const void* du;                         /* nullable (dim, tokens): the other consumer's gradient of x */
  void* d_x_dbl;                          /* (proj_rows, tokens) out */
  void* dx;                               /* (dim, tokens) out */
} mc_mixer_proj_bwd_params;

int mc_mixer_proj_bwd(const mc_mixer_proj_bwd_params* p, void* stream);

/* mc_colsum: out[c] = sum_{r < rows} x[r * ld + c] in fp32, c < cols, x fp32 / bf16 / fp16 row-major
 * (row stride ld elements).  Fixed row slices summed per workgroup, the slice partials folded in order:
 * deterministic, and no workgroup reads another's results during the launch.  Replaces torch's batch /
 * token reductions in the towers' glue -- the bias gradients of projections whose producer left no
 * column sums (ops.LinearSK), the ViT's cls_token / pos_embed and BERT's position gradients -- whose
 * cross-workgroup combine returned wrong sums beside concurrent library GEMMs.
 * Reference: the autograd reductions behind model.py:232-358's token embedding (open_clip / timm
 * VisionTransformer._pos_embed).  16-B vector loads when ld, cols and x allow.  Workspace:
 * mc_colsum_workspace_bytes(rows, cols). */
size_t mc_colsum_workspace_bytes(int32_t rows, int32_t cols);
int mc_colsum(int32_t rows, int32_t cols, int32_t dtype, const void* x, int64_t ld, float* out,
              void* workspace, size_t workspace_bytes, void* stream);
/* out[c] = sum_k part[k * cols + c] (fp32), k = 0 .. nslices-1, in a fixed order: the fold of per-slice /
 * per-tile column partials (e.g. mc_linear's GELU' epilogue, one row per 256-token tile). */
int mc_colsum_fold(int32_t nslices, int32_t cols, const float* part, float* out, void* stream);

/* mc_l2norm_fwd / _bwd: torch.nn.functional.normalize(x, dim=-1) for a (rows, cols) matrix -- the
 * features ClipModel.encode_image / encode_text(normalize=True) return (reference model.py:1011-1017).
 * Forward y = x / max(||x||, eps) in fp32, norm[r] = ||x_r||; backward dx = (g - y (y . g)) / ||x||
 * (g / eps where the clamp is active), dx in x's dtype.  One wave per row: no cross-workgroup
 * reduction (torch's norm launch splits each row over 8 workgroups). */
int mc_l2norm_fwd(int32_t rows, int32_t cols, int32_t dtype, const void* x, int64_t ldx, float eps,
                  float* y, int64_t ldy, float* norm, void* stream);
int mc_l2norm_bwd(int32_t rows, int32_t cols, int32_t dtype, const void* x, int64_t ldx, const float* norm,
                  float eps, const float* g, int64_t ldg, void* dx, int64_t lddx, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MAMBA_CLIP_AMD_MC_OPS_H */
