/*
 * mc_ss2d.h -- C ABI of the SS2D cross-scan glue kernels (libmamba_clip_amd.so).
 *
 * The reference SS2D block (src/mamba_clip/model.py:297-647) builds its four scan directions by
 * copying -- xs = stack[x, x^T, flip x, flip x^T] (forward_corev0, model.py:510-517) -- and merges
 * them back with flips, transposes and adds (model.py:553-565, 640-644) around its depthwise conv
 * (model.py:636-637) and its out_norm / silu(z) gate (model.py:642-643).  The flips live in the
 * scan kernels' addressing (mc_scan.h reverse_groups / u_groups); these two fused ops own the rest:
 *
 *   mc_ss2d_conv_stack_fwd/bwd    depthwise k x k conv (+ bias) + SiLU over the channels-last
 *                                 in_proj half, written straight into the scan input
 *                                 u = [x, x^T] in fp32 (model.py:531-537 casts xs to fp32):
 *                                 the permute copy, the conv, the SiLU, the stack and the
 *                                 transposed copy in one pass (backward: the sum of the two
 *                                 frames' gradients, SiLU', the transposed depthwise conv and
 *                                 deterministic weight / bias gradients);
 *   mc_ss2d_merge_ln_gate_fwd/bwd the four direction outputs summed in the reference order
 *                                 ((y1 + y2) + y3) + y4 with the two column-major directions
 *                                 read transposed, LayerNorm over channels, times silu(z),
 *                                 written channels-last for out_proj (backward: dz, the
 *                                 LayerNorm parameter gradients and each direction's output
 *                                 gradient in its own frame).
 *
 * Conventions as mc_scan.h: device pointers, caller-owned buffers, asynchronous on `stream`,
 * MC_OK / MC_ERR_* return codes, mc_last_error() for the message.  Channels-last tensors have
 * unit channel stride; strides are in elements.  Requirements: channels % 4 == 0, channels-last
 * rows and strides 4-element aligned, ksize == 3 (SS2D's d_conv, model.py:331-339).
 */
#ifndef MAMBA_CLIP_AMD_MC_SS2D_H
#define MAMBA_CLIP_AMD_MC_SS2D_H

#include <stddef.h>
#include <stdint.h>

#include "mc_scan.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mc_ss2d_conv_params {
  int32_t batch, height, width, channels, ksize;
  int32_t xtype;                                          /* mc_dtype of x (and dx) */
  int64_t x_batch_stride, x_row_stride, x_col_stride;    /* x (B, H, W, C), channel stride 1 */
  const void* x;
  const float* weight;    /* (C, 1, k, k) fp32: nn.Conv2d(C, C, k, groups=C, padding=k/2).weight */
  const float* bias;      /* (C,) fp32, nullable */
  float* u;               /* (B, 2, C, H*W) fp32: u[b,0,c,h*W+w] = u[b,1,c,w*H+h] = silu(conv(x))[b,c,h,w] */
} mc_ss2d_conv_params;

int mc_ss2d_conv_stack_fwd(const mc_ss2d_conv_params* p, void* stream);

typedef struct mc_ss2d_conv_bwd_params {
  mc_ss2d_conv_params fwd;  /* the forward's inputs (fwd.u unused) */
  const float* du;          /* (B, 2, C, H*W) fp32: gradient of u */
  void* dx;                 /* (B, H, W, C) contiguous, xtype */
  float* dweight;           /* (C, k, k) fp32 */
  float* dbias;             /* (C,) fp32, nullable */
  void* workspace;
  size_t workspace_bytes;   /* >= mc_ss2d_conv_bwd_workspace_bytes(...) */
} mc_ss2d_conv_bwd_params;

size_t mc_ss2d_conv_bwd_workspace_bytes(int32_t batch, int32_t height, int32_t width, int32_t channels,
                                        int32_t ksize);
int mc_ss2d_conv_stack_bwd(const mc_ss2d_conv_bwd_params* p, void* stream);

typedef struct mc_ss2d_merge_params {
  int32_t batch, height, width, channels;
  int32_t ztype, ytype;     /* mc_dtype of z (and dz), of y (and dy) */
  float eps;                /* LayerNorm eps */
  const float* out;         /* (B, 4, C, H*W) fp32 scan outputs, each in its own frame:
                               directions 0, 2 at h*W + w, directions 1, 3 at w*H + h */
  const void* z;
  int64_t z_batch_stride, z_row_stride, z_col_stride;    /* z (B, H, W, C), channel stride 1 */
  const float* ln_weight;   /* (C,) fp32 */
  const float* ln_bias;     /* (C,) fp32, nullable */
  void* y;                  /* (B, H, W, C) contiguous, ytype: LayerNorm(merge(out)) * silu(z) */
  float* mean;              /* (B*H*W,) fp32, saved for the backward */
  float* rstd;              /* (B*H*W,) fp32 */
} mc_ss2d_merge_params;

int mc_ss2d_merge_ln_gate_fwd(const mc_ss2d_merge_params* p, void* stream);

typedef struct mc_ss2d_merge_bwd_params {
  mc_ss2d_merge_params fwd; /* the forward's inputs and its saved mean / rstd (fwd.y unused) */
  const void* dy;
  int64_t dy_batch_stride, dy_row_stride, dy_col_stride;  /* dy (B, H, W, C) ytype, channel stride 1 */
  float* dout;              /* (B, 4, C, H*W) fp32: gradient of each direction's output, own frame */
  void* dz;                 /* (B, H, W, C) contiguous, ztype */
  float* dln_weight;        /* (C,) fp32 */
  float* dln_bias;          /* (C,) fp32, nullable */
  void* workspace;
  size_t workspace_bytes;   /* >= mc_ss2d_merge_bwd_workspace_bytes(...) */
} mc_ss2d_merge_bwd_params;

size_t mc_ss2d_merge_bwd_workspace_bytes(int32_t batch, int32_t height, int32_t width, int32_t channels);
int mc_ss2d_merge_ln_gate_bwd(const mc_ss2d_merge_bwd_params* p, void* stream);

/*
 * mc_ss2d_group_proj: the per-direction projections of SS2D (model.py:519-528, x_proj and dt_proj as
 * einsums over the four directions, in fp32: model.py:531-537) and their input gradients, as one
 * grouped product over sequence slabs, without operand permutes:
 *
 *   Y[b][g][m][l] = (acc ? A[b][g][m][l] : 0) + sum_n W[g][m][n] * X[b][g % x_group_mod][n][l]
 *
 * for b < batch, g < groups, m < rows_out, n < rows_in, l < seqlen; fp32 everywhere; the sum over n
 * runs in order (deterministic).  Element addresses (in floats): W at g*w_gs + m*w_ms + n*w_ns,
 * X at b*x_bs + (g % x_group_mod)*x_gs + n*x_ns + l, A at b*a_bs + g*a_gs + m*a_ms + l, Y likewise with
 * y_*.  A may alias Y (in-place accumulation).  Uses (SS2D, k = 2 i + j the direction):
 *   x_dbl[b,k] = x_proj[k] u[b, k % 2]       (x_group_mod 2: u = [x, x^T] holds two frames)
 *   delta[b,k] = dt_proj[k] x_dbl[b,k,:R]    (the dt rows)
 *   d(dt rows)[b,k] = dt_proj[k]^T ddelta[b,k]   (w_ms / w_ns swapped)
 *   du[b,j] = x_proj[j]^T dx_dbl[b,j] + x_proj[2+j]^T dx_dbl[b,2+j]   (two calls, the second with acc)
 */
typedef struct mc_ss2d_group_proj_params {
  int32_t batch, groups, rows_out, rows_in, seqlen;
  int32_t x_group_mod;      /* >= 1 */
  const float* w;  int64_t w_gs, w_ms, w_ns;
  const float* x;  int64_t x_bs, x_gs, x_ns;
  const float* acc; int64_t a_bs, a_gs, a_ms;     /* nullable */
  float* y;        int64_t y_bs, y_gs, y_ms;
} mc_ss2d_group_proj_params;

int mc_ss2d_group_proj(const mc_ss2d_group_proj_params* p, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MAMBA_CLIP_AMD_MC_SS2D_H */
