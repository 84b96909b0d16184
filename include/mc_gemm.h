/*
 * mc_gemm.h -- C ABI of the MI355X weight-gradient GEMM (libmamba_clip_amd.so, csrc/gemm_wgrad.hip).
 *
 *   mc_gemm_wgrad   C (M x N, fp32) = sum over T of A(t, m) B(t, n), bf16 / f16 operands
 *   mc_linear       Y (rows x cols, 16-bit) = X W^T with a fused epilogue (bias, bias + GELU, GELU'),
 *                   the towers' Linear forward / input-gradient GEMMs on the same 256 x 256 kernel
 *
 * It replaces the library GEMM behind every tower Linear's weight gradient, dW = G^T X
 * (reference: the towers' Linear / MLP layers behind encode_image / encode_text,
 * /root/reference/src/mamba_clip/model.py:1011-1017, built at model.py:1270; autograd's
 * `grad_weight = grad_output.t() @ input`).  T (batch x tokens) is long and M x N short, so the
 * kernel splits T over several workgroups per output tile and sums the fp32 partials in a fixed
 * order: the result is deterministic (bitwise run to run) for a given (M, N, T, splits).
 *
 * Operand layouts, per operand:
 *   MC_WGRAD_TOKEN_MAJOR   A(t, m) = A[t * lda + m]   (a Linear's (tokens, features) rows)
 *   MC_WGRAD_FEATURE_MAJOR A(t, m) = A[m * lda + t]   (the Mamba mixer's channel-major activations)
 * Requirements: T % 64 == 0; 16-B aligned bases; leading dims % 8 == 0; token-major feature
 * counts % 8 == 0; C contiguous (ldc == N).  Same conventions as mc_scan.h: device pointers,
 * caller-owned buffers, asynchronous on `stream`, MC_OK / MC_ERR_* return codes.
 */
#ifndef MAMBA_CLIP_AMD_MC_GEMM_H
#define MAMBA_CLIP_AMD_MC_GEMM_H

#include <stddef.h>
#include <stdint.h>

#include "mc_scan.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MC_WGRAD_TOKEN_MAJOR 0
#define MC_WGRAD_FEATURE_MAJOR 1

typedef struct mc_wgrad_params {
  int32_t M, N, T;
  int32_t dtype;                 /* MC_DTYPE_BF16 / MC_DTYPE_F16 (both operands) */
  int32_t a_layout, b_layout;    /* MC_WGRAD_* */
  const void* A;
  int64_t lda;                   /* elements */
  const void* B;
  int64_t ldb;
  float* C;
  int64_t ldc;                   /* must equal N */
  int32_t splits;                /* reduction splits; 0 = automatic (about one workgroup per CU) */
  int32_t reserved;
  void* workspace;               /* >= mc_gemm_wgrad_workspace_bytes(p), 16-B aligned (fp32 partial slabs) */
  size_t workspace_bytes;
} mc_wgrad_params;

size_t mc_gemm_wgrad_workspace_bytes(const mc_wgrad_params* p);
int mc_gemm_wgrad(const mc_wgrad_params* p, void* stream);

/*
 * mc_linear: Y[t][f] = sum_k X[t][k] W[f][k] (+ epilogue), fp32 accumulation, Y rounded once to the
 * operand dtype.  The forward of a tower Linear (X = input, W = weight) and its input gradient
 * (X = output gradient, W = the TRANSPOSED weight copy, (in, out)) -- reference: the towers' Linear /
 * MLP layers behind encode_image / encode_text, model.py:1011-1017 (timm Mlp: fc1 -> nn.GELU() exact
 * erf -> fc2).  Epilogues:
 *   MC_LINEAR_EPI_NONE       Y = XW^T
 *   MC_LINEAR_EPI_BIAS       Y = XW^T + bias
 *   MC_LINEAR_EPI_BIAS_GELU  Y = h = XW^T + bias (the pre-activation, kept for the backward) and
 *                            Y2 = gelu(h) = h * Phi(h), exact erf, of the ROUNDED h (as torch's
 *                            F.gelu of the stored h) -- fc1 + GELU in one pass
 *   MC_LINEAR_EPI_GELU_GRAD  Y = round(XW^T) * gelu'(H) -- fc2's input gradient times GELU's
 *                            derivative at fc1's saved pre-activation H, rounded as torch's
 *                            gelu_backward of the stored fc2 input gradient; with `colsum`, also
 *                            the fp32 column sums of Y as stored (fc1's bias gradient), per
 *                            256-token tile into the workspace and folded in a fixed order
 * Requirements: K % 64 == 0, cols % 8 == 0, 16-B aligned bases, leading dims % 8 == 0, unit stride
 * along K (X, W) and along the features (Y, Y2, H).  Deterministic: one workgroup per output tile.
 */
#define MC_LINEAR_EPI_NONE 0
#define MC_LINEAR_EPI_BIAS 1
#define MC_LINEAR_EPI_BIAS_GELU 2
#define MC_LINEAR_EPI_GELU_GRAD 3

typedef struct mc_linear_params {
  int32_t rows, cols, K;         /* tokens, output features, reduction */
  int32_t dtype;                 /* MC_DTYPE_BF16 / MC_DTYPE_F16 (X, W, Y, Y2, H) */
  int32_t epilogue;              /* MC_LINEAR_EPI_* */
  int32_t reserved;
  const void* X; int64_t ldx;    /* (rows, K) */
  const void* W; int64_t ldw;    /* (cols, K) */
  void* Y; int64_t ldy;          /* (rows, cols) */
  void* Y2; int64_t ldy2;        /* BIAS_GELU: (rows, cols) gelu(h) */
  const void* bias;              /* BIAS / BIAS_GELU: (cols,) in the operand dtype, 8-B aligned */
  const void* H; int64_t ldh;    /* GELU_GRAD: (rows, cols) pre-activation */
  float* colsum;                 /* GELU_GRAD, optional: (cols,) column sums of Y */
  void* workspace;               /* >= mc_linear_workspace_bytes(p) when colsum is set, 16-B aligned */
  size_t workspace_bytes;
} mc_linear_params;

size_t mc_linear_workspace_bytes(const mc_linear_params* p);
int mc_linear(const mc_linear_params* p, void* stream);

/*
 * mc_gemm_small_k: Y (M x T) = W (M x K) X (K x T), 16-bit, fp32 accumulation, one rounding -- a short
 * reduction (K in {16, 32, 48, 64}) over rows of X with unit token stride: the Mamba mixer's dt_proj
 * forward, delta = W_dt dt_raw (reference: Mamba's dt_proj Linear applied to x_proj's dt rows; the SS2D
 * form is the einsum at model.py:519-528).  W rows 8-B aligned (ldw % 4 == 0), X / Y rows 16-B aligned
 * (ldx % 8, ldy % 8 == 0), T % 8 == 0.
 */
int mc_gemm_small_k(int32_t M, int32_t K, int32_t T, int32_t dtype, const void* W, int64_t ldw, const void* X,
                    int64_t ldx, void* Y, int64_t ldy, void* stream);

/*
 * mc_gemm_skinny_m: Y (M x T) = W (M x K) X (K x T), 16-bit, fp32 accumulation summed in a fixed order,
 * one rounding -- few output rows (M <= 96) over a long reduction (K % 256 == 0): the Mamba mixer's
 * x_proj forward, x_dbl = W_x x (reference: Mamba's x_proj Linear; the SS2D form at model.py:519-528).
 * Same layout requirements as mc_gemm_small_k.
 */
int mc_gemm_skinny_m(int32_t M, int32_t K, int32_t T, int32_t dtype, const void* W, int64_t ldw, const void* X,
                     int64_t ldx, void* Y, int64_t ldy, void* stream);

#ifdef __cplusplus
}
#endif

#endif
