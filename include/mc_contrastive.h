/*
 * mc_contrastive.h -- C ABI of the MI355X contrastive-loss kernels (libmamba_clip_amd.so).
 *
 * Replaces the dense math of the reference's ClipLoss
 * (/root/reference/src/mamba_clip/loss.py):
 *   get_logits     loss.py:89-113   logits = logit_scale * I @ T^T (global, local or single process)
 *   forward        loss.py:124-147  (CE(logits_img, labels) + CE(logits_txt, labels)) / 2
 *   get_ground_truth loss.py:76-87  labels = arange(n) (+ n * rank for local_loss)
 * The feature all-gather (loss.py:16-44) stays in torch.distributed (RCCL)
 * on the host side; these entry points see plain device pointers.
 *
 * Conventions: row-major matrices with a leading dimension in elements; all
 * statistics and logits fp32; launches are asynchronous on `stream`; the
 * library never allocates.  Return MC_OK (0) or a negative MC_ERR_* code
 * (see mc_scan.h) with mc_last_error() describing it.
 */
#ifndef MAMBA_CLIP_AMD_MC_CONTRASTIVE_H
#define MAMBA_CLIP_AMD_MC_CONTRASTIVE_H

#include <stddef.h>
#include <stdint.h>

#include "mc_scan.h" /* mc_dtype, MC_OK / MC_ERR_* */

#ifdef __cplusplus
extern "C" {
#endif

/* C[m, n] = alpha * sa[m] * sb[n] * sum_k A[m, k] * B[n, k]   (A: M x K, B: N x K, K contiguous)
 * dtype of A and B: MC_DTYPE_BF16 (MFMA bf16, fp32 accumulate),
 * MC_DTYPE_F32 (exact-fp32 MFMA) or MC_DTYPE_FP8_E4M3 (fp8 MFMA, fp32
 * accumulate; K, lda, ldb multiples of 16 and A, B 16-B aligned -- the
 * quantiser below pads K).  alpha = *alpha_dev if alpha_dev != NULL
 * (a device scalar such as logit_scale.exp(): no host sync), else alpha.
 * sa / sb: optional per-row dequantisation factors of A / B (fp32, M / N
 * entries; NULL = 1), as written by mc_quant_rows_fp8.
 * C is fp32 (out_dtype MC_DTYPE_F32) or bf16 (MC_DTYPE_BF16).
 * Replaces the similarity matmul of ClipModel.get_logits (model.py:1104-1112)
 * and ClipLoss.get_logits (loss.py:89-113). */
typedef struct mc_gemm_nt_params {
  int32_t M, N, K;
  int32_t in_dtype, out_dtype;
  const void* A; int64_t lda;
  const void* B; int64_t ldb;
  void* C; int64_t ldc;
  float alpha;
  const float* alpha_dev;
  const float* row_scale_a;
  const float* row_scale_b;
} mc_gemm_nt_params;

int mc_gemm_nt(const mc_gemm_nt_params* p, void* stream);

/* Which kernel mc_gemm_nt runs for p (no launch): MC_GEMM_KERNEL_TILE (128 x 128 tiles, bf16 / fp32 /
 * fp8 with K % 16), MC_GEMM_KERNEL_FP8_TILE (fp8, K % 128, block-scaled 16x16x128 MFMA tiles) or
 * MC_GEMM_KERNEL_FP8_PANEL (fp8, K % 64 and K <= 512, N % 8, ldc % 8, 16-B aligned C: the register-panel
 * kernel that serves the C5 similarity).  0 for an empty problem. */
#define MC_GEMM_KERNEL_TILE 1
#define MC_GEMM_KERNEL_FP8_TILE 2
#define MC_GEMM_KERNEL_FP8_PANEL 3
int32_t mc_gemm_nt_kernel(const mc_gemm_nt_params* p);

/* Row-wise fp8 quantisation of a rows x cols matrix X (fp32 / bf16 / f16,
 * leading dimension ldx) for the fp8 similarity GEMM (stage-2 / frozen
 * features, BASELINE config 5):
 *   amax_i = max_j |X[i, j]|,  s_i = 448 / amax_i  (1 if amax_i == 0)
 *   Q[i, j] = e4m3fn_rne(clamp(X[i, j] * s_i, -448, 448))   for j < cols
 *   Q[i, j] = 0                                           for cols <= j < ldq
 *   inv_scale[i] = 1 / s_i
 * ldq must be a multiple of 16 and >= cols; Q 16-B aligned. */
int mc_quant_rows_fp8(int32_t rows, int32_t cols, int32_t in_dtype, const void* X, int64_t ldx, uint8_t* Q,
                      int64_t ldq, float* inv_scale, void* stream);

/* Softmax cross-entropy statistics along the rows (axis = 0: one value per
 * row, reduce over columns) or the columns (axis = 1) of an fp32 matrix S
 * (rows x cols, leading dimension lds):
 *   lse[i]     = log sum_j exp(S[i, j])            (row i; or column i for axis 1)
 *   nll[i]     = lse[i] - S[i, label_i]            label_i = i + label_offset
 * loss_out (device scalar, nullable) = sum_i nll[i] * loss_coef. */
int mc_ce_stats(int32_t rows, int32_t cols, const float* S, int64_t lds, int32_t axis, int64_t label_offset,
                float* lse, float* nll, float loss_coef, float* loss_out, void* workspace, size_t workspace_bytes,
                void* stream);
size_t mc_ce_stats_workspace_bytes(int32_t rows, int32_t cols, int32_t axis);

/* Gradient of  coef_r * sum_i nll_row[i] + coef_c * sum_j nll_col[j]  w.r.t. S,
 * times the upstream scalar *gout_dev:
 *   G[i, j] = gout * ( coef_r * (exp(S_ij - lse_r[i]) - [j == i + off_r])
 *                    + coef_c * (exp(S_ij - lse_c[j]) - [i == j + off_c]) )
 * (lse_c == NULL drops the column term).  G is written in out_dtype
 * (fp32 / bf16).  If dscale_out != NULL it also accumulates
 * sum_ij G_ij * S_ij / scale (scale = *scale_dev): the gradient of the loss
 * w.r.t. logit_scale, deterministic two-pass reduction in workspace. */
int mc_ce_grad(int32_t rows, int32_t cols, const float* S, int64_t lds, const float* lse_r, int64_t off_r,
               float coef_r, const float* lse_c, int64_t off_c, float coef_c, const float* gout_dev,
               int32_t out_dtype, void* G, int64_t ldg, const float* scale_dev, float* dscale_out, void* workspace,
               size_t workspace_bytes, void* stream);
size_t mc_ce_grad_workspace_bytes(int32_t rows, int32_t cols);

/* Fused logits + softmax cross-entropy (no M x N matrix in memory).
 *   S[i, j] = scale * sx[i] * sy[j] * sum_k X[i, k] Y[j, k]        (never stored)
 *   loss    = coef_r * sum_i (lse_r[i] - S[i, i + row_off])
 *           + coef_c * sum_j (lse_c[j] - S[j + col_off, j])        (column term iff lse_c != NULL)
 * mc_ce_fused_fwd: the GEMM tiles of mc_gemm_nt reduce their logits in
 * registers to per-row / per-column (max, sum exp) partials and target logits;
 * a second kernel folds them into lse_r (M), lse_c (N) and *loss_out.  The
 * workspace holds the partials (mc_ce_fused_fwd_workspace_bytes; about
 * 8 * (M * ceil(N/128) + N * ceil(M/128)) bytes).
 * mc_ce_fused_grad: recomputes the same tiles from (lse_r, lse_c) and writes
 *   G[i, j] = gmul * gout * ( coef_r (exp(S_ij - lse_r[i]) - [j == i + row_off])
 *                           + coef_c (exp(S_ij - lse_c[j]) - [i == j + col_off]) )
 * with gmul = scale if g_times_scale else 1 (so G @ Y is dX directly) and,
 * if dscale_out != NULL, *dscale_out = sum_ij G_ij S_ij / (gmul * scale):
 * the logit_scale gradient.  lse_r or lse_c NULL drops that term.  Called on
 * a block of rows of X (or, with the roles swapped, of Y) it yields one
 * block of dS (or dS^T) at a time, so the backward never holds M x N either.
 * Row / column offsets must satisfy |off| < 2^30.  in_dtype: bf16, fp32 or
 * fp8 e4m3 (fp8: forward only is meaningful, operands from mc_quant_rows_fp8
 * with sx / sy their inverse scales).
 * Replaces ClipLoss.get_logits + the two F.cross_entropy calls
 * (loss.py:89-147) and their autograd backward. */
typedef struct mc_ce_fused_params {
  int32_t M, N, K;
  int32_t in_dtype;
  const void* X; int64_t ldx;
  const void* Y; int64_t ldy;
  const float* row_scale_x;     /* sx, nullable */
  const float* row_scale_y;     /* sy, nullable */
  float scale;                  /* used when scale_dev == NULL */
  const float* scale_dev;
  int64_t row_off; float coef_r;
  int64_t col_off; float coef_c;
  float* lse_r;                 /* fwd: out (M);  grad: in, nullable */
  float* lse_c;                 /* fwd: out (N), NULL = no column term;  grad: in, nullable */
  float* loss_out;              /* fwd: device scalar */
  const float* gout_dev;        /* grad: upstream scalar, NULL = 1 */
  int32_t g_dtype;              /* grad: fp32 or bf16 */
  int32_t g_times_scale;
  void* G; int64_t ldg;         /* grad: M x N block */
  float* dscale_out;            /* grad: device scalar, nullable */
  void* workspace; size_t workspace_bytes;
} mc_ce_fused_params;

int mc_ce_fused_fwd(const mc_ce_fused_params* p, void* stream);
size_t mc_ce_fused_fwd_workspace_bytes(int32_t M, int32_t N, int32_t with_columns);
int mc_ce_fused_grad(const mc_ce_fused_params* p, void* stream);
size_t mc_ce_fused_grad_workspace_bytes(int32_t M, int32_t N);

#ifdef __cplusplus
}
#endif
#endif /* MAMBA_CLIP_AMD_MC_CONTRASTIVE_H */
