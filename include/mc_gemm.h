/*
 * mc_gemm.h -- C ABI of the MI355X weight-gradient GEMM (libmamba_clip_amd.so, csrc/gemm_wgrad.hip).
 *
 *   mc_gemm_wgrad   C (M x N, fp32) = sum over T of A(t, m) B(t, n), bf16 / f16 operands
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

#ifdef __cplusplus
}
#endif

#endif
