/*
 * mc_attn.h -- C ABI of the fused short-sequence multi-head attention (libmamba_clip_amd.so).
 *
 * The towers' self-attention (ViT-B/16 image tower: 197 tokens; BERT text tower: <= 256
 * tokens; 12 heads of 64).  The reference gets it from timm / open_clip / HF through
 * torch's scaled_dot_product_attention (model.py:1019-1064 builds
 * the towers); it replaces that call for the unmasked, dropout-free case:
 *   o = softmax(scale * q k^T) v          per (batch, head)
 * One workgroup owns one (batch, head): the whole sequence's K / V (and, backward, Q / dO)
 * sit in LDS, so the softmax is exact in one pass (no online rescaling) and dQ / dK / dV
 * need no cross-workgroup sums.
 *
 * Layout: every tensor is addressed as base + b * bs + n * ns + h * hs + d (element
 * strides, d contiguous), so q / k / v can be slices of one packed (B, N, 3, H, D)
 * projection output and o / dq / dk / dv can be written straight into the layouts the
 * next GEMM reads.  Requirements: head_dim == 64, 1 <= seqlen <= 256, dtype bf16 or f16,
 * 16-B aligned rows (pointers and the three strides multiples of 8 elements).
 * Same conventions as mc_scan.h: device pointers, asynchronous on `stream`,
 * MC_OK / MC_ERR_* return codes.
 */
#ifndef MAMBA_CLIP_AMD_MC_ATTN_H
#define MAMBA_CLIP_AMD_MC_ATTN_H

#include <stddef.h>
#include <stdint.h>

#include "mc_scan.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MC_ATTN_HEAD_DIM 64
#define MC_ATTN_MAX_SEQ 256

typedef struct {
  int32_t batch, heads, seqlen, head_dim, dtype;
  float scale;                        /* softmax scale, 1/sqrt(head_dim) for SDPA's default */
  const void* q; const void* k; const void* v;
  int64_t q_bs, q_ns, q_hs;           /* element strides of q, k and v (shared) */
  void* o; int64_t o_bs, o_ns, o_hs;
  float* lse;                         /* (batch, heads, seqlen) fp32: ln sum exp(scale q.k), for the backward */
} mc_attn_fwd_params;

/* o = softmax(scale q k^T) v and the row log-sum-exp. */
int mc_attn_fwd(const mc_attn_fwd_params* p, void* stream);

typedef struct {
  int32_t batch, heads, seqlen, head_dim, dtype;
  float scale;
  const void* q; const void* k; const void* v;
  int64_t q_bs, q_ns, q_hs;           /* shared by q, k, v */
  const void* o; const void* dout;
  int64_t o_bs, o_ns, o_hs;           /* shared by o and dout */
  const float* lse;                   /* from mc_attn_fwd */
  void* dq; void* dk; void* dv;
  int64_t dq_bs, dq_ns, dq_hs;        /* shared by dq, dk, dv */
  float* dsum;                        /* (batch, 3, heads, head_dim) fp32, nullable: per-batch sums over the
                                         sequence of dq | dk | dv as stored -- summed over the batch, the bias
                                         gradient of a packed qkv projection (no second pass over dq / dk / dv) */
} mc_attn_bwd_params;

/* dq, dk, dv of the above given dout (recomputes the probabilities from q, k and lse). */
int mc_attn_bwd(const mc_attn_bwd_params* p, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MAMBA_CLIP_AMD_MC_ATTN_H */
