// contrastive.hip -- gathered InfoNCE (ClipLoss) math for MI355X (gfx950).
//
// Reference: /root/reference/src/mamba_clip/loss.py:89-147 (get_logits + forward):
//   logits = logit_scale * I @ T^T ;  loss = (CE(logits, arange) + CE(logits^T, arange)) / 2
// (local_loss: two (b x N) logit blocks against the gathered features, labels
//  offset by b * rank).  The gather itself is torch.distributed (RCCL).
//
// Kernels
//  * gemm_nt: C = alpha * A B^T on the matrix cores.  128x128 output tile per
//    256-thread workgroup (4 waves, 64x64 each = 4x4 MFMA tiles), K staged
//    through LDS in 64-byte row slices (80-byte padded rows: conflict-free
//    fragment reads), next slice prefetched into registers under the MFMAs.
//    bf16 inputs use v_mfma_f32_16x16x32_bf16 (fp32 accumulate); fp32 inputs
//    use the exact-fp32 v_mfma_f32_16x16x4_f32, fp8 (OCP e4m3fn) inputs
//    v_mfma_f32_16x16x32_fp8_fp8 with a 64-element K slice (two MFMA k-steps
//    per LDS fragment read) and per-row dequantisation factors applied in the
//    epilogue.  alpha may live on the device (logit_scale.exp()), so the loss
//    needs no host sync.
//  * quant_rows_fp8: one wave per row, amax -> 448/amax scale -> v_cvt_pk_fp8_f32.
//  * ce_rows / ce_cols(+finalize): log-sum-exp statistics and per-label NLL
//    along rows or columns, online max/sum, deterministic fixed-order
//    partial reductions (no atomics).
//  * ce_grad: fused softmax-minus-onehot gradient for the row and column CE
//    terms in one pass, plus the logit_scale gradient sum(G*S)/scale.
#include <algorithm>
#include <cstdlib>

#include "mc_common.h"
#include "../../include/mc_contrastive.h"

#ifndef MC_SIM_EXP
#define MC_SIM_EXP 0
#endif
#ifndef MC_NT_STORE
#define MC_NT_STORE 0
#endif
namespace mc {
namespace ctr {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int BM = 128, BN = 128;
constexpr int kRowBytes = 64;            // one K slice of a tile row
constexpr int kLdsStride = 80;           // padded row (bytes): conflict-free 16-lane fragment reads
constexpr int kTileBytes = BM * kLdsStride;

struct GemmArgs {
  int M, N, K;
  const void* A; int64_t lda;
  const void* B; int64_t ldb;
  void* C; int64_t ldc;
  float alpha; const float* alpha_dev;
  const float* sa; const float* sb;   // per-row dequantisation (fp8), nullable
  int tiles_m, tiles_n;
  int c_vec;                           // C 16-B aligned and ldc % 4 == 0: vector stores in full tiles
  int c_vec16;                         // 16-bit C: ldc % 8 == 0 as well (16-B stores of 8 values)
  // fused cross-entropy epilogues (kEpi 1 = statistics, 2 = gradient).  Labels:
  // row i's target column is i + off_r, column j's target row is j + off_c.
  int off_r, off_c;
  float coef_r, coef_c;
  const float* lse_r; const float* lse_c;   // kEpi 2 inputs; NULL drops that term
  const float* gout_dev;                    // kEpi 2 upstream scalar (NULL = 1)
  int g_times_alpha;                        // kEpi 2: store alpha * G (then G @ Y is dX directly)
  float2* rpart; float2* cpart;             // kEpi 1: (max, sumexp) partials [tiles_n][M], [tiles_m][N]
  float* tgt_r; float* tgt_c;               // kEpi 1: target logits (written by the tile holding them)
  float* gpart;                             // kEpi 2: per-workgroup sum(G * S), nullable
};

typedef uint8_t fp8_t;   // OCP e4m3fn bits

__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int xcd = bid & 7, q = nblocks >> 3, r = nblocks & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mm = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
  m = mm;
}

// Statistics epilogue of the fused logits + cross-entropy forward: the 128x128
// logit tile never leaves registers.  Each wave reduces its 64x64 quadrant to
// per-row and per-column (max, sum exp) partials with a transpose-reduce
// (every shuffle step halves the entries a lane carries, so 16 row entries
// need 15 exchanges, not 64), the two waves sharing rows / columns merge
// through LDS, and one (max, sumexp) per row and tile column-block lands in
// rpart[tn][row] (cpart[tm][col] likewise).  The tiles that hold a label
// also record the target logit.  ce_fused_reduce_kernel folds the partials.
__device__ __forceinline__ void ce_stats_epilogue(const GemmArgs& g, f32x4 (&acc)[4][4], const float (&row_scale)[4][4],
                                                  const float (&col_scale)[4], float alpha, int row_base, int col_base,
                                                  char* lds, int tm, int tn, int m0, int n0) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = (row_base + i * 16 + r < g.M) && (col_base + j * 16 < g.N);
        acc[i][j][r] = ok ? (acc[i][j][r] * row_scale[i][r]) * (alpha * col_scale[j]) : -INFINITY;
      }
  const int dbase = col_base - row_base;   // col - row of acc[0][0][0]
  // target logits: only tiles crossing a label diagonal (uniform tests)
  if (m0 + g.off_r < n0 + BN && m0 + BM - 1 + g.off_r >= n0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = 0.f;
        bool hit = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool h = dbase + 16 * (j - i) - r == g.off_r && acc[i][j][r] != -INFINITY;
          t = h ? acc[i][j][r] : t;
          hit = hit || h;
        }
        if (hit) g.tgt_r[row_base + i * 16 + r] = t;
      }
  }
  const bool cols = g.cpart != nullptr;
  if (cols && n0 + g.off_c < m0 + BM && n0 + BN - 1 + g.off_c >= m0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float t = 0.f;
      bool hit = false;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool h = dbase + 16 * (j - i) - r == -g.off_c && acc[i][j][r] != -INFINITY;
          t = h ? acc[i][j][r] : t;
          hit = hit || h;
        }
      if (hit) g.tgt_c[col_base + j * 16] = t;
    }
  }

  // rows: 16 entries (k = 4i + r) per lane over its 4 columns, then 4 exchange steps
  float rm[16], rs[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int i = k >> 2, r = k & 3;
    const float m = fmaxf(fmaxf(acc[i][0][r], acc[i][1][r]), fmaxf(acc[i][2][r], acc[i][3][r]));
    const float mr = m == -INFINITY ? 0.f : m;
    rm[k] = m;
    rs[k] = (__expf(acc[i][0][r] - mr) + __expf(acc[i][1][r] - mr)) + (__expf(acc[i][2][r] - mr) + __expf(acc[i][3][r] - mr));
  }
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const int o = 8 >> st;               // partner lane distance == entries kept
    const bool hi = (lane & o) != 0;
#pragma unroll
    for (int k = 0; k < o; ++k) {
      const float sm = hi ? rm[k] : rm[k + o], ss = hi ? rs[k] : rs[k + o];
      float km = hi ? rm[k + o] : rm[k], ks = hi ? rs[k + o] : rs[k];
      lse_merge(km, ks, __shfl_xor(sm, o), __shfl_xor(ss, o));
      rm[k] = km;
      rs[k] = ks;
    }
  }
  // lane now holds row entry k = lane & 15 of its 16-lane group, over the wave's 64 columns
  // columns: 4 entries (j) per lane over its 16 rows, then 2 exchange steps across the lane groups
  float cm[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY}, cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4 && cols; ++j) {
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) m = fmaxf(m, acc[i][j][r]);
    const float mr = m == -INFINITY ? 0.f : m;
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) sum += __expf(acc[i][j][r] - mr);
    cm[j] = m;
    cs[j] = sum;
  }
  if (cols) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int o = 2 >> st, ol = 32 >> st;
      const bool hi = (lane & ol) != 0;
#pragma unroll
      for (int k = 0; k < o; ++k) {
        const float sm = hi ? cm[k] : cm[k + o], ss = hi ? cs[k] : cs[k + o];
        float km = hi ? cm[k + o] : cm[k], ks = hi ? cs[k + o] : cs[k];
        lse_merge(km, ks, __shfl_xor(sm, ol), __shfl_xor(ss, ol));
        cm[k] = km;
        cs[k] = ks;
      }
    }
  }
  // lane holds column entry j = lane >> 4

  float2* rowp = reinterpret_cast<float2*>(lds);          // [4 waves][64 rows]
  float2* colp = rowp + 4 * 64;                            // [4 waves][64 cols]
  __syncthreads();                                         // main-loop LDS reads done
  {
    const int k = lane & 15;
    rowp[w * 64 + (k >> 2) * 16 + 4 * (lane >> 4) + (k & 3)] = make_float2(rm[0], rs[0]);
    colp[w * 64 + (lane >> 4) * 16 + (lane & 15)] = make_float2(cm[0], cs[0]);
  }
  __syncthreads();
  if (wc == 0) {            // waves 0, 2: rows of their half, both column halves
    float2 a = rowp[w * 64 + lane];
    const float2 b = rowp[(w + 1) * 64 + lane];
    lse_merge(a.x, a.y, b.x, b.y);
    const int row = m0 + wr * 64 + lane;
    if (row < g.M) g.rpart[(int64_t)tn * g.M + row] = a;
  }
  if (cols && wr == 0) {    // waves 0, 1: columns of their half, both row halves
    float2 a = colp[w * 64 + lane];
    const float2 b = colp[(w + 2) * 64 + lane];
    lse_merge(a.x, a.y, b.x, b.y);
    const int col = n0 + wc * 64 + lane;
    if (col < g.N) g.cpart[(int64_t)tm * g.N + col] = a;
  }
}

// kEpi 0: C = alpha * sa * sb * A B^T.  kEpi 1 / 2: the same tile feeds a fused
// softmax cross-entropy epilogue instead (statistics / gradient, see below).
template <typename TIn, typename TOut, bool kAligned, int kEpi>
__global__ __launch_bounds__(256) void gemm_nt_kernel(const GemmArgs g) {
  constexpr int E = (int)sizeof(TIn);
  constexpr int BK = kRowBytes / E;       // K elements per slice: 32 (bf16) or 16 (fp32)
  constexpr int V = 16 / E;               // elements per 16-B vector
  __shared__ __attribute__((aligned(16))) char lds[4 * kTileBytes];   // A0 B0 A1 B1

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  // Each XCD gets a contiguous range of tile ids (xcd_remap); inside it, tiles
  // go in groups of kGroupM tile rows swept column by column, so the
  // workgroups resident on one XCD at a time share ~8 A row blocks and a
  // dozen B column blocks in that XCD's 4 MB L2 instead of streaming all of B
  // (C5: 8192 x 512 fp8 = 4 MB per operand, each block read 64 times).
  constexpr int kGroupM = 8;
  const int bid = xcd_remap(blockIdx.x, g.tiles_m * g.tiles_n);
  const int first_m = (bid / (kGroupM * g.tiles_n)) * kGroupM;
  const int gm = min(g.tiles_m - first_m, kGroupM);
  const int local = bid % (kGroupM * g.tiles_n);
  const int tm = first_m + local % gm, tn = local / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const TIn* __restrict__ A = reinterpret_cast<const TIn*>(g.A);
  const TIn* __restrict__ B = reinterpret_cast<const TIn*>(g.B);

  // each thread moves 2 vectors of A and 2 of B per slice: v = tid + 256*i -> row v/4, chunk v%4
  uint4 ra[2], rb[2];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + 256 * i;
      const int r = v >> 2, c = v & 3;
      const int kk = k0 + c * V;
      const int am = m0 + r, bn = n0 + r;
      if constexpr (E == 1) {   // fp8: K % 16 == 0 and 16-B rows (host-checked)
        ra[i] = (am < g.M && kk < g.K) ? ld16(A + (int64_t)am * g.lda + kk) : make_uint4(0u, 0u, 0u, 0u);
        rb[i] = (bn < g.N && kk < g.K) ? ld16(B + (int64_t)bn * g.ldb + kk) : make_uint4(0u, 0u, 0u, 0u);
      } else if (kAligned && kk + V <= g.K) {
        ra[i] = am < g.M ? ld16(A + (int64_t)am * g.lda + kk) : make_uint4(0u, 0u, 0u, 0u);
        rb[i] = bn < g.N ? ld16(B + (int64_t)bn * g.ldb + kk) : make_uint4(0u, 0u, 0u, 0u);
      } else {
        const int nv = max(0, min(V, g.K - kk));
        ra[i] = am < g.M ? ld16_masked(A + (int64_t)am * g.lda + kk, nv) : make_uint4(0u, 0u, 0u, 0u);
        rb[i] = bn < g.N ? ld16_masked(B + (int64_t)bn * g.ldb + kk, nv) : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  };
  auto store = [&](int buf) {
    char* la = lds + (2 * buf) * kTileBytes;
    char* lb = la + kTileBytes;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + 256 * i;
      const int r = v >> 2, c = v & 3;
      st16(la + r * kLdsStride + c * 16, ra[i]);
      st16(lb + r * kLdsStride + c * 16, rb[i]);
    }
  };

  // epilogue scale factors loaded up front: their latency hides under the K loop
  // instead of sitting in the epilogue's dependency chain
  const float alpha = g.alpha_dev ? *g.alpha_dev : g.alpha;
  float col_scale[4], row_scale[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wc * 64 + j * 16 + (lane & 15);
    col_scale[j] = (g.sb && col < g.N) ? g.sb[col] : 1.f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wr * 64 + i * 16 + 4 * (lane >> 4) + r;
      row_scale[i][r] = (g.sa && row < g.M) ? g.sa[row] : 1.f;
    }

  // gradient epilogue inputs, also loaded before the K loop
  float lr[4][4], lcol[4], gout = 1.f;
  if constexpr (kEpi == 2) {
    gout = g.gout_dev ? *g.gout_dev : 1.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wc * 64 + j * 16 + (lane & 15);
      lcol[j] = (g.lse_c && col < g.N) ? g.lse_c[col] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * 64 + i * 16 + 4 * (lane >> 4) + r;
        lr[i][r] = (g.lse_r && row < g.M) ? g.lse_r[row] : 0.f;
      }
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) load((ks + 1) * BK);
    const char* la = lds + (2 * buf) * kTileBytes;
    const char* lb = la + kTileBytes;
    if constexpr (E == 2) {
      // lane: row (l & 15) of each 16-row tile, k = 8*(l>>4) .. +7 of the 32-wide slice
      bf16x8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = *reinterpret_cast<const bf16x8*>(la + (wr * 64 + i * 16 + (lane & 15)) * kLdsStride + (lane >> 4) * 16);
        bf[i] = *reinterpret_cast<const bf16x8*>(lb + (wc * 64 + i * 16 + (lane & 15)) * kLdsStride + (lane >> 4) * 16);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    } else if constexpr (E == 1) {
      // fp8: lane reads 16 bytes = k 16*(l>>4) .. +15 of the 64-wide slice and feeds
      // bytes 0-7 to k-step 0 and 8-15 to k-step 1.  A and B use the same lane -> k
      // map, so each k of the slice is paired once (the sum is order-free in k).
      uint4 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = *reinterpret_cast<const uint4*>(la + (wr * 64 + i * 16 + (lane & 15)) * kLdsStride + (lane >> 4) * 16);
        bf[i] = *reinterpret_cast<const uint4*>(lb + (wc * 64 + i * 16 + (lane & 15)) * kLdsStride + (lane >> 4) * 16);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const long a8 = h ? (long)(((uint64_t)af[i].w << 32) | af[i].z) : (long)(((uint64_t)af[i].y << 32) | af[i].x);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const long b8 = h ? (long)(((uint64_t)bf[j].w << 32) | bf[j].z) : (long)(((uint64_t)bf[j].y << 32) | bf[j].x);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a8, b8, acc[i][j], 0, 0, 0);
          }
        }
    } else {
      // exact fp32: 4 MFMA K-steps of 4; lane holds A[row l&15][k = 4s + (l>>4)]
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        float af[4], bf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          af[i] = *reinterpret_cast<const float*>(la + (wr * 64 + i * 16 + (lane & 15)) * kLdsStride + (4 * s + (lane >> 4)) * 4);
          bf[i] = *reinterpret_cast<const float*>(lb + (wc * 64 + i * 16 + (lane & 15)) * kLdsStride + (4 * s + (lane >> 4)) * 4);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
    }
    if (ks + 1 < nk) {
      __syncthreads();  // everyone done reading the other buffer (two slices ago)
      store(buf ^ 1);
      __syncthreads();
    }
  }

  // Accumulator map (16x16 MFMA C/D): acc[i][j][r] is row wr*64 + i*16 + 4*(lane>>4) + r,
  // column wc*64 + j*16 + (lane & 15) of the tile.
  const int row_base = m0 + wr * 64 + 4 * (lane >> 4), col_base = n0 + wc * 64 + (lane & 15);
  if constexpr (kEpi == 1) {
    ce_stats_epilogue(g, acc, row_scale, col_scale, alpha, row_base, col_base, lds, tm, tn, m0, n0);
    return;
  }
  if constexpr (kEpi == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = (acc[i][j][r] * row_scale[i][r]) * (alpha * col_scale[j]);
  } else {
    // G = gout * (coef_r (softmax_row - onehot) + coef_c (softmax_col - onehot)) from the
    // recomputed logits; the labels are diagonals of col - row, so one integer compare each.
    const bool has_r = g.lse_r != nullptr, has_c = g.lse_c != nullptr;
    const float gmul = g.g_times_alpha ? gout * alpha : gout;
    const int dbase = col_base - row_base;
    float dsum = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = (acc[i][j][r] * row_scale[i][r]) * (alpha * col_scale[j]);
          const int d = dbase + 16 * (j - i) - r;
          float gv = 0.f;
          if (has_r) gv = g.coef_r * (__expf(v - lr[i][r]) - (d == g.off_r ? 1.f : 0.f));
          if (has_c) gv = fmaf(g.coef_c, __expf(v - lcol[j]) - (d == -g.off_c ? 1.f : 0.f), gv);
          const bool ok = (row_base + i * 16 + r < g.M) && (col_base + j * 16 < g.N);
          gv = ok ? gv : 0.f;
          dsum = fmaf(gv, v, dsum);
          acc[i][j][r] = gv * gmul;
        }
    if (g.gpart) {
      __shared__ float red[4];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) dsum += __shfl_xor(dsum, o);
      if (lane == 0) red[w] = dsum * gout;
      __syncthreads();
      if (tid == 0) g.gpart[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
    }
  }

  TOut* __restrict__ C = reinterpret_cast<TOut*>(g.C);
  // Epilogue through LDS.  The 16x16 MFMA C/D map (col = lane & 15, row =
  // 4*(lane >> 4) + r) would make every store instruction write 64-B pieces of
  // four rows; instead each wave stages 32 x 64 of its results at a time
  // (68-float padded rows: conflict-free both ways) and writes them back as
  // 16-B vectors, 16 lanes per 256-B row segment (the two column waves of a
  // tile complete each 512-B row).  For the N x N logits (C5: 268 MB fp32)
  // this store stream is the kernel's HBM side.
  constexpr int kEpStride = 68;
  __syncthreads();                                          // main-loop LDS reads done
  float* ep = reinterpret_cast<float*>(lds) + w * (32 * kEpStride);
  const bool full = g.c_vec && (m0 + BM <= g.M) && (n0 + BN <= g.N);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2) {
      const int i = 2 * p + i2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col_l = j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row_l = i2 * 16 + 4 * (lane >> 4) + r;
          ep[row_l * kEpStride + col_l] = acc[i][j][r];
        }
      }
    }
    __syncthreads();
    if constexpr (sizeof(TOut) == 4) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {      // 4 floats per lane, 16 lanes per row segment
        const int q = lane + 64 * t;
        const int row_l = q >> 4, c4 = (q & 15) * 4;
        const f32x4 v = *reinterpret_cast<const f32x4*>(ep + row_l * kEpStride + c4);
        const int row = m0 + wr * 64 + p * 32 + row_l, col = n0 + wc * 64 + c4;
        TOut* dst = C + (int64_t)row * g.ldc + col;
        if (full) {
#if MC_NT_STORE
          __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst));   // streamed: nothing re-reads it here
#else
          *reinterpret_cast<f32x4*>(dst) = v;
#endif
        } else if (row < g.M) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e < g.N) dst[e] = from_f<TOut>(v[e]);
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {      // 8 values -> one 16-B store per lane, 8 lanes per row segment
        const int q = lane + 64 * t;
        const int row_l = q >> 3, c8 = (q & 7) * 8;
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + row_l * kEpStride + c8);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + row_l * kEpStride + c8 + 4);
        const int row = m0 + wr * 64 + p * 32 + row_l, col = n0 + wc * 64 + c8;
        TOut* dst = C + (int64_t)row * g.ldc + col;
        if (full && g.c_vec16) {
          const u32x4_t pk = {bits16<TOut>(v0[0]) | (bits16<TOut>(v0[1]) << 16),
                              bits16<TOut>(v0[2]) | (bits16<TOut>(v0[3]) << 16),
                              bits16<TOut>(v1[0]) | (bits16<TOut>(v1[1]) << 16),
                              bits16<TOut>(v1[2]) | (bits16<TOut>(v1[3]) << 16)};
#if MC_NT_STORE
          __builtin_nontemporal_store(pk, reinterpret_cast<u32x4_t*>(dst));
#else
          *reinterpret_cast<u32x4_t*>(dst) = pk;
#endif
        } else if (row < g.M) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (col + e < g.N) dst[e] = from_f<TOut>(e < 4 ? v0[e] : v1[e - 4]);
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ fp8 similarity (config 5)
// C = alpha * sa[m] * sb[n] * A B^T for fp8 e4m3 rows with K % 128 == 0 (the C5 similarity:
// N = 8192, K = E = 512).  Same 128 x 128 tile / 4-wave decomposition as gemm_nt_kernel, but:
//  * K steps of 128 bytes on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (unit block
//    scales): twice the non-scaled fp8 MFMA rate, 16 MFMAs per wave and step;
//  * operands land in LDS by global_load_lds (16 B per lane, no VGPR round trip), two steps in
//    flight, waited with a counted vmcnt and a raw s_barrier (no vmcnt(0) drain per step);
//  * the LDS image is lane-linear (glds), so the bank swizzle sits on the SOURCE chunk and the
//    matching read: chunk c of row r lives at slot c ^ ((r >> 1) & 7) -- sixteen consecutive rows
//    reading one chunk hit sixteen distinct 4-bank groups;
//  * plain (not non-temporal) 16-B epilogue stores: the 268 MB fp32 logit matrix streams at
//    6.9 TB/s with plain stores vs 5.2-5.9 non-temporal (tools/ubench/hbm_rw.hip).
constexpr int kSBK = 128;                      // K bytes per step
constexpr int kSStage = 2 * BM * kSBK;         // A + B bytes per stage (32 KB)
typedef int i32x8 __attribute__((ext_vector_type(8)));

// One global_load_lds_dwordx4: 16 B per lane from gsrc to LDS byte address m0v + 16 * lane
// (m0v wave-uniform).  Written as asm so hipcc does not track it: its waitcnt pass would otherwise
// drain every in-flight LDS-DMA with vmcnt(0) before the first ds_read of each K step.  The caller
// counts completion with its own vmcnt.  M0 is compiler-reserved: saved and restored in the statement.
__device__ __forceinline__ void glds16_asm(const void* gsrc, uint32_t m0v) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(m0v) : "memory");
}

template <typename TOut>
__global__ __launch_bounds__(256, 2) void sim_fp8_kernel(const GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char lds[2 * kSStage];   // the only LDS object (glds + epilogue)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  constexpr int kGroupM = 8;
  const int bid = xcd_remap(blockIdx.x, g.tiles_m * g.tiles_n);
  const int first_m = (bid / (kGroupM * g.tiles_n)) * kGroupM;
  const int gm = min(g.tiles_m - first_m, kGroupM);
  const int local = bid % (kGroupM * g.tiles_n);
  const int tm = first_m + local % gm, tn = local / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const uint8_t* __restrict__ A = reinterpret_cast<const uint8_t*>(g.A);
  const uint8_t* __restrict__ B = reinterpret_cast<const uint8_t*>(g.B);

  // glds: wave w, instruction j, lane l -> chunk q = (4w + j) * 64 + l of a 128-row slice image:
  // row q >> 3, slot q & 7, loading the row's chunk (slot ^ swz(row)) (rows past M / N clamped)
  const uint8_t* srcA[4];
  const uint8_t* srcB[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = (4 * w + j) * 64 + lane, r = q >> 3, slot = q & 7;
    const int c = slot ^ ((r >> 1) & 7);
    srcA[j] = A + (int64_t)min(m0 + r, g.M - 1) * g.lda + c * 16;
    srcB[j] = B + (int64_t)min(n0 + r, g.N - 1) * g.ldb + c * 16;
  }
  typedef __attribute__((address_space(3))) char lds_char;
  const uint32_t lds_w = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)(lds) + 4 * 1024 * w);
  auto issue = [&](int step) __attribute__((always_inline)) {   // one K step into buffer step & 1
    const uint32_t la = lds_w + (step & 1) * kSStage, lb = la + BM * kSBK;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      glds16_asm(srcA[j] + step * kSBK, la + j * 1024);
      glds16_asm(srcB[j] + step * kSBK, lb + j * 1024);
    }
  };

  const float alpha = g.alpha_dev ? *g.alpha_dev : g.alpha;
  float col_scale[4], row_scale[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wc * 64 + j * 16 + (lane & 15);
    col_scale[j] = (g.sb && col < g.N) ? g.sb[col] : 1.f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wr * 64 + i * 16 + 4 * (lane >> 4) + r;
      row_scale[i][r] = (g.sa && row < g.M) ? g.sa[row] : 1.f;
    }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#if MC_SIM_EXP == 2
  const int nk = 0;
#else
  const int nk = g.K / kSBK;
#endif
  if (nk > 0) issue(0);
  if (nk > 1) issue(1);
  // fragment read offsets: lane row (l & 15) of a 16-row tile, K bytes [32 (l >> 4), +32) = chunks 2g, 2g + 1
  const int fr = lane & 15, fg = lane >> 4;
  for (int s = 0; s < nk; ++s) {
    // this wave's glds of step s done (step s + 1's 8 may stay in flight), then everyone's
    if (s + 1 < nk) __builtin_amdgcn_s_waitcnt(0x0F78);   // vmcnt(8)
    else __builtin_amdgcn_s_waitcnt(0x0F70);              // vmcnt(0)
    __builtin_amdgcn_s_barrier();
    const char* la = lds + (s & 1) * kSStage;
    const char* lb = la + BM * kSBK;
    i32x8 af[4], bf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ra = wr * 64 + i * 16 + fr, rb = wc * 64 + i * 16 + fr;
      const int sa = (ra >> 1) & 7, sb = (rb >> 1) & 7;
      const uint4 a0 = *reinterpret_cast<const uint4*>(la + ra * kSBK + (((2 * fg) ^ sa) << 4));
      const uint4 a1 = *reinterpret_cast<const uint4*>(la + ra * kSBK + (((2 * fg + 1) ^ sa) << 4));
      const uint4 b0 = *reinterpret_cast<const uint4*>(lb + rb * kSBK + (((2 * fg) ^ sb) << 4));
      const uint4 b1 = *reinterpret_cast<const uint4*>(lb + rb * kSBK + (((2 * fg + 1) ^ sb) << 4));
      af[i] = i32x8{(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
      bf[i] = i32x8{(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bf[j], acc[i][j], 0, 0, 0, 127, 0, 127);
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's fragment reads are done
    __builtin_amdgcn_s_barrier();         // ... and everyone's: the buffer can be refilled
    if (s + 2 < nk) issue(s + 2);
  }

#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = (acc[i][j][r] * row_scale[i][r]) * (alpha * col_scale[j]);

  // epilogue through LDS (as gemm_nt_kernel): 32 x 64 per wave and pass, 16-B stores
  TOut* __restrict__ C = reinterpret_cast<TOut*>(g.C);
  constexpr int kEpStride = 68;
  float* ep = reinterpret_cast<float*>(lds) + w * (32 * kEpStride);
  const bool full = g.c_vec && (m0 + BM <= g.M) && (n0 + BN <= g.N);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ep[(i2 * 16 + 4 * (lane >> 4) + r) * kEpStride + j * 16 + (lane & 15)] = acc[2 * p + i2][j][r];
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if constexpr (sizeof(TOut) == 4) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int q = lane + 64 * t;
        const int row_l = q >> 4, c4 = (q & 15) * 4;
        const f32x4 v = *reinterpret_cast<const f32x4*>(ep + row_l * kEpStride + c4);
        const int row = m0 + wr * 64 + p * 32 + row_l, col = n0 + wc * 64 + c4;
        TOut* dst = C + (int64_t)row * g.ldc + col;
#if MC_SIM_EXP == 1
        if (v[0] == 1234.5f) *reinterpret_cast<f32x4*>(dst) = v;
#else
        if (full) {
          *reinterpret_cast<f32x4*>(dst) = v;
        } else if (row < g.M) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e < g.N) dst[e] = v[e];
        }
#endif
      }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int q = lane + 64 * t;
        const int row_l = q >> 3, c8 = (q & 7) * 8;
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + row_l * kEpStride + c8);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + row_l * kEpStride + c8 + 4);
        const int row = m0 + wr * 64 + p * 32 + row_l, col = n0 + wc * 64 + c8;
        TOut* dst = C + (int64_t)row * g.ldc + col;
        if (full && g.c_vec16) {
          *reinterpret_cast<uint4*>(dst) = make_uint4(cvt_pk2<TOut>(v0[0], v0[1]), cvt_pk2<TOut>(v0[2], v0[3]),
                                                      cvt_pk2<TOut>(v1[0], v1[1]), cvt_pk2<TOut>(v1[2], v1[3]));
        } else if (row < g.M) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (col + e < g.N) dst[e] = from_f<TOut>(e < 4 ? v0[e] : v1[e - 4]);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // this wave's staging reads done before the next pass writes
  }
}

// ------------------------------------------------------------------ fp8 similarity, panel kernel (round 6)
// The C5 shape (K = E <= 512) has 4 MFMA K-steps of 128 bytes per output tile: sim_fp8_kernel's
// 128 x 128 tiles re-stream both operands from L2 for every tile (537 MB of LDS-DMA per call at
// N = 8192) and expose each tile's epilogue.  Here a workgroup (8 waves, one per CU) owns a 256-row
// PANEL of A and a range of 64-column tiles of B:
//  * the panel lives in registers for the whole launch: wave w keeps rows 64 (w & 3) .. +63 as
//    v_mfma_scale_f32_32x32x64_f8f6f4 B-operand fragments (2 row blocks x K/64 steps x 32 B per lane =
//    128 VGPRs at K = 512); A is read once per panel and n-range (32 MB at C5 instead of 268 MB);
//  * B tiles (64 rows x K bytes) stream through a two-stage LDS image by LDS-DMA, one tile ahead,
//    retired by a counted vmcnt and one raw s_barrier per tile (the swizzle sits on the source chunk,
//    slot = chunk ^ (row & 15): a fragment read of 8 consecutive rows hits 8 distinct bank groups);
//  * waves 0-3 take tile columns 0-31, waves 4-7 columns 32-63: 2 x 1 MFMAs of 32 x 32 per K-step,
//    with the B tile as the MFMA's A operand so each lane ends with 4 consecutive COLUMNS of one output
//    row per accumulator group (C^T orientation);
//  * epilogue through a per-wave LDS block (row stride 36 floats: conflict-free 16-B writes and reads),
//    scaled by the row factor (registers) and alpha x the column factor (LDS, loaded once), written as
//    whole 128-B (fp32) / 64-B (bf16) row pieces with buffer stores -- always the same number of store
//    instructions per tile (masked lanes address past the buffer), so the next tile's vmcnt is static;
//    the stores stay in flight under the next tile's MFMAs (two waves per SIMD).
// Grid: one workgroup per (panel, n-range), n-ranges sized for ~256 workgroups; consecutive logical
// workgroups (xcd_remap) share an n-range, so one XCD's L2 serves that range's B tiles to its panels.
constexpr int kP8Rows = 256;                 // panel rows per workgroup
constexpr int kP8Cols = 64;                  // B tile columns
constexpr int kP8Row = 512;                  // LDS bytes per B row (K <= 512)
constexpr int kP8Stage = kP8Cols * kP8Row;   // 32 KB
constexpr int kP8EpStride = 36;              // floats per staged output row (32 + 4 pad)
constexpr int kP8EpWave = 64 * kP8EpStride;  // floats per wave
constexpr int kP8MaxTiles = 32;              // tiles per workgroup (column factors held in LDS)
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <typename TOut, int NKS>
__global__ __launch_bounds__(512, 1) void sim8_panel_kernel(const GemmArgs g, int nr, int tpr, int ilv) {
  __shared__ __attribute__((aligned(16))) char lds[2 * kP8Stage + 8 * kP8EpWave * 4 + kP8MaxTiles * kP8Cols * 4];
  float* ep_all = reinterpret_cast<float*>(lds + 2 * kP8Stage);
  float* colf = ep_all + 8 * kP8EpWave;        // alpha * column factor of the workgroup's columns
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rg = w & 3, cg = w >> 2;
  const int lin = xcd_remap(blockIdx.x, g.tiles_m * nr);
  const int nrange = lin / g.tiles_m, panel = lin % g.tiles_m;
  const int m0 = panel * kP8Rows;
  const int ntiles = (g.N + kP8Cols - 1) / kP8Cols;
  // the workgroup's B tiles: j = 0 .. cnt - 1 -> tile_of(j); contiguous (t0 + j) or, with ilv, every nr-th
  // (nrange + j nr: the n-ranges of one panel then write neighbouring 256-B row pieces at the same time)
  const int t0 = ilv ? nrange : nrange * tpr;
  const int cnt = ilv ? max(0, (ntiles - nrange + nr - 1) / nr) : max(0, min(ntiles, t0 + tpr) - t0);
  const int tstep = ilv ? nr : 1;
  if (cnt <= 0) return;   // uniform across the workgroup
  const uint8_t* __restrict__ A = reinterpret_cast<const uint8_t*>(g.A);
  const uint8_t* __restrict__ B = reinterpret_cast<const uint8_t*>(g.B);
  constexpr int kChunks = 4 * NKS;             // 16-B chunks of a row (K = 64 NKS bytes)

  // ---- A panel fragments (B operand of the MFMA: lane = row l & 31, K bytes [32 (l >> 5), +32) per step)
  i32x8 af[2][NKS];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int row = min(m0 + rg * 64 + rb * 32 + (lane & 31), g.M - 1);
    const uint8_t* ap = A + (int64_t)row * g.lda + 32 * (lane >> 5);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const uint4 lo = *reinterpret_cast<const uint4*>(ap + ks * 64);
      const uint4 hi = *reinterpret_cast<const uint4*>(ap + ks * 64 + 16);
      af[rb][ks] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
  }
  // ---- row factors of the rows this lane writes in the epilogue; column factors (x alpha) -> LDS
  constexpr int kRowsPerStore = sizeof(TOut) == 4 ? 8 : 16;       // output rows per store instruction
  constexpr int kStores = 64 / kRowsPerStore;                     // store instructions per tile and wave
  const int er = sizeof(TOut) == 4 ? (lane >> 3) : (lane >> 2);   // row within a store's row group
  const int ec = sizeof(TOut) == 4 ? 4 * (lane & 7) : 8 * (lane & 3);   // first column (of the wave's 32)
  float rsf[kStores];
#pragma unroll
  for (int j = 0; j < kStores; ++j) {
    const int m = m0 + rg * 64 + j * kRowsPerStore + er;
    rsf[j] = (g.sa && m < g.M) ? g.sa[m] : 1.f;
  }
  {
    const float alpha = g.alpha_dev ? *g.alpha_dev : g.alpha;
    const int ncols = cnt * kP8Cols;
    for (int i = tid; i < ncols; i += 512) {
      const int n = (t0 + (i / kP8Cols) * tstep) * kP8Cols + i % kP8Cols;
      colf[i] = alpha * ((g.sb && n < g.N) ? g.sb[n] : 1.f);
    }
  }

  // ---- B tile LDS-DMA: wave w, instruction j, lane l -> chunk q = (4w + j) * 64 + l of the 64 x 32-chunk image
  int boff[4];
  const int bslot0 = w * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = (bslot0 + j) * 64 + lane, r = q >> 5, slot = q & 31;
    boff[j] = min(slot ^ (r & 15), kChunks - 1) * 16;   // chunks past K: a valid chunk, never read
  }
  typedef __attribute__((address_space(3))) char lds_char;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)(lds));
  auto issue = [&](int tile, int st) __attribute__((always_inline)) {
    const int n0 = tile * kP8Cols;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = (bslot0 + j) * 64 + lane, r = q >> 5;
      const uint8_t* src = B + (int64_t)min(n0 + r, g.N - 1) * g.ldb + boff[j];
      glds16_asm(src, lds_base + st * kP8Stage + (bslot0 + j) * 1024);
    }
  };

  // ---- output: one buffer resource over this wave's 64 rows (masked lanes address past its end)
  TOut* __restrict__ C = reinterpret_cast<TOut*>(g.C);
  const int wrow0 = m0 + rg * 64;
  const int wrows = max(0, min(64, g.M - wrow0));
  const __amdgpu_buffer_rsrc_t rc =
      make_rsrc(C + (int64_t)min(wrow0, g.M - 1) * g.ldc,
                wrows > 0 ? (uint32_t)(((int64_t)(wrows - 1) * g.ldc + g.N) * (int64_t)sizeof(TOut)) : 0u);
  float* ep = ep_all + w * kP8EpWave;
  const int nl = cg * 32 + (lane & 31);        // this lane's B row (tile column) in the fragment reads

  issue(t0, 0);
  for (int j = 0; j < cnt; ++j) {
    const int t = t0 + j * tstep;
    const int st = j & 1;
    // this wave's DMA of tile t landed (the previous tile's kStores stores may stay in flight), this
    // wave's LDS reads of tile t - 1 are done, then everyone's: stage st is readable, st ^ 1 is free
    if (j == 0) __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0)
    else if constexpr (kStores == 8) __builtin_amdgcn_s_waitcnt(0x0078);   // vmcnt(8) lgkmcnt(0)
    else __builtin_amdgcn_s_waitcnt(0x0074);                                // vmcnt(4) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    if (j + 1 < cnt) issue(t + tstep, st ^ 1);
    asm volatile("" ::: "memory");

    const char* sb = lds + st * kP8Stage + nl * kP8Row;
    const int sw = nl & 15;
    f32x16 acc0 = {}, acc1 = {};
    auto bfrag = [&](int ks) __attribute__((always_inline)) {
      const int c0 = 4 * ks + 2 * (lane >> 5);
      const uint4 b0 = *reinterpret_cast<const uint4*>(sb + ((c0 ^ sw) << 4));
      const uint4 b1 = *reinterpret_cast<const uint4*>(sb + (((c0 + 1) ^ sw) << 4));
      return i32x8{(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
    };
    // two fragment buffers: step ks + 1's LDS reads are issued before step ks's MFMAs (sched_barrier keeps
    // the scheduler from sinking them behind the MFMAs, where they would wait for the operand read)
    i32x8 bfa = bfrag(0), bfb = bfa;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (ks + 1 < NKS) {
        if (ks & 1) bfa = bfrag(ks + 1);
        else bfb = bfrag(ks + 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      const i32x8 bcur = (ks & 1) ? bfb : bfa;
      acc0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bcur, af[0][ks], acc0, 0, 0, 0, 127, 0, 127);
      acc1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bcur, af[1][ks], acc1, 0, 0, 0, 127, 0, 127);
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- epilogue: C^T fragments -> this wave's LDS block [64 rows][32 cols] (row m = l & 31 of block rb,
    // columns 8 i + 4 (l >> 5) + [0, 4))
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = 8 * i + 4 * (lane >> 5);
      *reinterpret_cast<f32x4*>(ep + (lane & 31) * kP8EpStride + col) =
          f32x4{acc0[4 * i], acc0[4 * i + 1], acc0[4 * i + 2], acc0[4 * i + 3]};
      *reinterpret_cast<f32x4*>(ep + (32 + (lane & 31)) * kP8EpStride + col) =
          f32x4{acc1[4 * i], acc1[4 * i + 1], acc1[4 * i + 2], acc1[4 * i + 3]};
    }
    asm volatile("" ::: "memory");   // one wave's LDS operations run in program order
    const int n_w = t * kP8Cols + cg * 32 + ec;                       // first output column of this lane
    const float* cf = colf + j * kP8Cols + cg * 32 + ec;
    const bool col_ok = n_w < g.N;                                    // N % 8 == 0: whole vectors
#pragma unroll
    for (int j = 0; j < kStores; ++j) {
      const int rl = j * kRowsPerStore + er;                          // row within the wave's 64
      const bool ok = col_ok && rl < wrows;
      const uint32_t off = ok ? (uint32_t)(((int64_t)rl * g.ldc + n_w) * (int64_t)sizeof(TOut)) : 0x80000000u;
      if constexpr (sizeof(TOut) == 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(ep + rl * kP8EpStride + ec);
        const f32x4 c4 = *reinterpret_cast<const f32x4*>(cf);
        const f32x4 o = (v * rsf[j]) * c4;
        buf_st16(rc, off, make_uint4(__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]),
                                     __float_as_uint(o[3])));
      } else {
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(ep + rl * kP8EpStride + ec);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(ep + rl * kP8EpStride + ec + 4);
        const f32x4 c0 = *reinterpret_cast<const f32x4*>(cf);
        const f32x4 c1 = *reinterpret_cast<const f32x4*>(cf + 4);
        const f32x4 o0 = (v0 * rsf[j]) * c0, o1 = (v1 * rsf[j]) * c1;
        buf_st16(rc, off, make_uint4(cvt_pk2<TOut>(o0[0], o0[1]), cvt_pk2<TOut>(o0[2], o0[3]),
                                     cvt_pk2<TOut>(o1[0], o1[1]), cvt_pk2<TOut>(o1[2], o1[3])));
      }
    }
  }
}

// ------------------------------------------------------------------ CE statistics

// one wave per row: lse and nll, per-block partial NLL sums (4 rows per block)
__global__ __launch_bounds__(256) void ce_rows_kernel(int rows, int cols, const float* __restrict__ S, int64_t lds,
                                                      int64_t off, float* __restrict__ lse, float* __restrict__ nll,
                                                      float* __restrict__ partial) {
  __shared__ float pn[4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + w;
  float v = 0.f;
  if (row < rows) {
    const float* sr = S + (int64_t)row * lds;
    float m = -INFINITY, s = 0.f;
    for (int j = lane; j < cols; j += 64) {
      const float x = sr[j];
      if (x > m) { s = s * __expf(m - x) + 1.f; m = x; }
      else s += __expf(x - m);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float m2 = __shfl_xor(m, o), s2 = __shfl_xor(s, o);
      lse_merge(m, s, m2, s2);
    }
    const float l = m + __logf(s);
    const int64_t lab = row + off;
    const float tgt = (lab >= 0 && lab < cols) ? sr[lab] : 0.f;
    v = l - tgt;
    if (lane == 0) {
      lse[row] = l;
      if (nll) nll[row] = v;
    }
  }
  if (lane == 0) pn[w] = row < rows ? v : 0.f;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (pn[0] + pn[1]) + (pn[2] + pn[3]);
}

// columns: block = 64 columns x 4 row lanes, grid.y = row splits; writes (m, s) partials
__global__ __launch_bounds__(256) void ce_cols_partial_kernel(int rows, int cols, const float* __restrict__ S,
                                                              int64_t lds, int splits, float2* __restrict__ part) {
  __shared__ float2 red[4][64];
  const int cx = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cx;
  const int per = (rows + splits - 1) / splits;
  const int r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
  float m = -INFINITY, s = 0.f;
  if (col < cols) {
    for (int r = r0 + q; r < r1; r += 4) {
      const float x = S[(int64_t)r * lds + col];
      if (x > m) { s = s * __expf(m - x) + 1.f; m = x; }
      else s += __expf(x - m);
    }
  }
  red[q][cx] = make_float2(m, s);
  __syncthreads();
  if (q == 0 && col < cols) {
#pragma unroll
    for (int k = 1; k < 4; ++k) lse_merge(m, s, red[k][cx].x, red[k][cx].y);
    part[(int64_t)blockIdx.y * cols + col] = make_float2(m, s);
  }
}

__global__ __launch_bounds__(256) void ce_cols_final_kernel(int rows, int cols, const float* __restrict__ S,
                                                            int64_t lds, int splits, const float2* __restrict__ part,
                                                            int64_t off, float* __restrict__ lse,
                                                            float* __restrict__ nll, float* __restrict__ partial) {
  __shared__ float pn[256];
  const int col = blockIdx.x * 256 + threadIdx.x;
  float v = 0.f;
  if (col < cols) {
    float m = -INFINITY, s = 0.f;
    for (int k = 0; k < splits; ++k) {
      const float2 p = part[(int64_t)k * cols + col];
      lse_merge(m, s, p.x, p.y);
    }
    const float l = m + __logf(s);
    const int64_t lab = col + off;
    const float tgt = (lab >= 0 && lab < rows) ? S[lab * lds + col] : 0.f;
    v = l - tgt;
    lse[col] = l;
    if (nll) nll[col] = v;
  }
  pn[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o >= 1; o >>= 1) {
    if ((int)threadIdx.x < o) pn[threadIdx.x] += pn[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = pn[0];
}

// fixed-order sum of n partials -> out[0] = coef * sum  (one block)
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ part, int n, float coef,
                                                           const float* __restrict__ divisor, float* __restrict__ out) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o >= 1; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = coef * red[0] / (divisor ? *divisor : 1.f);
}

// Folds the fused forward's tile partials: blocks [0, nbr) take rows, the rest
// columns.  lse = m + log(s) merged over the tile partials in tile order;
// partial[block] = coef * sum(lse - target) (fixed order: deterministic).
__global__ __launch_bounds__(256) void ce_fused_reduce_kernel(int M, int N, int tiles_m, int tiles_n,
                                                              const float2* __restrict__ rpart,
                                                              const float2* __restrict__ cpart,
                                                              const float* __restrict__ tgt_r,
                                                              const float* __restrict__ tgt_c, int off_r, int off_c,
                                                              float coef_r, float coef_c, float* __restrict__ lse_r,
                                                              float* __restrict__ lse_c, int nbr,
                                                              float* __restrict__ partial) {
  __shared__ float red[256];
  const bool rows = (int)blockIdx.x < nbr;
  const int idx = (rows ? (int)blockIdx.x : (int)blockIdx.x - nbr) * 256 + threadIdx.x;
  const int n = rows ? M : N, other = rows ? N : M, parts = rows ? tiles_n : tiles_m;
  const float2* __restrict__ part = rows ? rpart : cpart;
  float v = 0.f;
  if (idx < n) {
    float m = -INFINITY, sum = 0.f;
    for (int k = 0; k < parts; ++k) {
      const float2 q = part[(int64_t)k * n + idx];
      lse_merge(m, sum, q.x, q.y);
    }
    const float l = m + __logf(sum);
    const int64_t lab = (int64_t)idx + (rows ? off_r : off_c);
    const float tgt = (lab >= 0 && lab < other) ? (rows ? tgt_r : tgt_c)[idx] : 0.f;
    (rows ? lse_r : lse_c)[idx] = l;
    v = (rows ? coef_r : coef_c) * (l - tgt);
  }
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o >= 1; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// G = gout * (coef_r (softmax_r - onehot_r) + coef_c (softmax_c - onehot_c)); partial sum(G * S)
template <typename TOut>
__global__ __launch_bounds__(256) void ce_grad_kernel(int rows, int cols, const float* __restrict__ S, int64_t lds,
                                                      const float* __restrict__ lse_r, int64_t off_r, float coef_r,
                                                      const float* __restrict__ lse_c, int64_t off_c, float coef_c,
                                                      const float* __restrict__ gout_dev, TOut* __restrict__ G,
                                                      int64_t ldg, float* __restrict__ partial) {
  __shared__ float red[256];
  const float gout = gout_dev ? *gout_dev : 1.f;
  const int64_t total = (int64_t)rows * cols;
  float acc = 0.f;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int i = (int)(idx / cols), j = (int)(idx % cols);
    const float s = S[(int64_t)i * lds + j];
    float gv = coef_r * (__expf(s - lse_r[i]) - ((int64_t)j == i + off_r ? 1.f : 0.f));
    if (lse_c) gv += coef_c * (__expf(s - lse_c[j]) - ((int64_t)i == j + off_c ? 1.f : 0.f));
    gv *= gout;
    G[(int64_t)i * ldg + j] = from_f<TOut>(gv);
    acc = fmaf(gv, s, acc);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o >= 1; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0 && partial) partial[blockIdx.x] = red[0];
}

// ------------------------------------------------------------------ fp8 quantiser
constexpr float kFp8Max = 448.f;   // e4m3fn max finite

template <typename TIn>
__global__ __launch_bounds__(256) void quant_rows_fp8_kernel(int rows, int cols, const TIn* __restrict__ X,
                                                             int64_t ldx, fp8_t* __restrict__ Q, int64_t ldq,
                                                             float* __restrict__ inv_scale) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + w;
  if (row >= rows) return;
  const TIn* xr = X + (int64_t)row * ldx;
  float amax = 0.f;
  for (int j = lane; j < cols; j += 64) amax = fmaxf(amax, fabsf(to_f(xr[j])));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
  const float s = amax > 0.f ? kFp8Max / amax : 1.f;
  if (lane == 0) inv_scale[row] = 1.f / s;
  // each lane packs 4 consecutive bytes (one dword store) per step
  uint32_t* qr = reinterpret_cast<uint32_t*>(Q + (int64_t)row * ldq);
  const int nw = (int)(ldq >> 2);
  for (int q = lane; q < nw; q += 64) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = 4 * q + e;
      v[e] = j < cols ? fminf(fmaxf(to_f(xr[j]) * s, -kFp8Max), kFp8Max) : 0.f;
    }
    int pk = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
    pk = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], pk, true);
    qr[q] = (uint32_t)pk;
  }
}

constexpr int kColSplits = 32;
constexpr int kGradGrid = 2048;

}  // namespace ctr
}  // namespace mc

using namespace mc;
using namespace mc::ctr;

namespace {
template <int kEpi>
void launch_gemm(const GemmArgs& g, int in_dtype, int out_dtype, bool aligned, hipStream_t s) {
  const dim3 grid(g.tiles_m * g.tiles_n), block(256);
#define MC_GEMM(TI, TO)                                                                         \
  do {                                                                                          \
    if (aligned) hipLaunchKernelGGL((gemm_nt_kernel<TI, TO, true, kEpi>), grid, block, 0, s, g); \
    else hipLaunchKernelGGL((gemm_nt_kernel<TI, TO, false, kEpi>), grid, block, 0, s, g);       \
  } while (0)
  if (in_dtype == MC_DTYPE_BF16) {
    if (out_dtype == MC_DTYPE_F32) MC_GEMM(bf16_t, float); else MC_GEMM(bf16_t, bf16_t);
  } else if (in_dtype == MC_DTYPE_FP8_E4M3) {
    if (out_dtype == MC_DTYPE_F32) MC_GEMM(fp8_t, float); else MC_GEMM(fp8_t, bf16_t);
  } else {
    if (out_dtype == MC_DTYPE_F32) MC_GEMM(float, float); else MC_GEMM(float, bf16_t);
  }
#undef MC_GEMM
}

// The panel kernel's eligibility: K % 64 == 0, K <= 512; whole 16-B output vectors (N % 8, ldc % 8 and a
// 16-B aligned C); 32-bit buffer offsets over the output.  MAMBA_CLIP_AMD_SIM8_PANEL=0 keeps the
// 128 x 128 tile kernel (A/B).
bool sim8_panel_ok(const GemmArgs& g, const mc_gemm_nt_params* p) {
  static const bool on = [] {
    const char* e = getenv("MAMBA_CLIP_AMD_SIM8_PANEL");
    return !(e && e[0] == '0');
  }();
  const int es = p->out_dtype == MC_DTYPE_F32 ? 4 : 2;
  return on && p->K > 0 && p->K % 64 == 0 && p->K <= kP8Row && p->N % 8 == 0 && p->ldc % 8 == 0 && aligned16(p->C) &&
         (int64_t)p->M * p->ldc * es < ((int64_t)1 << 31);
}

template <typename TOut>
void launch_sim8_panel_t(const GemmArgs& g0, hipStream_t s) {
  GemmArgs g = g0;
  g.tiles_m = (g.M + kP8Rows - 1) / kP8Rows;   // panels
  const int ntiles = (g.N + kP8Cols - 1) / kP8Cols;
  int nr = std::max((256 + g.tiles_m - 1) / g.tiles_m, (ntiles + kP8MaxTiles - 1) / kP8MaxTiles);
  nr = std::min(nr, ntiles);
  const int tpr = (ntiles + nr - 1) / nr;
  nr = (ntiles + tpr - 1) / tpr;               // no empty n-ranges
  const dim3 grid(g.tiles_m * nr), block(512);
  // interleaved n-ranges for fp32 logits (C5: 87 -> 70 us, the 8 n-ranges of a panel write one 2-KB row
  // piece per tile step instead of eight 256-B pieces 4 KB apart); bf16 logits keep contiguous ranges
  // (51.6 vs 60 us in a launch loop, equal under graph replay: profiles/r06/c5/interleave_ab.txt).
  // MAMBA_CLIP_AMD_SIM8_INTERLEAVE=0 / 1 forces either (A/B).
  static const int env_ilv = [] {
    const char* e = getenv("MAMBA_CLIP_AMD_SIM8_INTERLEAVE");
    return e ? (e[0] == '0' ? 0 : 1) : -1;
  }();
  const int ilv = env_ilv >= 0 ? env_ilv : (sizeof(TOut) == 4 ? 1 : 0);
  switch (g.K / 64) {
#define MC_P8(NK) case NK: hipLaunchKernelGGL((sim8_panel_kernel<TOut, NK>), grid, block, 0, s, g, nr, tpr, ilv); break;
    MC_P8(1) MC_P8(2) MC_P8(3) MC_P8(4) MC_P8(5) MC_P8(6) MC_P8(7) MC_P8(8)
#undef MC_P8
    default: break;
  }
}
void launch_sim8_panel(const GemmArgs& g, int out_dtype, hipStream_t s) {
  if (out_dtype == MC_DTYPE_F32) launch_sim8_panel_t<float>(g, s);
  else launch_sim8_panel_t<bf16_t>(g, s);
}

// shape / alignment checks shared by the plain GEMM and the fused CE entry points
int fill_operands(GemmArgs& g, const char* who, int M, int N, int K, int in_dtype, const void* A, int64_t lda,
                  const void* B, int64_t ldb, bool& aligned) {
  MC_CHECK(M > 0 && N > 0 && K >= 0, MC_ERR_SHAPE, "%s: bad shape", who);
  MC_CHECK(in_dtype == MC_DTYPE_BF16 || in_dtype == MC_DTYPE_F32 || in_dtype == MC_DTYPE_FP8_E4M3, MC_ERR_DTYPE,
           "%s: inputs must be bf16, fp32 or fp8 e4m3", who);
  MC_CHECK(A && B, MC_ERR_INVALID, "%s: null operand", who);
  g = GemmArgs{};
  g.M = M; g.N = N; g.K = K;
  g.A = A; g.lda = lda; g.B = B; g.ldb = ldb;
  g.tiles_m = (M + BM - 1) / BM;
  g.tiles_n = (N + BN - 1) / BN;
  const int eb = in_dtype == MC_DTYPE_F32 ? 4 : (in_dtype == MC_DTYPE_FP8_E4M3 ? 1 : 2);
  const int64_t v = 16 / eb;
  aligned = aligned16(A) && aligned16(B) && lda % v == 0 && ldb % v == 0;
  if (eb == 1)
    MC_CHECK(aligned && K % 16 == 0, MC_ERR_SHAPE,
             "%s: fp8 operands need K, lda, ldb multiples of 16 and 16-B aligned rows", who);
  return MC_OK;
}
}  // namespace

extern "C" int32_t mc_gemm_nt_kernel(const mc_gemm_nt_params* p) {
  if (!p || p->M <= 0 || p->N <= 0) return 0;
  GemmArgs g;
  bool aligned;
  if (fill_operands(g, "mc_gemm_nt_kernel", p->M, p->N, p->K, p->in_dtype, p->A, p->lda, p->B, p->ldb, aligned) != MC_OK)
    return 0;
  if (p->in_dtype == MC_DTYPE_FP8_E4M3 && sim8_panel_ok(g, p)) return MC_GEMM_KERNEL_FP8_PANEL;
  if (p->in_dtype == MC_DTYPE_FP8_E4M3 && p->K % kSBK == 0 && p->K > 0) return MC_GEMM_KERNEL_FP8_TILE;
  return MC_GEMM_KERNEL_TILE;
}

extern "C" int mc_gemm_nt(const mc_gemm_nt_params* p, void* stream) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_gemm_nt: null params");
  MC_CHECK(p->M >= 0 && p->N >= 0 && p->K >= 0, MC_ERR_SHAPE, "mc_gemm_nt: negative shape");
  MC_CHECK(p->in_dtype == MC_DTYPE_BF16 || p->in_dtype == MC_DTYPE_F32 || p->in_dtype == MC_DTYPE_FP8_E4M3,
           MC_ERR_DTYPE, "mc_gemm_nt: inputs must be bf16, fp32 or fp8 e4m3");
  MC_CHECK(p->out_dtype == MC_DTYPE_F32 || p->out_dtype == MC_DTYPE_BF16, MC_ERR_DTYPE,
           "mc_gemm_nt: output must be fp32 or bf16");
  if (p->M == 0 || p->N == 0) return MC_OK;
  MC_CHECK(p->C, MC_ERR_INVALID, "mc_gemm_nt: null C");
  GemmArgs g;
  bool aligned;
  const int rc = fill_operands(g, "mc_gemm_nt", p->M, p->N, p->K, p->in_dtype, p->A, p->lda, p->B, p->ldb, aligned);
  if (rc != MC_OK) return rc;
  g.C = p->C; g.ldc = p->ldc;
  g.alpha = p->alpha; g.alpha_dev = p->alpha_dev;
  g.sa = p->row_scale_a; g.sb = p->row_scale_b;
  g.c_vec = aligned16(p->C) && p->ldc % 4 == 0;
  g.c_vec16 = g.c_vec && p->ldc % 8 == 0;
  if (p->in_dtype == MC_DTYPE_FP8_E4M3 && sim8_panel_ok(g, p)) {   // the C5 similarity path (K <= 512)
    launch_sim8_panel(g, p->out_dtype, (hipStream_t)stream);
  } else if (p->in_dtype == MC_DTYPE_FP8_E4M3 && p->K % kSBK == 0 && p->K > 0) {   // fp8, longer K
    const dim3 grid(g.tiles_m * g.tiles_n), block(256);
    if (p->out_dtype == MC_DTYPE_F32) hipLaunchKernelGGL(sim_fp8_kernel<float>, grid, block, 0, (hipStream_t)stream, g);
    else hipLaunchKernelGGL(sim_fp8_kernel<bf16_t>, grid, block, 0, (hipStream_t)stream, g);
  } else {
    launch_gemm<0>(g, p->in_dtype, p->out_dtype, aligned, (hipStream_t)stream);
  }
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_gemm_nt: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

extern "C" size_t mc_ce_stats_workspace_bytes(int32_t rows, int32_t cols, int32_t axis) {
  if (rows <= 0 || cols <= 0) return 0;
  if (axis == 0) return (size_t)((rows + 3) / 4) * sizeof(float);
  return (size_t)kColSplits * cols * sizeof(float2) + (size_t)((cols + 255) / 256) * sizeof(float) + 256;
}

extern "C" int mc_ce_stats(int32_t rows, int32_t cols, const float* S, int64_t lds, int32_t axis,
                           int64_t label_offset, float* lse, float* nll, float loss_coef, float* loss_out,
                           void* workspace, size_t workspace_bytes, void* stream) {
  MC_CHECK(rows > 0 && cols > 0, MC_ERR_SHAPE, "mc_ce_stats: empty matrix");
  MC_CHECK(axis == 0 || axis == 1, MC_ERR_INVALID, "mc_ce_stats: axis must be 0 (rows) or 1 (columns)");
  MC_CHECK(S && lse, MC_ERR_INVALID, "mc_ce_stats: null S / lse");
  const size_t need = mc_ce_stats_workspace_bytes(rows, cols, axis);
  MC_CHECK(workspace && workspace_bytes >= need && aligned16(workspace), MC_ERR_WORKSPACE,
           "mc_ce_stats: workspace must be >= %zu bytes, 16-B aligned", need);
  hipStream_t s = (hipStream_t)stream;
  if (axis == 0) {
    const int nb = (rows + 3) / 4;
    float* part = reinterpret_cast<float*>(workspace);
    hipLaunchKernelGGL(ce_rows_kernel, dim3(nb), dim3(256), 0, s, rows, cols, S, lds, label_offset, lse, nll, part);
    if (loss_out) hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, part, nb, loss_coef, nullptr, loss_out);
  } else {
    float2* part = reinterpret_cast<float2*>(workspace);
    float* lpart = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + (size_t)kColSplits * cols * sizeof(float2));
    const int splits = std::min(kColSplits, rows);
    hipLaunchKernelGGL(ce_cols_partial_kernel, dim3((cols + 63) / 64, splits), dim3(256), 0, s, rows, cols, S, lds,
                       splits, part);
    const int nb = (cols + 255) / 256;
    hipLaunchKernelGGL(ce_cols_final_kernel, dim3(nb), dim3(256), 0, s, rows, cols, S, lds, splits, part,
                       label_offset, lse, nll, lpart);
    if (loss_out) hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, lpart, nb, loss_coef, nullptr, loss_out);
  }
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_ce_stats: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

extern "C" size_t mc_ce_grad_workspace_bytes(int32_t rows, int32_t cols) {
  (void)rows; (void)cols;
  return (size_t)kGradGrid * sizeof(float);
}

extern "C" int mc_ce_grad(int32_t rows, int32_t cols, const float* S, int64_t lds, const float* lse_r, int64_t off_r,
                          float coef_r, const float* lse_c, int64_t off_c, float coef_c, const float* gout_dev,
                          int32_t out_dtype, void* G, int64_t ldg, const float* scale_dev, float* dscale_out,
                          void* workspace, size_t workspace_bytes, void* stream) {
  MC_CHECK(rows > 0 && cols > 0, MC_ERR_SHAPE, "mc_ce_grad: empty matrix");
  MC_CHECK(S && lse_r && G, MC_ERR_INVALID, "mc_ce_grad: null S / lse_r / G");
  MC_CHECK(out_dtype == MC_DTYPE_F32 || out_dtype == MC_DTYPE_BF16, MC_ERR_DTYPE, "mc_ce_grad: G must be fp32/bf16");
  MC_CHECK(!dscale_out || (workspace && workspace_bytes >= mc_ce_grad_workspace_bytes(rows, cols)), MC_ERR_WORKSPACE,
           "mc_ce_grad: workspace too small for the logit_scale gradient");
  hipStream_t s = (hipStream_t)stream;
  const int64_t total = (int64_t)rows * cols;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, kGradGrid);
  float* part = dscale_out ? reinterpret_cast<float*>(workspace) : nullptr;
  if (out_dtype == MC_DTYPE_F32)
    hipLaunchKernelGGL((ce_grad_kernel<float>), dim3(grid), dim3(256), 0, s, rows, cols, S, lds, lse_r, off_r, coef_r,
                       lse_c, off_c, coef_c, gout_dev, reinterpret_cast<float*>(G), ldg, part);
  else
    hipLaunchKernelGGL((ce_grad_kernel<bf16_t>), dim3(grid), dim3(256), 0, s, rows, cols, S, lds, lse_r, off_r,
                       coef_r, lse_c, off_c, coef_c, gout_dev, reinterpret_cast<bf16_t*>(G), ldg, part);
  if (dscale_out)
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, part, grid, 1.f, scale_dev, dscale_out);
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_ce_grad: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

extern "C" int mc_quant_rows_fp8(int32_t rows, int32_t cols, int32_t in_dtype, const void* X, int64_t ldx, uint8_t* Q,
                                 int64_t ldq, float* inv_scale, void* stream) {
  MC_CHECK(rows >= 0 && cols >= 0, MC_ERR_SHAPE, "mc_quant_rows_fp8: negative shape");
  MC_CHECK(ldq % 16 == 0 && ldq >= cols, MC_ERR_SHAPE, "mc_quant_rows_fp8: ldq must be a multiple of 16 and >= cols");
  MC_CHECK(ldx >= cols, MC_ERR_SHAPE, "mc_quant_rows_fp8: ldx < cols");
  if (rows == 0) return MC_OK;
  MC_CHECK(X && Q && inv_scale, MC_ERR_INVALID, "mc_quant_rows_fp8: null pointer");
  MC_CHECK(aligned16(Q), MC_ERR_INVALID, "mc_quant_rows_fp8: Q must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((rows + 3) / 4), block(256);
  if (in_dtype == MC_DTYPE_F32)
    hipLaunchKernelGGL((quant_rows_fp8_kernel<float>), grid, block, 0, s, rows, cols,
                       reinterpret_cast<const float*>(X), ldx, Q, ldq, inv_scale);
  else if (in_dtype == MC_DTYPE_BF16)
    hipLaunchKernelGGL((quant_rows_fp8_kernel<bf16_t>), grid, block, 0, s, rows, cols,
                       reinterpret_cast<const bf16_t*>(X), ldx, Q, ldq, inv_scale);
  else if (in_dtype == MC_DTYPE_F16)
    hipLaunchKernelGGL((quant_rows_fp8_kernel<f16_t>), grid, block, 0, s, rows, cols,
                       reinterpret_cast<const f16_t*>(X), ldx, Q, ldq, inv_scale);
  else
    MC_CHECK(false, MC_ERR_DTYPE, "mc_quant_rows_fp8: input must be fp32, bf16 or f16");
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_quant_rows_fp8: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

// ------------------------------------------------------------------ fused logits + CE
namespace {
inline size_t al16(size_t b) { return (b + 15) & ~(size_t)15; }

struct FusedWs {
  float2* rpart; float2* cpart; float* tgt_r; float* tgt_c; float* partial;
  size_t bytes;
};

FusedWs fused_fwd_ws(int M, int N, bool cols, void* base) {
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  const int nb = (M + 255) / 256 + (cols ? (N + 255) / 256 : 0);
  char* p = reinterpret_cast<char*>(base);
  FusedWs w;
  size_t off = 0;
  w.rpart = reinterpret_cast<float2*>(p + off); off += al16((size_t)tn * M * sizeof(float2));
  w.cpart = cols ? reinterpret_cast<float2*>(p + off) : nullptr; off += cols ? al16((size_t)tm * N * sizeof(float2)) : 0;
  w.tgt_r = reinterpret_cast<float*>(p + off); off += al16((size_t)M * sizeof(float));
  w.tgt_c = reinterpret_cast<float*>(p + off); off += cols ? al16((size_t)N * sizeof(float)) : 0;
  w.partial = reinterpret_cast<float*>(p + off); off += al16((size_t)nb * sizeof(float));
  w.bytes = off;
  return w;
}

int fused_common(const mc_ce_fused_params* p, const char* who, GemmArgs& g, bool& aligned) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "%s: null params", who);
  const int rc = fill_operands(g, who, p->M, p->N, p->K, p->in_dtype, p->X, p->ldx, p->Y, p->ldy, aligned);
  if (rc != MC_OK) return rc;
  MC_CHECK(p->row_off > -(1 << 30) && p->row_off < (1 << 30) && p->col_off > -(1 << 30) && p->col_off < (1 << 30),
           MC_ERR_SHAPE, "%s: label offsets out of range", who);
  g.alpha = p->scale; g.alpha_dev = p->scale_dev;
  g.sa = p->row_scale_x; g.sb = p->row_scale_y;
  g.off_r = (int)p->row_off; g.off_c = (int)p->col_off;
  g.coef_r = p->coef_r; g.coef_c = p->coef_c;
  return MC_OK;
}
}  // namespace

extern "C" size_t mc_ce_fused_fwd_workspace_bytes(int32_t M, int32_t N, int32_t with_columns) {
  if (M <= 0 || N <= 0) return 0;
  return fused_fwd_ws(M, N, with_columns != 0, nullptr).bytes;
}

extern "C" int mc_ce_fused_fwd(const mc_ce_fused_params* p, void* stream) {
  GemmArgs g;
  bool aligned;
  const int rc = fused_common(p, "mc_ce_fused_fwd", g, aligned);
  if (rc != MC_OK) return rc;
  MC_CHECK(p->lse_r && p->loss_out, MC_ERR_INVALID, "mc_ce_fused_fwd: null lse_r / loss_out");
  const bool cols = p->lse_c != nullptr;
  const FusedWs w = fused_fwd_ws(p->M, p->N, cols, p->workspace);
  MC_CHECK(p->workspace && aligned16(p->workspace) && p->workspace_bytes >= w.bytes, MC_ERR_WORKSPACE,
           "mc_ce_fused_fwd: workspace must be >= %zu bytes, 16-B aligned", w.bytes);
  g.rpart = w.rpart; g.cpart = w.cpart; g.tgt_r = w.tgt_r; g.tgt_c = w.tgt_c;
  hipStream_t s = (hipStream_t)stream;
  launch_gemm<1>(g, p->in_dtype, MC_DTYPE_F32, aligned, s);
  const int nbr = (p->M + 255) / 256, nb = nbr + (cols ? (p->N + 255) / 256 : 0);
  hipLaunchKernelGGL(ce_fused_reduce_kernel, dim3(nb), dim3(256), 0, s, p->M, p->N, g.tiles_m, g.tiles_n, w.rpart,
                     w.cpart, w.tgt_r, w.tgt_c, g.off_r, g.off_c, p->coef_r, p->coef_c, p->lse_r, p->lse_c, nbr,
                     w.partial);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, w.partial, nb, 1.f, nullptr, p->loss_out);
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_ce_fused_fwd: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

extern "C" size_t mc_ce_fused_grad_workspace_bytes(int32_t M, int32_t N) {
  if (M <= 0 || N <= 0) return 0;
  return al16((size_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN) * sizeof(float));
}

extern "C" int mc_ce_fused_grad(const mc_ce_fused_params* p, void* stream) {
  GemmArgs g;
  bool aligned;
  const int rc = fused_common(p, "mc_ce_fused_grad", g, aligned);
  if (rc != MC_OK) return rc;
  MC_CHECK(p->lse_r || p->lse_c, MC_ERR_INVALID, "mc_ce_fused_grad: lse_r and lse_c both NULL");
  MC_CHECK(p->G, MC_ERR_INVALID, "mc_ce_fused_grad: null G");
  MC_CHECK(p->g_dtype == MC_DTYPE_F32 || p->g_dtype == MC_DTYPE_BF16, MC_ERR_DTYPE,
           "mc_ce_fused_grad: G must be fp32 or bf16");
  MC_CHECK(p->ldg >= p->N, MC_ERR_SHAPE, "mc_ce_fused_grad: ldg < N");
  const size_t need = mc_ce_fused_grad_workspace_bytes(p->M, p->N);
  MC_CHECK(!p->dscale_out || (p->workspace && aligned16(p->workspace) && p->workspace_bytes >= need),
           MC_ERR_WORKSPACE, "mc_ce_fused_grad: workspace must be >= %zu bytes, 16-B aligned", need);
  g.lse_r = p->lse_r; g.lse_c = p->lse_c; g.gout_dev = p->gout_dev; g.g_times_alpha = p->g_times_scale != 0;
  g.C = p->G; g.ldc = p->ldg;
  g.c_vec = aligned16(p->G) && p->ldg % 4 == 0;
  g.c_vec16 = g.c_vec && p->ldg % 8 == 0;
  g.gpart = p->dscale_out ? reinterpret_cast<float*>(p->workspace) : nullptr;
  hipStream_t s = (hipStream_t)stream;
  launch_gemm<2>(g, p->in_dtype, p->g_dtype, aligned, s);
  if (p->dscale_out)   // sum(G S) / scale: the scale gradient (G here is without gmul)
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, g.gpart, g.tiles_m * g.tiles_n,
                       p->scale_dev ? 1.f : 1.f / p->scale, p->scale_dev, p->dscale_out);
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_ce_fused_grad: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}
