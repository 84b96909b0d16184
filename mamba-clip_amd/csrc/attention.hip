// attention.hip -- fused multi-head self-attention for short sequences (mc_attn.h): the ViT-B/16
// image tower (197 tokens) and the BERT text tower (<= 256 tokens), 12 heads of 64, bf16 / f16.
//
// Replaces torch's scaled_dot_product_attention inside the towers' blocks (timm / open_clip / HF
// attention behind the reference's model dict, model.py:1019-1064).  At
// N = 197 the library kernels are tiled for long sequences and run at ~7 % of the MFMA rate; here
// one workgroup owns one (batch, head) and keeps the whole sequence in LDS:
//  * forward: K and V images in LDS; each wave takes 32-query blocks and computes S^T = K Q^T on
//    v_mfma_f32_32x32x16 with the KEY on the accumulator rows and the query on the lane, so the
//    softmax over keys is in-lane (plus one permlane32 swap for the other lane half) and exact
//    (the full row is in registers: no online rescale); the probabilities, converted to 16-bit,
//    are directly the B operand of O^T = V^T P^T (V^T by ds_read_b64_tr_b16 transposed reads).
//  * backward: Q, K, V, dO images in LDS plus the row constants lse and delta = rowsum(dO o O).
//    Phase 1: wave w owns key tile w and sweeps the query blocks with the key on the lane
//    (S = Q K^T, dP = dO V^T), so P and dS = P (dP - delta) are the B operands of dV^T += dO^T P
//    and dK^T += Q^T dS.  Phase 2: wave w owns query block w and sweeps the key tiles in the
//    forward orientation (S^T, dP^T) for dQ^T += K^T dS^T.  Recomputing S / dP in phase 2 costs
//    8 of the 28 MFMAs per tile pair and removes every cross-wave sum (no atomics, deterministic).
// LDS images: [rows][64 x 16-bit], 16-B chunk c of row r at slot c ^ g((r >> 1) & 7) with
// g(m) = m ^ ((m & 1) << 2): the row reads of the 32x32x16 operands (ds_read_b128, 16 rows of
// one chunk per lane group) and the transposed reads (rows r..r+3 x 4 chunks per half-wave) are
// both conflict-free (64 banks x 4 B).
#include <algorithm>

#include "mc_common.h"
#include "../../include/mc_attn.h"

namespace mc {
namespace attn {

constexpr int kD = 64;            // head dim
constexpr int kRowB = kD * 2;     // bytes per 16-bit row
constexpr int kFwdWaves = 8;   // one 32-query block per wave (N <= 256); two workgroups per CU
constexpr int kBwdWaves = 8;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T> struct M32;
template <> struct M32<bf16_t> {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 mma(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8, a), __builtin_bit_cast(v8, b), c, 0, 0, 0);
  }
};
template <> struct M32<f16_t> {
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 mma(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8, a), __builtin_bit_cast(v8, b), c, 0, 0, 0);
  }
};

__device__ __forceinline__ uint32_t img_off(int r, int c) {
  const int m = (r >> 1) & 7;
  return (uint32_t)(r * kRowB + 16 * (c ^ (m ^ ((m & 1) << 2))));
}
// 16-B row chunk c of row r (A / B operand of a 32x32x16 MFMA in natural k order)
__device__ __forceinline__ uint4 row_chunk(const char* img, int r, int c) {
  return *reinterpret_cast<const uint4*>(img + img_off(r, c));
}
// Transposed operand: rows r0 + {0..3} and r0 + 8 + {0..3} of the 16 columns d0 + [0, 16) of this
// lane's group (lane 4q + p of the group addresses row q, columns 4p..4p+3; lane i receives column i).
// Elements j of the result are rows r0 + 8 (j >> 2) + (j & 3): the k order of an accumulator tile
// used as the other operand (rows 16 s + 8 (j >> 2) + 4 h + (j & 3) with r0 = 16 s + 4 h).
__device__ __forceinline__ uint4 tr_chunk(const char* img, int r0, int d0, int lane) {
  const int li = lane & 15, q = li >> 2, d = d0 + 4 * (li & 3);
  const char* pa = img + img_off(r0 + q, d >> 3) + (d & 7) * 2;
  const char* pb = img + img_off(r0 + 8 + q, d >> 3) + (d & 7) * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)pa);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)pb);
  return make_uint4((uint32_t)(uint16_t)lo.x | ((uint32_t)(uint16_t)lo.y << 16),
                    (uint32_t)(uint16_t)lo.z | ((uint32_t)(uint16_t)lo.w << 16),
                    (uint32_t)(uint16_t)hi.x | ((uint32_t)(uint16_t)hi.y << 16),
                    (uint32_t)(uint16_t)hi.z | ((uint32_t)(uint16_t)hi.w << 16));
}
// registers 8 s .. 8 s + 7 of an accumulator tile as a 16-bit operand fragment (k-step s)
template <typename TI>
__device__ __forceinline__ uint4 acc_frag(const f32x16& x, int s) {
  return make_uint4(cvt_pk2<TI>(x[8 * s + 0], x[8 * s + 1]), cvt_pk2<TI>(x[8 * s + 2], x[8 * s + 3]),
                    cvt_pk2<TI>(x[8 * s + 4], x[8 * s + 5]), cvt_pk2<TI>(x[8 * s + 6], x[8 * s + 7]));
}
__device__ __forceinline__ float swap_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float swap_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
template <int kCtrl>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kCtrl, 0xF, 0xF, true));
}
__device__ __forceinline__ float row_xor4(float v) {   // banks 0 / 2 take lane + 4, banks 1 / 3 lane - 4
  const int iv = __float_as_int(v);
  const int lo = __builtin_amdgcn_update_dpp(iv, iv, 0x104, 0xF, 0x5, false);
  return __int_as_float(__builtin_amdgcn_update_dpp(lo, iv, 0x114, 0xF, 0xA, false));
}
// Column sums of a stored tile pair (x0: d in [0, 32), x1: [32, 64); lane = output row, accumulator
// rows = d), rows with `valid` false excluded.  Halving butterfly over the 32 lanes of each half:
// lane bit 4 by permlane16 swaps (32 -> 16 values), bits 3, 2, 1, 0 by DPP (16 -> 1); lane l ends
// with the sum of value index l & 31 = 16 db + r, i.e. d = 32 db + (r & 3) + 8 (r >> 2) + 4 hh.
// ~96 VALU per tile instead of a 5-step all-reduce of all 32 values.
__device__ __forceinline__ float tile_colsum(const f32x16& x0, const f32x16& x1, float mul, int lane) {
  float w[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x0[r] * mul), __float_as_uint(x1[r] * mul), false, false);
    w[r] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  }
  const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
  float u[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) u[k] = (b3 ? w[k + 8] : w[k]) + dpp_mov<0x128>(b3 ? w[k] : w[k + 8]);   // row_ror:8
  float t[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) t[k] = (b2 ? u[k + 4] : u[k]) + row_xor4(b2 ? u[k] : u[k + 4]);
  float q[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) q[k] = (b1 ? t[k + 2] : t[k]) + dpp_mov<0x4E>(b1 ? t[k] : t[k + 2]);   // lane ^ 2
  return (b0 ? q[1] : q[0]) + dpp_mov<0xB1>(b0 ? q[0] : q[1]);                                        // lane ^ 1
}

// Store a transposed accumulator pair (x0: d in [0, 32), x1: [32, 64); column = this lane's row
// `row`, accumulator rows = d) as 16-B pieces: permlane32 swaps turn each lane's 4-element groups
// into 8 consecutive d (T21).  rows >= nrows are dropped.
// csum (LDS, 64 floats, nullable): the tile's column sums (fp32, rows < nrows).
template <typename TI>
__device__ __forceinline__ void store_rows(TI* base, int64_t ns, int row, int nrows, int lane, const f32x16& x0,
                                           const f32x16& x1, float mul, float* csum = nullptr) {
  const int hh = lane >> 5;
  if (csum) {   // the tile's column sums (fp32, before the 16-bit rounding of the stores)
    const int i = lane & 31, r = i & 15;
    csum[32 * (i >> 4) + (r & 3) + 8 * (r >> 2) + 4 * hh] = tile_colsum(x0, x1, row < nrows ? mul : 0.f, lane);
  }
#pragma unroll
  for (int db = 0; db < 2; ++db) {
    const f32x16& x = db ? x1 : x0;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x[8 * m + i]), __float_as_uint(x[8 * m + 4 + i]),
                                                        false, false);
        v[i] = __uint_as_float(r[0]) * mul;
        v[4 + i] = __uint_as_float(r[1]) * mul;
      }
      const int d0 = db * 32 + 16 * m + 8 * hh;
      if (row < nrows) *reinterpret_cast<uint4*>(base + (int64_t)row * ns + d0) = pack_f<TI>(v);
    }
  }
}

// One global_load_lds_dwordx4: 16 B per lane from gsrc to LDS byte address m0v + 16 * lane (m0v
// wave-uniform), asm so hipcc does not track it (the caller waits with its own vmcnt); M0 is
// compiler-reserved: saved and restored in the statement.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t m0v) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(m0v) : "memory");
}
typedef __attribute__((address_space(3))) char lds_char;

struct FwdArgs {
  int B, H, N;
  float scale, c2;   // c2 = scale * log2(e)
  const void* q; const void* k; const void* v;
  int64_t q_bs, q_ns, q_hs;
  void* o; int64_t o_bs, o_ns, o_hs;
  float* lse;
};

template <typename TI, int NT>
__global__ __launch_bounds__(64 * kFwdWaves, 2) void attn_fwd_kernel(const FwdArgs a) {
  using M = M32<TI>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int Np = NT * 32;
  char* kimg = smem;
  char* vimg = smem + Np * kRowB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hh = lane >> 5, l32 = lane & 31;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int N = a.N;
  const int64_t off = (int64_t)b * a.q_bs + (int64_t)h * a.q_hs;
  const TI* qg = reinterpret_cast<const TI*>(a.q) + off;
  const TI* kg = reinterpret_cast<const TI*>(a.k) + off;
  const TI* vg = reinterpret_cast<const TI*>(a.v) + off;

  // K / V images: every piece of a thread in flight at once (buffer loads: rows past N read 0)
  constexpr int kPer = (Np * 8 + 64 * kFwdWaves - 1) / (64 * kFwdWaves);
  const uint32_t rng = (uint32_t)(((int64_t)(N - 1) * a.q_ns + kD) * (int64_t)sizeof(TI));
  const __amdgpu_buffer_rsrc_t rk = make_rsrc(kg, rng), rv = make_rsrc(vg, rng);
  uint4 kr[kPer], vr[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int i = tid + 64 * kFwdWaves * j, r = i >> 3, c = i & 7;
    const uint32_t o = r < N ? (uint32_t)(r * a.q_ns + 8 * c) * (uint32_t)sizeof(TI) : 0x80000000u;
    kr[j] = buf_ld16(rk, o);
    vr[j] = buf_ld16(rv, o);
  }
  // this wave's 32-query block (B operand: lane = query, 16-B chunks 2 s + hh of its row)
  const int qt = wave;
  const int q = qt * 32 + l32;
  uint4 qf[4];
  {
    const TI* qrow = qg + (int64_t)min(q, N - 1) * a.q_ns;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = ld16(qrow + 16 * s + 8 * hh);
  }
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int i = tid + 64 * kFwdWaves * j, r = i >> 3, c = i & 7;
    if (i < Np * 8) {
      *reinterpret_cast<uint4*>(kimg + img_off(r, c)) = kr[j];
      *reinterpret_cast<uint4*>(vimg + img_off(r, c)) = vr[j];
    }
  }
  __syncthreads();
  if (qt < NT) {
    // S^T tiles: rows = keys t*32 + (r & 3) + 8 (r >> 2) + 4 hh, column = this lane's query.
    // Two passes over the key tiles (the row max, then the probabilities and P V): recomputing
    // S costs 4 MFMAs per tile and keeps one tile of scores live instead of all NT (no spills).
    auto s_tile = [&](int t) __attribute__((always_inline)) {
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = M::mma(row_chunk(kimg, t * 32 + l32, 2 * s + hh), qf[s], acc);
      if (t == NT - 1 && Np > N) {   // keys past N (last tile only)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (t * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh >= N) acc[r] = -1e30f;
      }
      return acc;
    };
    float m = -1e30f;
#pragma unroll 1
    for (int t = 0; t < NT; ++t) {
      const f32x16 st = s_tile(t);
#pragma unroll
      for (int r = 0; r < 16; ++r) m = fmaxf(m, st[r]);
    }
    m = swap_max(m);
    const float mc = m * a.c2;
    // O^T = V^T P^T: two 32-row d blocks, lane = query
    float l = 0.f;
    f32x16 o0 = {}, o1 = {};
#pragma unroll 1
    for (int t = 0; t < NT; ++t) {
      f32x16 st = s_tile(t);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fast_exp2(st[r] * a.c2 - mc);
        st[r] = p;
        l += p;
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const uint4 pf = acc_frag<TI>(st, s2);
        const int r0 = t * 32 + 16 * s2 + 4 * hh;
        o0 = M::mma(tr_chunk(vimg, r0, 16 * ((lane >> 4) & 1), lane), pf, o0);
        o1 = M::mma(tr_chunk(vimg, r0, 32 + 16 * ((lane >> 4) & 1), lane), pf, o1);
      }
    }
    l = swap_sum(l);
    store_rows<TI>(reinterpret_cast<TI*>(a.o) + (int64_t)b * a.o_bs + (int64_t)h * a.o_hs, a.o_ns, q, N, lane, o0, o1,
                   1.f / l);
    if (hh == 0 && q < N) a.lse[(int64_t)bh * N + q] = m * a.scale + fast_log2(l) * kLn2;
  }
}

struct BwdArgs {
  int B, H, N;
  float scale, c2;
  const void* q; const void* k; const void* v;
  int64_t q_bs, q_ns, q_hs;
  const void* o; const void* g;
  int64_t o_bs, o_ns, o_hs;
  const float* lse;
  void* dq; void* dk; void* dv;
  int64_t d_bs, d_ns, d_hs;
  float* dsum;   // (B, 3, H, 64) or null
};

template <typename TI, int NT>
__global__ __launch_bounds__(64 * kBwdWaves, 1) void attn_bwd_kernel(const BwdArgs a) {
  using M = M32<TI>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int Np = NT * 32;
  constexpr int kImg = Np * kRowB;
  // N <= 224: persistent over heads with the next head's q / dO / O streamed into LDS during phase 2
  // (the images fit 160 KB with the O staging image); N = 256: one head per workgroup
  constexpr bool kPersist = NT <= 7;
  char* qimg = smem;
  char* kimg = smem + kImg;
  char* vimg = smem + 2 * kImg;
  char* gimg = smem + 3 * kImg;
  char* oimg = smem + 4 * kImg;                                              // kPersist only
  float* lse2 = reinterpret_cast<float*>(smem + (kPersist ? 5 : 4) * kImg);   // lse * log2(e); +inf past N (P = 0)
  float* dlt = lse2 + Np;                                                     // rowsum(dO o O)
  float* csl = dlt + Np;                                                      // [dq | dk | dv][wave][64] tile column sums
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hh = lane >> 5, l32 = lane & 31, g16 = 16 * ((lane >> 4) & 1);
  const int N = a.N, total = a.B * a.H;
  constexpr int kPer = (Np * 8 + 64 * kBwdWaves - 1) / (64 * kBwdWaves);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)smem);

  // q / dO / O rows of head bh -> qimg / gimg / oimg by LDS-DMA (lane-linear 1-KB pieces = 8 rows:
  // lane L takes slot L % 8 of row L / 8 and loads the chunk that belongs there, c = slot ^ g(row);
  // rows past N repeat row N - 1, harmless: their P and dS are 0, their outputs are not stored)
  float lv = 0.f;
  auto dma_qgo = [&](int bh) __attribute__((always_inline)) {
    const int b = bh / a.H, h = bh % a.H;
    const TI* qg = reinterpret_cast<const TI*>(a.q) + (int64_t)b * a.q_bs + (int64_t)h * a.q_hs;
    const TI* gg = reinterpret_cast<const TI*>(a.g) + (int64_t)b * a.o_bs + (int64_t)h * a.o_hs;
    const TI* og = reinterpret_cast<const TI*>(a.o) + (int64_t)b * a.o_bs + (int64_t)h * a.o_hs;
#pragma unroll
    for (int k = 0; k < (Np / 8 + kBwdWaves - 1) / kBwdWaves; ++k) {
      const int j = wave + kBwdWaves * k;
      if (j < Np / 8) {
        const uint32_t blk = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(1024 * j));   // wave-uniform M0 base
        const int r = 8 * j + (lane >> 3), m = (r >> 1) & 7;
        const int c = (lane & 7) ^ (m ^ ((m & 1) << 2));
        const int64_t rr = min(r, N - 1);
        glds16(qg + rr * a.q_ns + 8 * c, blk);
        glds16(gg + rr * a.o_ns + 8 * c, blk + (uint32_t)(3 * kImg));
        glds16(og + rr * a.o_ns + 8 * c, blk + (uint32_t)(4 * kImg));
      }
    }
    if (tid < Np) lv = a.lse[(int64_t)bh * N + min(tid, N - 1)];
  };
  if constexpr (kPersist) dma_qgo(blockIdx.x);

#pragma unroll 1
  for (int bh = blockIdx.x; bh < total; bh += gridDim.x) {
  const int b = bh / a.H, h = bh % a.H;
  const int64_t off = (int64_t)b * a.q_bs + (int64_t)h * a.q_hs;
  const int64_t offo = (int64_t)b * a.o_bs + (int64_t)h * a.o_hs;
  const TI* qg = reinterpret_cast<const TI*>(a.q) + off;
  const TI* kg = reinterpret_cast<const TI*>(a.k) + off;
  const TI* vg = reinterpret_cast<const TI*>(a.v) + off;
  const TI* og = reinterpret_cast<const TI*>(a.o) + offo;
  const TI* gg = reinterpret_cast<const TI*>(a.g) + offo;

  if constexpr (kPersist) {
    // ---- K / V of this head (registers -> images), delta from the streamed dO / O images, lse2
    const uint32_t rq = (uint32_t)(((int64_t)(N - 1) * a.q_ns + kD) * (int64_t)sizeof(TI));
    const __amdgpu_buffer_rsrc_t rsk = make_rsrc(kg, rq), rsv = make_rsrc(vg, rq);
    uint4 kv[kPer], vv[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int i = tid + 64 * kBwdWaves * j, r = i >> 3, c = i & 7;
      const uint32_t o1 = r < N ? (uint32_t)(r * a.q_ns + 8 * c) * (uint32_t)sizeof(TI) : 0x80000000u;
      kv[j] = buf_ld16(rsk, o1);
      vv[j] = buf_ld16(rsv, o1);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's LDS-DMA pieces (and K / V) landed
    __syncthreads();                      // ... and everyone's
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int i = tid + 64 * kBwdWaves * j, r = i >> 3, c = i & 7;
      float part = 0.f;
      if (i < Np * 8) {
        const uint4 gq = row_chunk(gimg, r, c), oq = row_chunk(oimg, r, c);
#pragma unroll
        for (int e = 0; e < 8; ++e) part += elem_f<TI>(gq, e) * elem_f<TI>(oq, e);
      }
      part += __shfl_xor(part, 1);
      part += __shfl_xor(part, 2);
      part += __shfl_xor(part, 4);
      if (i < Np * 8) {
        *reinterpret_cast<uint4*>(kimg + img_off(r, c)) = kv[j];
        *reinterpret_cast<uint4*>(vimg + img_off(r, c)) = vv[j];
        if (c == 0) dlt[r] = r < N ? part : 0.f;
      }
    }
    if (tid < Np) lse2[tid] = tid < N ? lv * kLog2e : __builtin_huge_valf();
  } else {
  // ---- prologue: four images, delta and lse2.  Every piece of a thread in flight at once (buffer
  // loads: rows past N read 0); 8 consecutive threads hold one row (delta's partial dots)
  {
    const uint32_t rq = (uint32_t)(((int64_t)(N - 1) * a.q_ns + kD) * (int64_t)sizeof(TI));
    const uint32_t ro = (uint32_t)(((int64_t)(N - 1) * a.o_ns + kD) * (int64_t)sizeof(TI));
    const __amdgpu_buffer_rsrc_t rsq = make_rsrc(qg, rq), rsk = make_rsrc(kg, rq), rsv = make_rsrc(vg, rq);
    const __amdgpu_buffer_rsrc_t rso = make_rsrc(og, ro), rsg = make_rsrc(gg, ro);
    uint4 qv[kPer], kv[kPer], vv[kPer], gv[kPer], ov[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int i = tid + 64 * kBwdWaves * j, r = i >> 3, c = i & 7;
      const uint32_t o1 = r < N ? (uint32_t)(r * a.q_ns + 8 * c) * (uint32_t)sizeof(TI) : 0x80000000u;
      const uint32_t o2 = r < N ? (uint32_t)(r * a.o_ns + 8 * c) * (uint32_t)sizeof(TI) : 0x80000000u;
      qv[j] = buf_ld16(rsq, o1);
      kv[j] = buf_ld16(rsk, o1);
      vv[j] = buf_ld16(rsv, o1);
      gv[j] = buf_ld16(rsg, o2);
      ov[j] = buf_ld16(rso, o2);
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int i = tid + 64 * kBwdWaves * j, r = i >> 3, c = i & 7;
      float part = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) part += elem_f<TI>(gv[j], e) * elem_f<TI>(ov[j], e);
      part += __shfl_xor(part, 1);
      part += __shfl_xor(part, 2);
      part += __shfl_xor(part, 4);
      if (i < Np * 8) {
        *reinterpret_cast<uint4*>(qimg + img_off(r, c)) = qv[j];
        *reinterpret_cast<uint4*>(kimg + img_off(r, c)) = kv[j];
        *reinterpret_cast<uint4*>(vimg + img_off(r, c)) = vv[j];
        *reinterpret_cast<uint4*>(gimg + img_off(r, c)) = gv[j];
        if (c == 0) {
          dlt[r] = part;
          lse2[r] = r < N ? a.lse[(int64_t)bh * N + r] * kLog2e : __builtin_huge_valf();
        }
      }
    }
  }
  }
  __syncthreads();

  // ---- phase 1: wave = key tile; dV^T += dO^T P, dK^T += Q^T dS over the query blocks.  (Issuing
  // the next block's S / dP MFMAs before this block's gradient MFMAs, with K / V re-read from LDS
  // to make room, measured 12 % slower: 325 vs 290 us at C2.)
  if (wave < NT) {
    const int kt = wave;
    uint4 kf[4], vf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = row_chunk(kimg, kt * 32 + l32, 2 * s + hh);
      vf[s] = row_chunk(vimg, kt * 32 + l32, 2 * s + hh);
    }
    f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
#pragma unroll 1
    for (int qt = 0; qt < NT; ++qt) {
      f32x16 sa = {}, pa = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sa = M::mma(row_chunk(qimg, qt * 32 + l32, 2 * s + hh), kf[s], sa);
        pa = M::mma(row_chunk(gimg, qt * 32 + l32, 2 * s + hh), vf[s], pa);
      }
      // rows of this lane's accumulators: queries qt*32 + 8 j + 4 hh + i  (register 4 j + i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 L = *reinterpret_cast<const f32x4*>(lse2 + qt * 32 + 8 * j + 4 * hh);
        const f32x4 Dl = *reinterpret_cast<const f32x4*>(dlt + qt * 32 + 8 * j + 4 * hh);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = fast_exp2(sa[4 * j + i] * a.c2 - L[i]);
          sa[4 * j + i] = p;
          pa[4 * j + i] = p * (pa[4 * j + i] - Dl[i]);
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const uint4 pf = acc_frag<TI>(sa, s2), df = acc_frag<TI>(pa, s2);
        const int r0 = qt * 32 + 16 * s2 + 4 * hh;
        dv0 = M::mma(tr_chunk(gimg, r0, g16, lane), pf, dv0);
        dv1 = M::mma(tr_chunk(gimg, r0, 32 + g16, lane), pf, dv1);
        dk0 = M::mma(tr_chunk(qimg, r0, g16, lane), df, dk0);
        dk1 = M::mma(tr_chunk(qimg, r0, 32 + g16, lane), df, dk1);
      }
    }
    const int64_t doff = (int64_t)b * a.d_bs + (int64_t)h * a.d_hs;
    store_rows<TI>(reinterpret_cast<TI*>(a.dk) + doff, a.d_ns, kt * 32 + l32, N, lane, dk0, dk1, a.scale,
                   a.dsum ? csl + (1 * kBwdWaves + wave) * kD : nullptr);
    store_rows<TI>(reinterpret_cast<TI*>(a.dv) + doff, a.d_ns, kt * 32 + l32, N, lane, dv0, dv1, 1.f,
                   a.dsum ? csl + (2 * kBwdWaves + wave) * kD : nullptr);
  }

  // ---- phase 2: wave = query block; dQ^T += K^T dS^T over the key tiles (forward orientation)
  const int qt = wave, q = qt * 32 + l32;
  uint4 qf[4], gf[4];
  float L = 0.f, Dl = 0.f;
  if (wave < NT) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = row_chunk(qimg, q, 2 * s + hh);
      gf[s] = row_chunk(gimg, q, 2 * s + hh);
    }
    L = lse2[q];
    Dl = dlt[q];
  }
  if constexpr (kPersist) {   // q / dO images and the row constants are free: stream the next head's
    __syncthreads();
    if (bh + (int)gridDim.x < total) dma_qgo(bh + gridDim.x);
  }
  if (wave < NT) {
    f32x16 dq0 = {}, dq1 = {};
#pragma unroll 1
    for (int kt = 0; kt < NT; ++kt) {
      f32x16 sa = {}, pa = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sa = M::mma(row_chunk(kimg, kt * 32 + l32, 2 * s + hh), qf[s], sa);
        pa = M::mma(row_chunk(vimg, kt * 32 + l32, 2 * s + hh), gf[s], pa);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fast_exp2(sa[r] * a.c2 - L);
        pa[r] = p * (pa[r] - Dl);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const uint4 df = acc_frag<TI>(pa, s2);
        const int r0 = kt * 32 + 16 * s2 + 4 * hh;
        dq0 = M::mma(tr_chunk(kimg, r0, g16, lane), df, dq0);
        dq1 = M::mma(tr_chunk(kimg, r0, 32 + g16, lane), df, dq1);
      }
    }
    const int64_t doff = (int64_t)b * a.d_bs + (int64_t)h * a.d_hs;
    store_rows<TI>(reinterpret_cast<TI*>(a.dq) + doff, a.d_ns, q, N, lane, dq0, dq1, a.scale,
                   a.dsum ? csl + wave * kD : nullptr);
  }
  if (a.dsum) {   // per-(batch, head) column sums, tiles in fixed order (deterministic)
    __syncthreads();
    if (tid < 3 * kD) {
      const int o = tid / kD, d = tid % kD;
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < NT; ++w) acc += csl[(o * kBwdWaves + w) * kD + d];
      a.dsum[(((int64_t)b * 3 + o) * a.H + h) * kD + d] = acc;
    }
  }
  __syncthreads();   // images, row constants and column sums are reused by the next head
  }
}

size_t fwd_lds(int NT) { return (size_t)2 * NT * 32 * kRowB; }
size_t bwd_lds(int NT) {
  return (size_t)(NT <= 7 ? 5 : 4) * NT * 32 * kRowB + (size_t)2 * NT * 32 * 4 + (size_t)3 * kBwdWaves * kD * 4;
}
static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <typename TI, int NT>
void launch_fwd_nt(const FwdArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((attn_fwd_kernel<TI, NT>), dim3(a.B * a.H), dim3(64 * kFwdWaves), fwd_lds(NT), s, a);
}
template <typename TI, int NT>
void launch_bwd_nt(const BwdArgs& a, hipStream_t s) {
  // NT <= 7: persistent, one workgroup per CU walks the heads (the LDS of one head fills the CU)
  const int grid = NT <= 7 ? std::min(a.B * a.H, num_cus()) : a.B * a.H;
  hipLaunchKernelGGL((attn_bwd_kernel<TI, NT>), dim3(grid), dim3(64 * kBwdWaves), bwd_lds(NT), s, a);
}
template <typename TI>
void launch_fwd(const FwdArgs& a, hipStream_t s) {
  switch ((a.N + 31) / 32) {
    case 1: launch_fwd_nt<TI, 1>(a, s); break;
    case 2: launch_fwd_nt<TI, 2>(a, s); break;
    case 3: launch_fwd_nt<TI, 3>(a, s); break;
    case 4: launch_fwd_nt<TI, 4>(a, s); break;
    case 5: launch_fwd_nt<TI, 5>(a, s); break;
    case 6: launch_fwd_nt<TI, 6>(a, s); break;
    case 7: launch_fwd_nt<TI, 7>(a, s); break;
    default: launch_fwd_nt<TI, 8>(a, s); break;
  }
}
template <typename TI>
void launch_bwd(const BwdArgs& a, hipStream_t s) {
  switch ((a.N + 31) / 32) {
    case 1: launch_bwd_nt<TI, 1>(a, s); break;
    case 2: launch_bwd_nt<TI, 2>(a, s); break;
    case 3: launch_bwd_nt<TI, 3>(a, s); break;
    case 4: launch_bwd_nt<TI, 4>(a, s); break;
    case 5: launch_bwd_nt<TI, 5>(a, s); break;
    case 6: launch_bwd_nt<TI, 6>(a, s); break;
    case 7: launch_bwd_nt<TI, 7>(a, s); break;
    default: launch_bwd_nt<TI, 8>(a, s); break;
  }
}

static bool rows_ok(const void* p, int64_t bs, int64_t ns, int64_t hs) {
  return p && aligned16(p) && bs % 8 == 0 && ns % 8 == 0 && hs % 8 == 0;
}
static int check_common(int B, int H, int N, int D, int dtype, const char* who) {
  MC_CHECK(B >= 0 && H > 0, MC_ERR_SHAPE, "%s: bad batch / heads (%d, %d)", who, B, H);
  MC_CHECK(D == MC_ATTN_HEAD_DIM, MC_ERR_SHAPE, "%s: head_dim %d (only %d is built)", who, D, MC_ATTN_HEAD_DIM);
  MC_CHECK(N >= 1 && N <= MC_ATTN_MAX_SEQ, MC_ERR_SHAPE, "%s: seqlen %d outside [1, %d]", who, N, MC_ATTN_MAX_SEQ);
  MC_CHECK(dtype == MC_DTYPE_BF16 || dtype == MC_DTYPE_F16, MC_ERR_DTYPE, "%s: dtype %d (bf16 / f16 only)", who, dtype);
  return MC_OK;
}

}  // namespace attn
}  // namespace mc

using namespace mc;

extern "C" int mc_attn_fwd(const mc_attn_fwd_params* p, void* stream) {
  MC_CHECK(p, MC_ERR_INVALID, "mc_attn_fwd: null params");
  const int rc = attn::check_common(p->batch, p->heads, p->seqlen, p->head_dim, p->dtype, "mc_attn_fwd");
  if (rc != MC_OK) return rc;
  MC_CHECK(attn::rows_ok(p->q, p->q_bs, p->q_ns, p->q_hs) && attn::rows_ok(p->k, p->q_bs, p->q_ns, p->q_hs) &&
               attn::rows_ok(p->v, p->q_bs, p->q_ns, p->q_hs) && attn::rows_ok(p->o, p->o_bs, p->o_ns, p->o_hs) && p->lse,
           MC_ERR_INVALID, "mc_attn_fwd: q / k / v / o need 16-B aligned rows (strides %% 8 elements), lse non-null");
  if (p->batch == 0) return MC_OK;
  attn::FwdArgs a;
  a.B = p->batch; a.H = p->heads; a.N = p->seqlen;
  a.scale = p->scale; a.c2 = p->scale * kLog2e;
  a.q = p->q; a.k = p->k; a.v = p->v;
  a.q_bs = p->q_bs; a.q_ns = p->q_ns; a.q_hs = p->q_hs;
  a.o = p->o; a.o_bs = p->o_bs; a.o_ns = p->o_ns; a.o_hs = p->o_hs;
  a.lse = p->lse;
  if (p->dtype == MC_DTYPE_BF16) attn::launch_fwd<bf16_t>(a, (hipStream_t)stream);
  else attn::launch_fwd<f16_t>(a, (hipStream_t)stream);
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_attn_fwd: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

extern "C" int mc_attn_bwd(const mc_attn_bwd_params* p, void* stream) {
  MC_CHECK(p, MC_ERR_INVALID, "mc_attn_bwd: null params");
  const int rc = attn::check_common(p->batch, p->heads, p->seqlen, p->head_dim, p->dtype, "mc_attn_bwd");
  if (rc != MC_OK) return rc;
  MC_CHECK(attn::rows_ok(p->q, p->q_bs, p->q_ns, p->q_hs) && attn::rows_ok(p->k, p->q_bs, p->q_ns, p->q_hs) &&
               attn::rows_ok(p->v, p->q_bs, p->q_ns, p->q_hs) && attn::rows_ok(p->o, p->o_bs, p->o_ns, p->o_hs) &&
               attn::rows_ok(p->dout, p->o_bs, p->o_ns, p->o_hs) && attn::rows_ok(p->dq, p->dq_bs, p->dq_ns, p->dq_hs) &&
               attn::rows_ok(p->dk, p->dq_bs, p->dq_ns, p->dq_hs) && attn::rows_ok(p->dv, p->dq_bs, p->dq_ns, p->dq_hs) &&
               p->lse,
           MC_ERR_INVALID, "mc_attn_bwd: every tensor needs 16-B aligned rows (strides %% 8 elements), lse non-null");
  if (p->batch == 0) return MC_OK;
  attn::BwdArgs a;
  a.B = p->batch; a.H = p->heads; a.N = p->seqlen;
  a.scale = p->scale; a.c2 = p->scale * kLog2e;
  a.q = p->q; a.k = p->k; a.v = p->v;
  a.q_bs = p->q_bs; a.q_ns = p->q_ns; a.q_hs = p->q_hs;
  a.o = p->o; a.g = p->dout; a.o_bs = p->o_bs; a.o_ns = p->o_ns; a.o_hs = p->o_hs;
  a.lse = p->lse;
  a.dq = p->dq; a.dk = p->dk; a.dv = p->dv;
  a.d_bs = p->dq_bs; a.d_ns = p->dq_ns; a.d_hs = p->dq_hs;
  a.dsum = p->dsum;
  if (p->dtype == MC_DTYPE_BF16) attn::launch_bwd<bf16_t>(a, (hipStream_t)stream);
  else attn::launch_bwd<f16_t>(a, (hipStream_t)stream);
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_attn_bwd: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}
