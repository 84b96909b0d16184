// mixer_proj.hip -- the Mamba mixer's skinny projections around the scan, fused (include/mc_ops.h:
// mc_mixer_proj_fwd / mc_mixer_proj_bwd), gfx950.
//
// Reference (the mixer the text tower stacks, upstream mamba_simple.Mamba, whose
// SS2D analogue is model.py:519-528 / 630-647):
//   x_dbl = x_proj(x)                   (P = R + 2N rows: dt_raw | B | C), P x D weight, K = D
//   delta = dt_proj.weight @ dt_raw     (D x R weight, K = R; the bias goes into the scan's softplus)
// and their input gradients
//   d_dtraw = dt_proj.weight^T @ ddelta,  dx = x_proj.weight^T @ [d_dtraw; dB; dC] + du (the scan's).
// Channel-major activations (D, T = batch * seqlen), tokens contiguous.  As library GEMMs these are
// four launches at 0.1-0.25 PFLOP/s: each moves a (D, T) activation with a reduction of 48-80, so they
// are HBM-bound, and the chain x -> x_dbl -> delta (dX <- d_xdbl <- ddelta) runs through HBM twice.
// Here one workgroup owns a 64-token tile and does the whole chain on-chip:
//  * forward: x_dbl tile (P x 64) accumulates on v_mfma_f32_16x16x16 over 64-channel chunks of x
//    (staged in LDS, double-buffered; the B operand by ds_read_b64_tr_b16 transposed reads), is
//    rounded to the activation dtype (what the x_proj GEMM stores) and kept in LDS; delta^T =
//    dt_raw^T Wdt^T on MFMA with the token on the accumulator rows, so each lane holds 4 consecutive
//    tokens of one channel; staged per wave in LDS and written as 128-B channel-row pieces.
//  * backward: d_dtraw (R x 64) over 64-channel chunks of ddelta (Wdt chunk and ddelta chunk in
//    LDS), rounded, joined with the scan's dB / dC rows into d_xdbl (written out for the weight
//    gradients: the B / C outputs are separate autograd outputs, so no zero-filled x_dbl gradient);
//    dx^T = d_xdbl^T Wx over 64-channel chunks of Wx (LDS), + du in the epilogue, 128-B row pieces.
// Bytes per token tile (C2, D 1536, P 80, R 48): forward reads 192 KB and writes 202 KB; backward reads
// 394 KB and writes 202 KB.  The weight gradients stay split-K library GEMMs (ops.wgrad): fused, each
// workgroup would emit a full fp32 partial of both weights.
#include <type_traits>

#include "scan_common.h"
#include "../../include/mc_ops.h"

namespace mc {
namespace mproj {
using scan::Mfma16;
using scan::xcd_remap;

constexpr int kTT = 64;                 // tokens per workgroup
constexpr int kKC = 64;                 // channels per staged chunk
constexpr int kLS = kKC + 8;            // LDS row stride in 16-bit elements (144 B: 16-B aligned, bank-skewed)
constexpr int kPMax = 128;              // x_dbl rows supported (R + 2N)
constexpr int kWaves = 8;              // two waves per SIMD per workgroup: the K loops are latency-bound
constexpr int kThreads = 64 * kWaves;
template <int I> using IC = std::integral_constant<int, I>;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// B-type fragment of a [row][col] 16-bit LDS image (row stride ls): lane l gets column col0 + (l & 15),
// rows row0 + 4 (l >> 4) + [0, 4).  ds_read_b64_tr_b16: lane 4q + p of each 16-lane group addresses
// row q, columns 4p .. 4p + 3; lane i receives column i of the 4 rows.
__device__ __forceinline__ s16x4 tr_frag(const uint16_t* img, int ls, int row0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15;
  const uint16_t* p = img + (row0 + 4 * g + (li >> 2)) * ls + col0 + 4 * (li & 3);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
}
// A-type fragment: lane l gets row row0 + (l & 15), columns col0 + 4 (l >> 4) + [0, 4) (8 contiguous B)
__device__ __forceinline__ s16x4 row_frag(const uint16_t* img, int ls, int row0, int col0, int lane) {
  return *reinterpret_cast<const s16x4*>(img + (row0 + (lane & 15)) * ls + col0 + 4 * (lane >> 4));
}

template <typename TI>
__device__ __forceinline__ f32x4 mma(s16x4 a, s16x4 b, f32x4 c) {
  using MM = Mfma16<TI>;
  return MM::mma(__builtin_bit_cast(typename MM::v4, a), __builtin_bit_cast(typename MM::v4, b), c);
}
template <typename TI>
__device__ __forceinline__ uint16_t h16(float x) { return (uint16_t)bits16<TI>(x); }

struct Args {
  int D, T, R, P;
  int64_t x_ld, xd_ld, dl_ld;              // forward: x, x_dbl, delta row strides
  int64_t gd_ld, gb_ld, gc_ld, du_ld, dxd_ld, dx_ld;   // backward
  const void* x; const void* wx; const void* wdt;
  void* xd; void* dl;
  const void* gd; const void* gb; const void* gc; const void* du;
  void* dxd; void* dx;
};

// 16-B pieces of a [rows][64 tokens] tile: global (row stride ld, tokens from t0) <-> LDS [row][kLS]
__device__ __forceinline__ uint4 ld_piece(__amdgpu_buffer_rsrc_t r, int64_t ld, int row, int t0, int cp) {
  return buf_ld16(r, (uint32_t)((row * ld + t0 + 8 * cp) * 2));
}

// ---------------------------------------------------------------------------- forward
// Phase 1: wave w owns token n-tile (w & 3) and k-steps {2 (w >> 2), 2 (w >> 2) + 1} of every 64-channel
// chunk (the two halves of the workgroup split K and sum through LDS at the end).  Phase 2: wave w owns
// delta n-tiles w, w + 8, ... with all four token m-tiles.  The next chunk's x / Wx pieces are loaded
// while the current one is multiplied (register sets by chunk parity).
template <typename TI, int MT>   // MT = P / 16 x_dbl row tiles
__global__ __launch_bounds__(kThreads, 1) void mixer_proj_fwd_kernel(const Args a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  constexpr int P = MT * 16;
  uint16_t* sx = smem;                                   // [2][kKC][kLS]   x chunks
  uint16_t* sw = sx + 2 * kKC * kLS;                     // [2][P][kLS]     Wx chunks; then the x_dbl tile [P][kLS]
  float* red = reinterpret_cast<float*>(sw + 2 * P * kLS);   // [P][kTT] fp32 K-half partials
  uint16_t* so = reinterpret_cast<uint16_t*>(red);       // phase 2: [kWaves][16][kLS] delta staging (over red)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int nw = w & 3, kh = w >> 2;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int t0 = tile * kTT;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (uint32_t)(((int64_t)(a.D - 1) * a.x_ld + a.T) * 2));
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.wx, (uint32_t)((int64_t)P * a.D * 2));

  constexpr int kWPer = (P * 8 + kThreads - 1) / kThreads;   // Wx pieces per thread
  uint4 rxv[2], rwv[2][kWPer];
  auto load_chunk = [&](int kc, auto set) __attribute__((always_inline)) {
    constexpr int S = decltype(set)::value;
    {
      const int row = tid >> 3, cp = tid & 7;   // 64 rows x 8 pieces: one per thread
      // tokens past T read 0 (range) or the row's tail (their columns are never stored)
      rxv[S] = ld_piece(rx, a.x_ld, kc * kKC + row, t0, cp);
    }
#pragma unroll
    for (int i = 0; i < kWPer; ++i) {
      const int q = tid + kThreads * i, row = q >> 3, cp = q & 7;
      rwv[S][i] = q < P * 8 ? buf_ld16(rw, (uint32_t)((row * a.D + kc * kKC + 8 * cp) * 2)) : make_uint4(0, 0, 0, 0);
    }
  };
  auto park_chunk = [&](auto set) __attribute__((always_inline)) {
    constexpr int S = decltype(set)::value;
    {
      const int row = tid >> 3, cp = tid & 7;
      *reinterpret_cast<uint4*>(sx + (S * kKC + row) * kLS + 8 * cp) = rxv[S];
    }
#pragma unroll
    for (int i = 0; i < kWPer; ++i) {
      const int q = tid + kThreads * i, row = q >> 3, cp = q & 7;
      if (q < P * 8) *reinterpret_cast<uint4*>(sw + (S * P + row) * kLS + 8 * cp) = rwv[S][i];
    }
  };

  // ---- phase 1: x_dbl (P x 64) = Wx . x_tile
  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = a.D / kKC;
  load_chunk(0, IC<0>());
  if (nk > 1) load_chunk(1, IC<1>());
  park_chunk(IC<0>());
  if (nk > 2) load_chunk(2, IC<0>());
  __syncthreads();
  auto step = [&](int kc, auto par) __attribute__((always_inline)) {
    constexpr int S = decltype(par)::value;   // kc & 1: LDS buffer and register set
    using N = IC<1 - S>;
    const uint16_t* cx = sx + S * kKC * kLS;
    const uint16_t* cw = sw + S * P * kLS;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int s = 2 * kh + s2;
      const s16x4 b = tr_frag(cx, kLS, 16 * s, 16 * nw, lane);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = mma<TI>(row_frag(cw, kLS, 16 * m, 16 * s, lane), b, acc[m]);
    }
    if (kc + 1 < nk) park_chunk(N());   // buffer 1 - S: its readers passed the last barrier
    if (kc + 3 < nk) load_chunk(kc + 3, N());
    __syncthreads();
  };
  for (int kc = 0; kc < nk; kc += 2) {
    step(kc, IC<0>());
    if (kc + 1 < nk) step(kc + 1, IC<1>());
  }
  // K halves summed through LDS (fixed order: half 0 + half 1), rounded to the activation dtype (what
  // the x_proj GEMM stores), kept as the x_dbl tile [p][token] over the Wx chunks
  if (kh == 1) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[(16 * m + 4 * g + j) * kTT + 16 * nw + li] = acc[m][j];
  }
  __syncthreads();
  uint16_t* sd = sw;
  if (kh == 0) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 16 * m + 4 * g + j;
        sd[r * kLS + 16 * nw + li] = h16<TI>(acc[m][j] + red[r * kTT + 16 * nw + li]);
      }
  }
  __syncthreads();
  for (int q = tid; q < P * 8; q += kThreads) {   // x_dbl to HBM
    const int row = q >> 3, cp = q & 7;
    if (t0 + 8 * cp < a.T)
      *reinterpret_cast<uint4*>(reinterpret_cast<TI*>(a.xd) + row * a.xd_ld + t0 + 8 * cp) =
          *reinterpret_cast<const uint4*>(sd + row * kLS + 8 * cp);
  }

  // ---- phase 2: delta^T (64 x D) = dt_raw^T (64 x R) . Wdt^T (R x D); token on the accumulator rows
  constexpr int RS = MT - 2;   // dstate 16: R = P - 32
  s16x4 afr[4][RS];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int s = 0; s < RS; ++s) afr[mt][s] = tr_frag(sd, kLS, 16 * s, 16 * mt, lane);
  uint16_t* sow = so + w * 16 * kLS;
  const TI* wdt = reinterpret_cast<const TI*>(a.wdt);
  // Wdt fragments (L2) one n-tile ahead
  s16x4 bfr[RS], bnx[RS];
#pragma unroll
  for (int s = 0; s < RS; ++s) bnx[s] = *reinterpret_cast<const s16x4*>(wdt + (int64_t)(16 * w + li) * a.R + 16 * s + 4 * g);
  for (int nt = w; nt < a.D / 16; nt += kWaves) {
    const int c0 = 16 * nt;
#pragma unroll
    for (int s = 0; s < RS; ++s) bfr[s] = bnx[s];
    if (nt + kWaves < a.D / 16) {
#pragma unroll
      for (int s = 0; s < RS; ++s)
        bnx[s] = *reinterpret_cast<const s16x4*>(wdt + (int64_t)(c0 + 16 * kWaves + li) * a.R + 16 * s + 4 * g);
    }
    f32x4 d[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      d[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < RS; ++s) d[mt] = mma<TI>(afr[mt][s], bfr[s], d[mt]);
    }
    // lane: channel c0 + li, tokens 16 mt + 4 g + [0, 4) -> staging [channel][token]
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      *reinterpret_cast<uint2*>(sow + li * kLS + 16 * mt + 4 * g) =
          make_uint2(cvt_pk2<TI>(d[mt][0], d[mt][1]), cvt_pk2<TI>(d[mt][2], d[mt][3]));
    asm volatile("" ::: "memory");   // one wave: its LDS ops complete in order
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = lane + 64 * i, ch = q >> 3, cp = q & 7;
      const uint4 v = *reinterpret_cast<const uint4*>(sow + ch * kLS + 8 * cp);
      if (t0 + 8 * cp < a.T)
        *reinterpret_cast<uint4*>(reinterpret_cast<TI*>(a.dl) + (int64_t)(c0 + ch) * a.dl_ld + t0 + 8 * cp) = v;
    }
    asm volatile("" ::: "memory");
  }
}

// ---------------------------------------------------------------------------- backward (input gradients)
// Phase 1 as the forward's (d_dtraw over chunks of ddelta, K halves per wave group).  Phase 2 per 64-channel
// chunk of Wx: wave w owns channel n-tile (w & 3) and token m-tiles {2 (w >> 2), +1}; the chunk's dx
// (64 channels x 64 tokens) is staged in LDS and written by all threads as 128-B row pieces.
template <typename TI, int MT>   // P = 16 MT, R = 16 (MT - 2): dstate 16
__global__ __launch_bounds__(kThreads, 1) void mixer_proj_bwd_kernel(const Args a) {
  constexpr int RT = MT - 2;
  constexpr int P = MT * 16;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int R = a.R;
  const int lsr = R + 8;                                  // Wdt chunk row stride (16-B rows: R % 16 == 0)
  uint16_t* sg = smem;                                   // phase 1: [2][kKC][kLS] ddelta chunks
  uint16_t* st = sg + 2 * kKC * kLS;                     //          [2][kKC][lsr] Wdt chunks
  uint16_t* swx = smem;                                  // phase 2: [2][P][kLS]   Wx column chunks (aliases)
  const int ph1 = 2 * kKC * kLS + 2 * kKC * lsr, ph2 = 2 * P * kLS;
  uint16_t* sdx = smem + (ph1 > ph2 ? ph1 : ph2);        // [P][kLS] d_xdbl tile
  float* red = reinterpret_cast<float*>(sdx + P * kLS);  // [R][kTT] fp32 K-half partials
  uint16_t* stg = reinterpret_cast<uint16_t*>(red);      // phase 2: [2][kKC][kLS] dx staging (over red)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int nw = w & 3, kh = w >> 2;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int t0 = tile * kTT;
  const __amdgpu_buffer_rsrc_t rg = make_rsrc(a.gd, (uint32_t)(((int64_t)(a.D - 1) * a.gd_ld + a.T) * 2));
  const __amdgpu_buffer_rsrc_t rt = make_rsrc(a.wdt, (uint32_t)((int64_t)a.D * R * 2));
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.wx, (uint32_t)((int64_t)P * a.D * 2));
  const int nk = a.D / kKC;

  // ---- phase 1: d_dtraw (R x 64) = Wdt^T . ddelta_tile over channel chunks
  {
    const int tpr = R / 8;                                // 16-B pieces per Wdt row
    const int tq = (kKC * tpr + kThreads - 1) / kThreads;  // per thread (R <= 96: <= 2)
    uint4 rgv[2], rtv[2][2];
    auto load_chunk = [&](int kc, auto set) __attribute__((always_inline)) {
      constexpr int S = decltype(set)::value;
      {
        const int row = tid >> 3, cp = tid & 7;
        rgv[S] = ld_piece(rg, a.gd_ld, kc * kKC + row, t0, cp);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int q = tid + kThreads * i, row = q / tpr, cp = q % tpr;
        rtv[S][i] = (i < tq && q < kKC * tpr) ? buf_ld16(rt, (uint32_t)(((kc * kKC + row) * R + 8 * cp) * 2))
                                              : make_uint4(0, 0, 0, 0);
      }
    };
    auto park_chunk = [&](auto set) __attribute__((always_inline)) {
      constexpr int S = decltype(set)::value;
      {
        const int row = tid >> 3, cp = tid & 7;
        *reinterpret_cast<uint4*>(sg + (S * kKC + row) * kLS + 8 * cp) = rgv[S];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int q = tid + kThreads * i, row = q / tpr, cp = q % tpr;
        if (i < tq && q < kKC * tpr) *reinterpret_cast<uint4*>(st + (S * kKC + row) * lsr + 8 * cp) = rtv[S][i];
      }
    };
    f32x4 acc[RT];
#pragma unroll
    for (int m = 0; m < RT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    load_chunk(0, IC<0>());
    if (nk > 1) load_chunk(1, IC<1>());
    park_chunk(IC<0>());
    if (nk > 2) load_chunk(2, IC<0>());
    __syncthreads();
    auto step = [&](int kc, auto par) __attribute__((always_inline)) {
      constexpr int S = decltype(par)::value;
      using N = IC<1 - S>;
      const uint16_t* cg = sg + S * kKC * kLS;
      const uint16_t* ct = st + S * kKC * lsr;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int s = 2 * kh + s2;
        const s16x4 b = tr_frag(cg, kLS, 16 * s, 16 * nw, lane);
#pragma unroll
        for (int m = 0; m < RT; ++m)   // A[r][c] = Wdt[c][r]: transposed read of the [c][r] chunk
          acc[m] = mma<TI>(tr_frag(ct, lsr, 16 * s, 16 * m, lane), b, acc[m]);
      }
      if (kc + 1 < nk) park_chunk(N());
      if (kc + 3 < nk) load_chunk(kc + 3, N());
      __syncthreads();
    };
    for (int kc = 0; kc < nk; kc += 2) {
      step(kc, IC<0>());
      if (kc + 1 < nk) step(kc + 1, IC<1>());
    }
    // rows 0 .. R-1 of d_xdbl: the K halves summed (half 0 + half 1), rounded as the dt_proj
    // input-gradient GEMM stores it; rows R .. P-1: dB / dC as given (16 rows each)
    if (kh == 1) {
#pragma unroll
      for (int m = 0; m < RT; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[(16 * m + 4 * g + j) * kTT + 16 * nw + li] = acc[m][j];
    }
    for (int q = tid; q < (P - R) * 8; q += kThreads) {
      const int row = q >> 3, cp = q & 7;   // row of the B / C block (0 .. 31)
      const TI* src = reinterpret_cast<const TI*>(row < 16 ? a.gb : a.gc);
      const int64_t ld = row < 16 ? a.gb_ld : a.gc_ld;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (src && t0 + 8 * cp < a.T) v = *reinterpret_cast<const uint4*>(src + (int64_t)(row & 15) * ld + t0 + 8 * cp);
      *reinterpret_cast<uint4*>(sdx + (R + row) * kLS + 8 * cp) = v;
    }
    __syncthreads();
    if (kh == 0) {
#pragma unroll
      for (int m = 0; m < RT; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 16 * m + 4 * g + j;
          sdx[r * kLS + 16 * nw + li] = h16<TI>(acc[m][j] + red[r * kTT + 16 * nw + li]);
        }
    }
  }
  __syncthreads();
  for (int q = tid; q < P * 8; q += kThreads) {   // d_xdbl to HBM (the weight gradients' operand)
    const int row = q >> 3, cp = q & 7;
    if (t0 + 8 * cp < a.T)
      *reinterpret_cast<uint4*>(reinterpret_cast<TI*>(a.dxd) + row * a.dxd_ld + t0 + 8 * cp) =
          *reinterpret_cast<const uint4*>(sdx + row * kLS + 8 * cp);
  }

  // ---- phase 2: dx^T (64 x D) = d_xdbl^T (64 x P) . Wx (P x D) + du^T
  const int mh = kh;   // token half: m-tiles 2 mh, 2 mh + 1
  s16x4 afr[2][MT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int s = 0; s < MT; ++s) afr[i][s] = tr_frag(sdx, kLS, 16 * s, 16 * (2 * mh + i), lane);
  constexpr int kWPer = (P * 8 + kThreads - 1) / kThreads;
  uint4 rwv[2][kWPer];   // Wx chunks, the next one in flight (register sets by chunk parity)
  uint2 duv[2][2];       // du pieces, one chunk ahead
  const TI* du = reinterpret_cast<const TI*>(a.du);
  auto load_w = [&](int kc, auto set) __attribute__((always_inline)) {
    constexpr int S = decltype(set)::value;
#pragma unroll
    for (int i = 0; i < kWPer; ++i) {
      const int q = tid + kThreads * i, row = q >> 3, cp = q & 7;
      rwv[S][i] = q < P * 8 ? buf_ld16(rw, (uint32_t)((row * a.D + kc * kKC + 8 * cp) * 2)) : make_uint4(0, 0, 0, 0);
    }
  };
  auto park_w = [&](auto set) __attribute__((always_inline)) {
    constexpr int S = decltype(set)::value;
#pragma unroll
    for (int i = 0; i < kWPer; ++i) {
      const int q = tid + kThreads * i, row = q >> 3, cp = q & 7;
      if (q < P * 8) *reinterpret_cast<uint4*>(swx + (S * P + row) * kLS + 8 * cp) = rwv[S][i];
    }
  };
  auto load_du = [&](int kc, auto set) __attribute__((always_inline)) {
    constexpr int S = decltype(set)::value;
    const int c = kc * kKC + 16 * nw + li;   // this lane's channel
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int t = t0 + 16 * (2 * mh + i) + 4 * g;
      duv[S][i] = (du && t < a.T) ? *reinterpret_cast<const uint2*>(du + (int64_t)c * a.du_ld + t) : make_uint2(0, 0);
    }
  };
  __syncthreads();   // phase-1 buffers and red are dead: Wx chunks / staging go over them
  load_w(0, IC<0>());
  if (nk > 1) load_w(1, IC<1>());
  load_du(0, IC<0>());
  park_w(IC<0>());
  if (nk > 2) load_w(2, IC<0>());
  __syncthreads();
  auto step = [&](int kc, auto par) __attribute__((always_inline)) {
    constexpr int S = decltype(par)::value;
    using N = IC<1 - S>;
    if (kc + 1 < nk) load_du(kc + 1, N());
    const uint16_t* cw = swx + S * P * kLS;
    s16x4 bfr[MT];
#pragma unroll
    for (int s = 0; s < MT; ++s) bfr[s] = tr_frag(cw, kLS, 16 * s, 16 * nw, lane);
    uint16_t* sgt = stg + S * kKC * kLS;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < MT; ++s) d = mma<TI>(afr[i][s], bfr[s], d);
      // + du (fp32, then one rounding: the library's beta = 1 epilogue); lane: channel 16 nw + li of the
      // chunk, tokens 16 (2 mh + i) + 4 g + j
      const uint4 q4 = make_uint4(duv[S][i].x, duv[S][i].y, 0u, 0u);
      const float v0 = d[0] + elem_f<TI>(q4, 0), v1 = d[1] + elem_f<TI>(q4, 1);
      const float v2 = d[2] + elem_f<TI>(q4, 2), v3 = d[3] + elem_f<TI>(q4, 3);
      *reinterpret_cast<uint2*>(sgt + (16 * nw + li) * kLS + 16 * (2 * mh + i) + 4 * g) =
          make_uint2(cvt_pk2<TI>(v0, v1), cvt_pk2<TI>(v2, v3));
    }
    __syncthreads();   // the chunk's dx tile is staged
    {
      const int row = tid >> 3, cp = tid & 7;   // 64 channels x 8 pieces: one per thread
      const uint4 v = *reinterpret_cast<const uint4*>(sgt + row * kLS + 8 * cp);
      if (t0 + 8 * cp < a.T)
        *reinterpret_cast<uint4*>(reinterpret_cast<TI*>(a.dx) + (int64_t)(kc * kKC + row) * a.dx_ld + t0 + 8 * cp) = v;
    }
    if (kc + 1 < nk) park_w(N());   // buffer 1 - S: its readers passed the barrier above
    if (kc + 3 < nk) load_w(kc + 3, N());
    __syncthreads();
  };
  for (int kc = 0; kc < nk; kc += 2) {
    step(kc, IC<0>());
    if (kc + 1 < nk) step(kc + 1, IC<1>());
  }
}

size_t fwd_lds(int P) {
  const size_t red = (size_t)P * kTT * 4, stage = (size_t)kWaves * 16 * kLS * 2;
  return (size_t)(2 * kKC * kLS + 2 * P * kLS) * 2 + (red > stage ? red : stage);
}
size_t bwd_lds(int P, int R) {
  const int ph1 = 2 * kKC * kLS + 2 * kKC * (R + 8), ph2 = 2 * P * kLS;
  const size_t red = (size_t)R * kTT * 4, stage = (size_t)2 * kKC * kLS * 2;
  return (size_t)((ph1 > ph2 ? ph1 : ph2) + P * kLS) * 2 + (red > stage ? red : stage);
}

template <typename TI, int MT>
static void launch(bool fwd, const Args& a, hipStream_t s) {
  const dim3 grid((a.T + kTT - 1) / kTT), block(kThreads);
  if (fwd) hipLaunchKernelGGL((mixer_proj_fwd_kernel<TI, MT>), grid, block, fwd_lds(MT * 16), s, a);
  else hipLaunchKernelGGL((mixer_proj_bwd_kernel<TI, MT>), grid, block, bwd_lds(MT * 16, a.R), s, a);
}
template <typename TI>
static void launch_t(bool fwd, const Args& a, hipStream_t s) {
  switch (a.P / 16) {   // P = R + 32 (dstate 16), R >= 16
    case 3: launch<TI, 3>(fwd, a, s); break;
    case 4: launch<TI, 4>(fwd, a, s); break;
    case 5: launch<TI, 5>(fwd, a, s); break;
    case 6: launch<TI, 6>(fwd, a, s); break;
    case 7: launch<TI, 7>(fwd, a, s); break;
    default: launch<TI, 8>(fwd, a, s); break;
  }
}

static bool a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

static int check_common(int D, int T, int R, int P, int dtype, const char* who) {
  MC_CHECK(dtype == MC_DTYPE_BF16 || dtype == MC_DTYPE_F16, MC_ERR_DTYPE, "%s: bf16 / f16 only (got %d)", who, dtype);
  MC_CHECK(D > 0 && D % kKC == 0 && T >= 0 && T % 8 == 0 && R >= 16 && R % 16 == 0 && P == R + 32 && P <= kPMax,
           MC_ERR_SHAPE, "%s: needs dim %% 64 == 0, tokens %% 8 == 0, rank %% 16 == 0 in [16, 96], proj_rows = rank + 32 "
           "(dstate 16) (got dim %d, tokens %d, rank %d, proj_rows %d)", who, D, T, R, P);
  return MC_OK;
}

}  // namespace mproj
}  // namespace mc

using namespace mc;
using namespace mc::mproj;

extern "C" int mc_mixer_proj_fwd(const mc_mixer_proj_params* p, void* stream) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_mixer_proj_fwd: null params");
  int rc = check_common(p->dim, p->tokens, p->rank, p->proj_rows, p->dtype, "mc_mixer_proj_fwd");
  if (rc) return rc;
  if (p->tokens == 0) return MC_OK;
  MC_CHECK(p->x && p->w_x && p->w_dt && p->x_dbl && p->delta, MC_ERR_INVALID, "mc_mixer_proj_fwd: null pointer");
  MC_CHECK(a16(p->x) && a16(p->x_dbl) && a16(p->delta) && a16(p->w_x) && (reinterpret_cast<uintptr_t>(p->w_dt) & 7) == 0 &&
               p->x_ld % 8 == 0 && p->x_dbl_ld % 8 == 0 && p->delta_ld % 8 == 0 && p->x_ld >= p->tokens &&
               p->x_dbl_ld >= p->tokens && p->delta_ld >= p->tokens &&
               ((int64_t)(p->dim - 1) * p->x_ld + p->tokens) * 2 < ((int64_t)1 << 31),
           MC_ERR_INVALID, "mc_mixer_proj_fwd: 16-B aligned rows (strides %% 8), strides >= tokens, 32-bit spans");
  Args a{};
  a.D = p->dim; a.T = p->tokens; a.R = p->rank; a.P = p->proj_rows;
  a.x_ld = p->x_ld; a.xd_ld = p->x_dbl_ld; a.dl_ld = p->delta_ld;
  a.x = p->x; a.wx = p->w_x; a.wdt = p->w_dt; a.xd = p->x_dbl; a.dl = p->delta;
  hipStream_t s = (hipStream_t)stream;
  if (p->dtype == MC_DTYPE_BF16) launch_t<bf16_t>(true, a, s);
  else launch_t<f16_t>(true, a, s);
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_mixer_proj_fwd: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

extern "C" int mc_mixer_proj_bwd(const mc_mixer_proj_bwd_params* p, void* stream) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_mixer_proj_bwd: null params");
  int rc = check_common(p->dim, p->tokens, p->rank, p->proj_rows, p->dtype, "mc_mixer_proj_bwd");
  if (rc) return rc;
  if (p->tokens == 0) return MC_OK;
  MC_CHECK(p->g_delta && p->w_x && p->w_dt && p->d_x_dbl && p->dx, MC_ERR_INVALID, "mc_mixer_proj_bwd: null pointer");
  MC_CHECK(a16(p->g_delta) && a16(p->d_x_dbl) && a16(p->dx) && a16(p->w_x) && a16(p->w_dt) &&
               (!p->g_b || (a16(p->g_b) && p->g_b_ld % 8 == 0 && p->g_b_ld >= p->tokens)) &&
               (!p->g_c || (a16(p->g_c) && p->g_c_ld % 8 == 0 && p->g_c_ld >= p->tokens)) &&
               (!p->du || ((reinterpret_cast<uintptr_t>(p->du) & 7) == 0 && p->du_ld % 4 == 0 && p->du_ld >= p->tokens)) &&
               p->g_delta_ld % 8 == 0 && p->d_x_dbl_ld % 8 == 0 && p->dx_ld % 8 == 0 && p->g_delta_ld >= p->tokens &&
               p->d_x_dbl_ld >= p->tokens && p->dx_ld >= p->tokens &&
               ((int64_t)(p->dim - 1) * p->g_delta_ld + p->tokens) * 2 < ((int64_t)1 << 31),
           MC_ERR_INVALID, "mc_mixer_proj_bwd: 16-B aligned rows (du: 8-B), strides >= tokens, 32-bit spans");
  Args a{};
  a.D = p->dim; a.T = p->tokens; a.R = p->rank; a.P = p->proj_rows;
  a.gd_ld = p->g_delta_ld; a.gb_ld = p->g_b_ld; a.gc_ld = p->g_c_ld; a.du_ld = p->du_ld; a.dxd_ld = p->d_x_dbl_ld;
  a.dx_ld = p->dx_ld;
  a.wx = p->w_x; a.wdt = p->w_dt; a.gd = p->g_delta; a.gb = p->g_b; a.gc = p->g_c; a.du = p->du; a.dxd = p->d_x_dbl;
  a.dx = p->dx;
  hipStream_t s = (hipStream_t)stream;
  if (p->dtype == MC_DTYPE_BF16) launch_t<bf16_t>(false, a, s);
  else launch_t<f16_t>(false, a, s);
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_mixer_proj_bwd: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}
