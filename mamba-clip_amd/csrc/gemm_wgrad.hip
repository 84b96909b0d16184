// gemm_wgrad.hip -- long-reduction weight-gradient GEMM of the towers' projections (bf16 / f16 in, fp32 out).
//
//   C[m][n] = sum_t A(t, m) B(t, n)      (M, N <= a few thousand; T = batch * tokens, tens of thousands)
//
// This is dW = G^T X of every Linear in the image / text towers' backward (reference: the towers behind
// encode_image / encode_text, /root/reference/src/mamba_clip/model.py:1011-1017; built at model.py:1270):
// G is the output gradient, X the saved input, T the token count (C2 ViT: 50,432).  The output is
// small (<= 9 tiles of 256 x 256 for the 768-wide layers) and the reduction long, so the launch
// splits T over S workgroups per output tile (S ~ 256 CUs / tiles), writes one fp32 partial tile per
// split into a slab workspace and sums the S slabs in a fixed order (mc_sum_slabs): deterministic.
//
// Operand layouts (per operand, template flags):
//  * token-major (TM): row t holds the features, A(t, m) = A[t * lda + m] -- a Linear's (tokens,
//    features) activations / gradients.  The LDS tile is [64 t][256 features] (512-B rows, as the
//    rows arrive from HBM) and MFMA fragments are read TRANSPOSED with ds_read_b64_tr_b16 (each lane
//    gets 4 consecutive t of one feature; two reads make the 8 of a 16x16x32 operand);
//  * feature-major (FM): row m holds the tokens, A(t, m) = A[m * lda + t] -- the Mamba mixer's
//    channel-major activations.  The LDS tile is [256 features][64 t] (128-B rows) and fragments
//    are plain ds_read_b128 row reads.
// Both land in LDS by global_load_lds_dwordx4 (16 B per lane, no VGPR round trip); the image is
// lane-linear, so the bank swizzle sits on the SOURCE address and the matching read:
//  * TM: 16-B chunk c of row r lives at slot c ^ 2 s(r), s(r) = (r & 3) | ((r >> 3) & 1) << 2 --
//    the 8 rows of a half-wave's transposed read (4 rows per 16-lane group, groups 8 rows apart)
//    land on 8 distinct 32-B bank slots: conflict-free;
//  * FM: chunk c of row r at slot c ^ ((r >> 1) & 7) (16 consecutive rows reading one chunk hit 16
//    distinct 16-B bank slots; as sim_fp8_kernel).
// Tile 256 x 256 x 64, 8 waves as 2 (m) x 4 (n), 128 x 64 per wave on v_mfma_f32_16x16x32_{bf16,f16}
// (32 accumulators); two LDS stages of 64 KB, the next step's loads in flight across the step's
// MFMAs (counted vmcnt, raw s_barrier), one workgroup per CU.
#include <type_traits>

#include "mc_common.h"
#include "../../include/mc_gemm.h"

extern "C" int mc_sum_slabs(int32_t s, int64_t n, const float* src, int64_t slab_stride, float* dst, void* stream);
extern "C" int mc_colsum_fold(int32_t nslices, int32_t cols, const float* part, float* out, void* stream);

namespace mc {
namespace wgrad {

constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kThreads = 512;
constexpr int kTileBytes = kBM * kBK * 2;       // one operand tile (32 KB)
constexpr int kStage = 2 * kTileBytes;          // A + B (64 KB)

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) char lds_char;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

struct Args {
  int M, N, T, splits, tiles_m, tiles_n, nk;
  const char* A; const char* B;
  int64_t lda, ldb;          // elements
  float* C; int64_t ldc;     // output (splits == 1) or slab base (slab s at C + s * slab_stride)
  int64_t slab_stride;
  // 16-bit epilogues (kEpi != kEpiSlab, mc_linear): the tile is stored TRANSPOSED, Y[n][m] -- n the
  // token (Y's row), m the feature (Y's column)
  void* Y; int64_t ldy;
  void* Y2; int64_t ldy2;    // kEpiBiasGelu: gelu(h)
  const void* bias;          // kEpiBias / kEpiBiasGelu: per feature m, operand dtype
  const void* H; int64_t ldh;   // kEpiGeluGrad: pre-activation at Y's positions
  float* colpart;            // kEpiGeluGrad: column sums of Y per token tile, [tiles_n][M] (or null)
};

// epilogues of wgrad4p_kernel
constexpr int kEpiSlab = 0;       // fp32 C (or split-K slab), row m / column n
constexpr int kEpiStore = 1;      // Y = C^T, 16-bit
constexpr int kEpiBias = 2;       // Y = C^T + bias
constexpr int kEpiBiasGelu = 3;   // Y = h = C^T + bias, Y2 = gelu(h)
constexpr int kEpiGeluGrad = 4;   // Y = round(C^T) * gelu'(H), column sums of Y

// One global_load_lds_dwordx4: 16 B per lane from gsrc to LDS byte address m0v + 16 * lane (m0v
// wave-uniform).  asm, so hipcc's waitcnt pass does not drain it at the next LDS read; the loop
// counts completion with its own vmcnt.  M0 is compiler-reserved: saved and restored here.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t m0v) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(m0v) : "memory");
}

template <typename T>
__device__ __forceinline__ f32x4 mfma(const s16x8& a, const s16x8& b, const f32x4& c) {
  if constexpr (std::is_same<T, bf16_t>::value)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

__device__ __forceinline__ s16x8 cat8(s16x4 lo, s16x4 hi) {
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// swizzled 16-B slot of chunk c in row r
__device__ __forceinline__ int tm_slot(int r, int c) { return c ^ (2 * ((r & 3) | (((r >> 3) & 1) << 2))); }
__device__ __forceinline__ int fm_slot(int r, int c) { return c ^ ((r >> 1) & 7); }

// glds source pointers of one operand tile for this lane (kInstr = 4 per wave): TM rows of 512 B (two
// rows per instruction), FM rows of 128 B (eight rows per instruction).  Features past `dim` are
// clamped (their results are never stored); the token range is always in bounds (T % 64 == 0).
template <bool kFM>
__device__ __forceinline__ void tile_sources(const char* base, int64_t ld, int dim, int f0, int w, int lane,
                                             const char* (&src)[4], int64_t& step_bytes) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int pos = w * 4096 + j * 1024 + lane * 16;   // byte in the tile image
    if constexpr (!kFM) {
      const int r = pos >> 9, slot = (pos >> 4) & 31;   // row = token, 32 chunks of 8 features
      const int c = tm_slot(r, slot);                   // involution: slot <-> chunk
      const int f = min(f0 + 8 * c, dim - 8);
      src[j] = base + ((int64_t)r * ld + f) * 2;
    } else {
      const int r = pos >> 7, slot = (pos >> 4) & 7;    // row = feature, 8 chunks of 8 tokens
      const int c = fm_slot(r, slot);
      const int f = min(f0 + r, dim - 1);
      src[j] = base + ((int64_t)f * ld + 8 * c) * 2;
    }
  }
  step_bytes = kFM ? (int64_t)kBK * 2 : (int64_t)kBK * ld * 2;
}

template <typename T, bool kAFM, bool kBFM>
__global__ __launch_bounds__(kThreads, 1) void wgrad_kernel(const Args g) {
  __shared__ __attribute__((aligned(16))) char lds[2 * kStage];   // the only LDS object
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  // XCD-aware order: consecutive linear ids (same split, neighbouring tiles) share an XCD's L2
  const int tiles = g.tiles_m * g.tiles_n;
  const int nwg = tiles * g.splits;
  const int bid0 = blockIdx.x, xcd = bid0 & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid0 >> 3);
  const int split = lin / tiles, tile = lin % tiles;
  const int tm = tile % g.tiles_m, tn = tile / g.tiles_m;
  const int m0 = tm * kBM, n0 = tn * kBN;
  const int k_begin = (int)(((int64_t)split * g.nk) / g.splits), k_end = (int)(((int64_t)(split + 1) * g.nk) / g.splits);
  const int nk = k_end - k_begin;

  const char* srcA[4];
  const char* srcB[4];
  int64_t stepA, stepB;
  tile_sources<kAFM>(g.A, g.lda, g.M, m0, w, lane, srcA, stepA);
  tile_sources<kBFM>(g.B, g.ldb, g.N, n0, w, lane, srcB, stepB);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    srcA[j] += stepA * k_begin;
    srcB[j] += stepB * k_begin;
  }
  const uint32_t lds_w = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)(lds) + 4096u * w);
  auto issue = [&](int step) __attribute__((always_inline)) {   // K step `step` (local) into stage step & 1
    const uint32_t la = lds_w + (uint32_t)(step & 1) * kStage, lb = la + kTileBytes;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      glds16(srcA[j] + stepA * step, la + j * 1024);
      glds16(srcB[j] + stepB * step, lb + j * 1024);
    }
  };

  // ---- fragment read offsets (bytes within a stage's operand image)
  // TM (transposed reads): lane l = 16 g + 4 q + p supplies row 8 g + 4 h + q (+ 32 kk), features
  // [base + 4 p, +4): chunk base / 8 + (p >> 1), half 8 (p & 1).  s(r) = q | (g & 1) << 2 for every
  // kk / h, so the slot XOR is a per-lane constant.
  // FM (row reads): lane row (l & 15) of a 16-row tile, tokens [8 (l >> 4), +8) (+ 32 kk): chunk
  // (l >> 4) + 4 kk.
  const int fg = lane >> 4, fi = lane & 15, fq = fi >> 2, fp = fi & 3;
  int offA[8], offB[4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const int base = wr * 128 + mi * 16;
    if constexpr (!kAFM) {
      const int r = 8 * fg + fq;
      offA[mi] = r * 512 + (tm_slot(r, base / 8 + (fp >> 1)) << 4) + 8 * (fp & 1);
    } else {
      const int r = base + fi;
      offA[mi] = r * 128;   // + slot (depends on kk) at the read
    }
  }
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int base = wc * 64 + ni * 16;
    if constexpr (!kBFM) {
      const int r = 8 * fg + fq;
      offB[ni] = r * 512 + (tm_slot(r, base / 8 + (fp >> 1)) << 4) + 8 * (fp & 1);
    } else {
      const int r = base + fi;
      offB[ni] = r * 128;
    }
  }
  auto frag = [&](const char* img, int off, int row_for_fm, int kk, auto is_fm) __attribute__((always_inline)) -> s16x8 {
    if constexpr (!decltype(is_fm)::value) {
      const lds_char* p = (const lds_char*)(img) + off + kk * 32 * 512;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * 512));
      return cat8(lo, hi);
    } else {
      const int slot = fm_slot(row_for_fm, fg + 4 * kk);
      return *reinterpret_cast<const s16x8*>(img + off + (slot << 4));
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) issue(0);
  if (nk > 1) issue(1);
  for (int s = 0; s < nk; ++s) {
    // this wave's 8 loads of step s done (step s + 1's 8 may stay in flight), then everyone's
    if (s + 1 < nk) __builtin_amdgcn_s_waitcnt(0x0F78);   // vmcnt(8)
    else __builtin_amdgcn_s_waitcnt(0x0F70);              // vmcnt(0)
    __builtin_amdgcn_s_barrier();
    const char* la = lds + (s & 1) * kStage;
    const char* lb = la + kTileBytes;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s16x8 af[8], bfr[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        bfr[ni] = frag(lb, offB[ni], wc * 64 + ni * 16 + fi, kk, std::integral_constant<bool, kBFM>());
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
        af[mi] = frag(la, offA[mi], wr * 128 + mi * 16 + fi, kk, std::integral_constant<bool, kAFM>());
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma<T>(af[mi], bfr[ni], acc[mi][ni]);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's fragment reads are done
    __builtin_amdgcn_s_barrier();         // ... and everyone's: the stage can be refilled
    if (s + 2 < nk) issue(s + 2);
  }

  // ---- epilogue: fp32 tile (or this split's partial tile) -> C / slab.  acc[mi][ni] lane l holds
  // rows 4 (l >> 4) + [0, 4) and column l & 15 of its 16 x 16 block.
  float* C = g.C + (int64_t)split * g.slab_stride;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col = n0 + wc * 64 + ni * 16 + fi;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * 128 + mi * 16 + 4 * fg + r;
        if (row < g.M && col < g.N) C[(int64_t)row * g.ldc + col] = acc[mi][ni][r];
      }
    }
}

// ------------------------------------------------------------------ 4-phase-per-K-step pipeline
// Same tile / waves / operand layouts as wgrad_kernel, but each 64-deep K step is split into four
// phases of 16 MFMAs (one quadrant of a wave's 128 x 64 output: 64 x 32 over K 64), and the stage
// is split into HALF-tiles by quadrant: A half qm = the rows {wr * 128 + qm * 64 + [0, 64)} of both
// wave rows, B half qn = the columns {wc * 64 + qn * 32 + [0, 32)} of the four wave columns.  Each
// half is read in known phases only, so it is restaged for the step after next as soon as its last
// reader phase has retired its reads (a barrier later), one half-tile (two glds per thread) per phase:
//   phase 1: read B qn0 + A qm0, MFMA (0, 0);  issue B half 0 of step t + 1   (last read: t - 1, phase 4)
//   phase 2: read B qn1,         MFMA (0, 1);  issue A half 0 of step t + 2   (last read: t, phase 1)
//   phase 3: read A qm1,         MFMA (1, 1);  issue B half 1 of step t + 2   (last read: t, phase 2)
//   phase 4: read B qn0,         MFMA (1, 0);  issue A half 1 of step t + 2   (last read: t, phase 3)
// and the only vmcnt wait is at phase 4: vmcnt(6) leaves phases 2-4's three half-tiles in flight and
// retires everything step t + 1 needs.  Two LDS stages x 4 half-tiles x 16 KB = 128 KB.
// (cdna_hip_programming.md section 5, "the 256^2 8-phase template": the same structure, one K step
// per four phases.)
constexpr int kHalf = 16 * 1024;     // one half-tile image (A or B, 128 features x 64 tokens)

template <bool kFM, bool kIsA>
__device__ __forceinline__ void half_sources(const char* base, int64_t ld, int dim, int f0, int h, int w, int lane,
                                             const char* (&src)[2]) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int pos = w * 2048 + j * 1024 + lane * 16;   // byte in the half image
    int r, c, fl;                                       // image row, logical chunk, feature of the chunk / row
    if constexpr (!kFM) {
      r = pos >> 8;                                     // token row of 256 B = 16 chunks of 8 features
      c = tm_slot(r, (pos >> 4) & 15);
      fl = kIsA ? ((c >> 3) * 128 + h * 64 + (c & 7) * 8) : ((c >> 2) * 64 + h * 32 + (c & 3) * 8);
      const int f = min(f0 + fl, dim - 8);
      src[j] = base + ((int64_t)r * ld + f) * 2;
    } else {
      r = pos >> 7;                                     // feature row of 128 B = 8 chunks of 8 tokens
      c = fm_slot(r, (pos >> 4) & 7);
      fl = kIsA ? ((r >> 6) * 128 + h * 64 + (r & 63)) : ((r >> 5) * 64 + h * 32 + (r & 31));
      const int f = min(f0 + fl, dim - 1);
      src[j] = base + ((int64_t)f * ld + 8 * c) * 2;
    }
  }
}

// kStagger: the wave row wr = 1 runs one barrier behind wr = 0 (an extra s_barrier before the loop,
// wr = 0 takes its extra one after it), so on every SIMD -- which holds one wave of each row -- one
// wave's fragment reads overlap the other's MFMA cluster.  Each phase then retires its reads
// (lgkmcnt(0)) BEFORE its first barrier: the half-tile restaged one phase later is only written after
// that barrier, which both rows have passed with their reads of it done (cdna_hip_programming.md
// section 5: "one barrier MORE when two wave groups run staggered").
constexpr int kHPre = 8;   // kEpiGeluGrad: H vectors per thread requested during the last K step

template <typename T, int kEpi>
__device__ __forceinline__ void epilogue16(const Args& g, char* lds, const f32x4 (&acc)[2][2][4][2], int m0, int n0,
                                           int tn, int wr, int wc, int fg, int fi, int tid, const uint4 (&hpre)[kHPre]);

template <typename T, bool kAFM, bool kBFM, bool kStagger, int kEpi = kEpiSlab>
__global__ __launch_bounds__(kThreads, 1) void wgrad4p_kernel(const Args g) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 4 * kHalf];   // [stage][A h0, A h1, B h0, B h1]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int tiles = g.tiles_m * g.tiles_n;
  const int nwg = tiles * g.splits;
  const int bid0 = blockIdx.x, xcd = bid0 & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid0 >> 3);
  const int split = lin / tiles, tile = lin % tiles;
  const int tm = tile % g.tiles_m, tn = tile / g.tiles_m;
  const int m0 = tm * kBM, n0 = tn * kBN;
  const int k_begin = (int)(((int64_t)split * g.nk) / g.splits), k_end = (int)(((int64_t)(split + 1) * g.nk) / g.splits);
  const int nk = k_end - k_begin;

  // glds sources: [half][instr]
  const char* srcA[2][2];
  const char* srcB[2][2];
  half_sources<kAFM, true>(g.A, g.lda, g.M, m0, 0, w, lane, srcA[0]);
  half_sources<kAFM, true>(g.A, g.lda, g.M, m0, 1, w, lane, srcA[1]);
  half_sources<kBFM, false>(g.B, g.ldb, g.N, n0, 0, w, lane, srcB[0]);
  half_sources<kBFM, false>(g.B, g.ldb, g.N, n0, 1, w, lane, srcB[1]);
  const int64_t stepA = kAFM ? (int64_t)kBK * 2 : (int64_t)kBK * g.lda * 2;
  const int64_t stepB = kBFM ? (int64_t)kBK * 2 : (int64_t)kBK * g.ldb * 2;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char*)(lds) + 2048u * w);
  // half-tile image index: 0 A h0, 1 A h1, 2 B h0, 3 B h1
  auto issue = [&](int step, int img) __attribute__((always_inline)) {
    const int ks = k_begin + step;
    const uint32_t dst = lds0 + (uint32_t)(((step & 1) * 4 + img) * kHalf);
    const char* const* s = img < 2 ? srcA[img] : srcB[img - 2];
    const int64_t st = img < 2 ? stepA : stepB;
    glds16(s[0] + st * ks, dst);
    glds16(s[1] + st * ks, dst + 1024);
  };

  // fragment read offsets within a half image
  const int fg = lane >> 4, fi = lane & 15, fq = fi >> 2, fp = fi & 3;
  int offA[4], offB[2];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int base = wr * 64 + mi * 16;                 // feature within the half
    if constexpr (!kAFM) {
      const int r = 8 * fg + fq;
      offA[mi] = r * 256 + (tm_slot(r, base / 8 + (fp >> 1)) << 4) + 8 * (fp & 1);
    } else {
      offA[mi] = (base + fi) * 128;
    }
  }
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    const int base = wc * 32 + ni * 16;
    if constexpr (!kBFM) {
      const int r = 8 * fg + fq;
      offB[ni] = r * 256 + (tm_slot(r, base / 8 + (fp >> 1)) << 4) + 8 * (fp & 1);
    } else {
      offB[ni] = (base + fi) * 128;
    }
  }
  auto frag = [&](const char* img, int off, int row, int kk, auto is_fm) __attribute__((always_inline)) -> s16x8 {
    if constexpr (!decltype(is_fm)::value) {
      const lds_char* p = (const lds_char*)(img) + off + kk * 32 * 256;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * 256));
      return cat8(lo, hi);
    } else {
      return *reinterpret_cast<const s16x8*>(img + off + (fm_slot(row, fg + 4 * kk) << 4));
    }
  };
  auto read_a = [&](const char* img, s16x8 (&af)[4][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        af[mi][kk] = frag(img, offA[mi], wr * 64 + mi * 16 + fi, kk, std::integral_constant<bool, kAFM>());
  };
  auto read_b = [&](const char* img, s16x8 (&bf)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        bf[ni][kk] = frag(img, offB[ni], wc * 32 + ni * 16 + fi, kk, std::integral_constant<bool, kBFM>());
  };

  f32x4 acc[2][2][4][2];   // [qm][qn][mi][ni]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma_q = [&](int qm, int qn, const s16x8 (&af)[4][2], const s16x8 (&bf)[2][2]) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) acc[qm][qn][mi][ni] = mfma<T>(af[mi][kk], bf[ni][kk], acc[qm][qn][mi][ni]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync_reads = [&]() __attribute__((always_inline)) {
    if constexpr (kStagger) {
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0) first: the reads are retired before the barrier
      __builtin_amdgcn_s_barrier();
    } else {
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this phase's fragment reads are in
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: step 0 whole, step 1's A h0 / B h1 / A h1 (phases 2-4 of step -1); step 0 ready
  if (nk > 0) {
#pragma unroll
    for (int img = 0; img < 4; ++img) issue(0, img);
  }
  if (nk > 1) {
    issue(1, 0);
    issue(1, 3);
    issue(1, 1);
    __builtin_amdgcn_s_waitcnt(0x0F76);   // vmcnt(6): step 0's eight loads done
  } else {
    __builtin_amdgcn_s_waitcnt(0x0F70);
  }
  __builtin_amdgcn_s_barrier();

  s16x8 af[4][2], bf0[2][2], bf1[2][2];
  if (kStagger && wr == 1) __builtin_amdgcn_s_barrier();   // wr is wave-uniform (readfirstlane'd w)
  // kEpiGeluGrad: the epilogue's first H vectors are requested at the start of the last K step, so their
  // latency hides behind its MFMAs (nothing else is in flight then: the step before retired with vmcnt(0))
  uint4 hpre[kHPre];
  for (int t = 0; t < nk; ++t) {
    const char* st = lds + (t & 1) * 4 * kHalf;
    if constexpr (kEpi == kEpiGeluGrad) {
      if (t == nk - 1) {
        const int c = tid & 31, sub = tid >> 5, f = m0 + c * 8;
#pragma unroll
        for (int p = 0; p < kHPre; ++p) {
          const int tt = min(n0 + p * 16 + sub, g.N - 1);
          hpre[p] = f < g.M ? ld16(reinterpret_cast<const T*>(g.H) + (int64_t)tt * g.ldh + f) : make_uint4(0, 0, 0, 0);
        }
      }
    }
    // ---- phase 1: B qn0 + A qm0 -> quadrant (0, 0); stage B h0 of step t + 1
    read_b(st + 2 * kHalf, bf0);
    read_a(st + 0 * kHalf, af);
    if (t + 1 < nk) issue(t + 1, 2);
    sync_reads();
    mma_q(0, 0, af, bf0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 2: B qn1 -> (0, 1); stage A h0 of step t + 2
    read_b(st + 3 * kHalf, bf1);
    if (t + 2 < nk) issue(t + 2, 0);
    sync_reads();
    mma_q(0, 1, af, bf1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 3: A qm1 -> (1, 1); stage B h1 of step t + 2
    read_a(st + 1 * kHalf, af);
    if (t + 2 < nk) issue(t + 2, 3);
    sync_reads();
    mma_q(1, 1, af, bf1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 4: B qn0 (re-read) -> (1, 0); stage A h1 of step t + 2; step t + 1 retired
    read_b(st + 2 * kHalf, bf0);
    if (t + 2 < nk) {
      issue(t + 2, 1);
      __builtin_amdgcn_s_waitcnt(0x0F76);   // vmcnt(6): all but step t + 2's three half-tiles
    } else {
      __builtin_amdgcn_s_waitcnt(0x0F70);   // tail: nothing of a later step in flight
    }
    sync_reads();
    mma_q(1, 0, af, bf0);
    __builtin_amdgcn_s_barrier();
  }
  if (kStagger && wr == 0) __builtin_amdgcn_s_barrier();   // equal barrier counts for both rows

  if constexpr (kEpi != kEpiSlab) {
    epilogue16<T, kEpi>(g, lds, acc, m0, n0, tn, wr, wc, fg, fi, tid, hpre);
    return;
  }
  // ---- epilogue: quadrant (qm, qn), tile (mi, ni): rows wr*128 + qm*64 + mi*16 + 4 (l >> 4) + r,
  // column wc*64 + qn*32 + ni*16 + (l & 15)
  float* C = g.C + (int64_t)split * g.slab_stride;
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const int col = n0 + wc * 64 + qn * 32 + ni * 16 + fi;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = m0 + wr * 128 + qm * 64 + mi * 16 + 4 * fg + r;
            if (row < g.M && col < g.N) C[(int64_t)row * g.ldc + col] = acc[qm][qn][mi][ni][r];
          }
        }
}

// 16-bit epilogue through LDS.  Every wave is past its last fragment read (the K loop's closing
// barrier), so the stage memory becomes the image of the transposed output tile: 256 token rows of
// 512 B (256 features), 16-B chunk c of row n at slot c ^ (n & 31).  A lane holds 4 consecutive
// features of one token per accumulator (rows 4 (l >> 4) + r of the MFMA tile): one 8-B LDS write
// each, the bias added before the rounding.  Then the workgroup walks the image row by row -- a
// wave moves two whole 512-B rows -- and writes Y (and Y2 / reads H) with full-line 16-B accesses;
// GELU / GELU' are evaluated there, on coalesced vectors.  The column sums (kEpiGeluGrad) meet in
// LDS in a fixed order: one fp32 partial per (token tile, feature), folded by the caller.
template <typename T, int kEpi>
__device__ __forceinline__ void epilogue16(const Args& g, char* lds, const f32x4 (&acc)[2][2][4][2], int m0, int n0,
                                           int tn, int wr, int wc, int fg, int fi, int tid, const uint4 (&hpre)[kHPre]) {
  const int c = tid & 31, sub = tid >> 5;   // read-back: chunk of 8 features, row within a group of 16
  const int f = m0 + c * 8;
  const bool fok = f < g.M;
  // kEpiGeluGrad: this thread's 16 vectors of H, requested before the staging pass so their latency
  // hides behind it (the accumulators' registers are still live; H takes 64 more)
  uint4 hq[16];
  if constexpr (kEpi == kEpiGeluGrad) {
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const int t = min(n0 + p * 16 + sub, g.N - 1);
      hq[p] = p < kHPre ? hpre[p]
                        : (fok ? ld16(reinterpret_cast<const T*>(g.H) + (int64_t)t * g.ldh + f) : make_uint4(0, 0, 0, 0));
    }
  }
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int m = wr * 128 + qm * 64 + mi * 16 + 4 * fg;   // 4 consecutive features
      f32x4 b = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (kEpi == kEpiBias || kEpi == kEpiBiasGelu) {
        if (m0 + m < g.M) {
          const uint2 bq = *reinterpret_cast<const uint2*>(reinterpret_cast<const T*>(g.bias) + m0 + m);
          const uint4 b4 = make_uint4(bq.x, bq.y, 0u, 0u);
          b = f32x4{elem_f<T>(b4, 0), elem_f<T>(b4, 1), elem_f<T>(b4, 2), elem_f<T>(b4, 3)};
        }
      }
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const int n = wc * 64 + qn * 32 + ni * 16 + fi;     // token
          const f32x4 v = acc[qm][qn][mi][ni] + b;
          const uint2 pk = make_uint2(cvt_pk2<T>(v[0], v[1]), cvt_pk2<T>(v[2], v[3]));
          *reinterpret_cast<uint2*>(lds + n * 512 + ((((m >> 3) ^ (n & 31))) << 4) + (m & 7) * 2) = pk;
        }
    }
  __syncthreads();
  float cs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = 0.f;
  if constexpr (kEpi == kEpiGeluGrad) {
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const int n = p * 16 + sub;
      const int t = n0 + n;
      const uint4 q = *reinterpret_cast<const uint4*>(lds + n * 512 + ((c ^ (n & 31)) << 4));
      if (!fok || t >= g.N) continue;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        f32x2 phi, pdf;
        const f32x2 x = f32x2{elem_f<T>(hq[p], e), elem_f<T>(hq[p], e + 1)};
        phi_pdf_f2(x, phi, pdf);
        const f32x2 gr = x * pdf + phi;   // gelu'(x), torch's cdf + x * pdf
        o[e] = elem_f<T>(q, e) * gr.x;
        o[e + 1] = elem_f<T>(q, e + 1) * gr.y;
      }
      const uint4 oq = pack_f<T>(o);
      st16(reinterpret_cast<T*>(g.Y) + (int64_t)t * g.ldy + f, oq);
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[e] += elem_f<T>(oq, e);
    }
  } else {
#pragma unroll 1
    for (int p0 = 0; p0 < 16; p0 += 4) {
      uint4 q[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = (p0 + j) * 16 + sub;
        q[j] = *reinterpret_cast<const uint4*>(lds + n * 512 + ((c ^ (n & 31)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int t = n0 + (p0 + j) * 16 + sub;
        if (!fok || t >= g.N) continue;
        st16(reinterpret_cast<T*>(g.Y) + (int64_t)t * g.ldy + f, q[j]);
        if constexpr (kEpi == kEpiBiasGelu) {
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = gelu_f(elem_f<T>(q[j], e));   // library erff, torch's F.gelu form
          st16(reinterpret_cast<T*>(g.Y2) + (int64_t)t * g.ldy2 + f, pack_f<T>(o));
        }
      }
    }
  }
  if constexpr (kEpi == kEpiGeluGrad) {
    if (g.colpart == nullptr) return;
    __syncthreads();                                   // the image is read: reuse it for the sums
    float* red = reinterpret_cast<float*>(lds);        // [16 rows of the group][256 features]
#pragma unroll
    for (int e = 0; e < 8; ++e) red[sub * 256 + c * 8 + e] = cs[e];
    __syncthreads();
    if (tid < 256 && m0 + tid < g.M) {
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) s += red[r * 256 + tid];
      g.colpart[(int64_t)tn * g.M + m0 + tid] = s;
    }
  }
}

// MC_WGRAD_PIPE: 5 = four-phase pipeline with staggered wave rows (default), 4 = four-phase, rows in
// step, 2 = wgrad_kernel (two barriers per K step)
static int wgrad_pipe() {   // read per call: A/B runs flip it inside one process
  const char* e = getenv("MC_WGRAD_PIPE");
  return e ? atoi(e) : 5;
}

template <typename T>
static void launch_t(const Args& a, bool afm, bool bfm, hipStream_t s) {
  const dim3 grid(a.tiles_m * a.tiles_n * a.splits), block(kThreads);
  if (wgrad_pipe() == 2) {
    if (!afm && !bfm) hipLaunchKernelGGL((wgrad_kernel<T, false, false>), grid, block, 0, s, a);
    else if (!afm && bfm) hipLaunchKernelGGL((wgrad_kernel<T, false, true>), grid, block, 0, s, a);
    else if (afm && !bfm) hipLaunchKernelGGL((wgrad_kernel<T, true, false>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((wgrad_kernel<T, true, true>), grid, block, 0, s, a);
    return;
  }
  if (wgrad_pipe() == 4) {
    if (!afm && !bfm) hipLaunchKernelGGL((wgrad4p_kernel<T, false, false, false>), grid, block, 0, s, a);
    else if (!afm && bfm) hipLaunchKernelGGL((wgrad4p_kernel<T, false, true, false>), grid, block, 0, s, a);
    else if (afm && !bfm) hipLaunchKernelGGL((wgrad4p_kernel<T, true, false, false>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((wgrad4p_kernel<T, true, true, false>), grid, block, 0, s, a);
    return;
  }
  if (!afm && !bfm) hipLaunchKernelGGL((wgrad4p_kernel<T, false, false, true>), grid, block, 0, s, a);
  else if (!afm && bfm) hipLaunchKernelGGL((wgrad4p_kernel<T, false, true, true>), grid, block, 0, s, a);
  else if (afm && !bfm) hipLaunchKernelGGL((wgrad4p_kernel<T, true, false, true>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((wgrad4p_kernel<T, true, true, true>), grid, block, 0, s, a);
}

static int auto_splits(int tiles, int nk) {
  // about one workgroup per CU (256), at least 4 K steps per split
  int s = (256 + tiles / 2) / tiles;
  s = std::max(1, std::min(s, nk / 4));
  return s;
}

}  // namespace wgrad
}  // namespace mc

using namespace mc;
using namespace mc::wgrad;

static int resolve(const mc_wgrad_params* p, int& splits, int& tiles_m, int& tiles_n, int& nk) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_gemm_wgrad: null params");
  MC_CHECK(p->M > 0 && p->N > 0 && p->T >= 0, MC_ERR_SHAPE, "mc_gemm_wgrad: bad shape M %d N %d T %d", p->M, p->N, p->T);
  MC_CHECK(p->dtype == MC_DTYPE_BF16 || p->dtype == MC_DTYPE_F16, MC_ERR_DTYPE, "mc_gemm_wgrad: operands must be bf16 or f16");
  MC_CHECK(p->T % kBK == 0, MC_ERR_SHAPE, "mc_gemm_wgrad: T %d must be a multiple of %d", p->T, kBK);
  MC_CHECK(p->a_layout == MC_WGRAD_TOKEN_MAJOR || p->a_layout == MC_WGRAD_FEATURE_MAJOR, MC_ERR_INVALID,
           "mc_gemm_wgrad: bad a_layout %d", p->a_layout);
  MC_CHECK(p->b_layout == MC_WGRAD_TOKEN_MAJOR || p->b_layout == MC_WGRAD_FEATURE_MAJOR, MC_ERR_INVALID,
           "mc_gemm_wgrad: bad b_layout %d", p->b_layout);
  auto ok = [&](const void* t, int64_t ld, int dim, int layout) {
    const int64_t rows = layout == MC_WGRAD_TOKEN_MAJOR ? p->T : dim;
    const int64_t cols = layout == MC_WGRAD_TOKEN_MAJOR ? dim : p->T;
    return t && aligned16(t) && ld % 8 == 0 && ld >= cols && (layout != MC_WGRAD_TOKEN_MAJOR || dim % 8 == 0) &&
           rows * ld < ((int64_t)1 << 40);
  };
  MC_CHECK(ok(p->A, p->lda, p->M, p->a_layout) && ok(p->B, p->ldb, p->N, p->b_layout), MC_ERR_SHAPE,
           "mc_gemm_wgrad: operands need 16-B aligned bases, leading dims %% 8 == 0 and >= the row length, and "
           "token-major feature counts %% 8 == 0 (M %d lda %lld, N %d ldb %lld)", p->M, (long long)p->lda, p->N,
           (long long)p->ldb);
  MC_CHECK(p->C && p->ldc == p->N, MC_ERR_SHAPE, "mc_gemm_wgrad: C must be a contiguous M x N fp32 matrix");
  tiles_m = (p->M + kBM - 1) / kBM;
  tiles_n = (p->N + kBN - 1) / kBN;
  nk = p->T / kBK;
  splits = p->splits > 0 ? std::min(p->splits, std::max(nk, 1)) : auto_splits(tiles_m * tiles_n, nk);
  return MC_OK;
}

extern "C" size_t mc_gemm_wgrad_workspace_bytes(const mc_wgrad_params* p) {
  int splits, tm, tn, nk;
  if (resolve(p, splits, tm, tn, nk) != MC_OK) return 0;
  return splits > 1 ? (size_t)splits * p->M * p->N * 4 : 0;
}

extern "C" int mc_gemm_wgrad(const mc_wgrad_params* p, void* stream) {
  int splits, tiles_m, tiles_n, nk;
  int rc = resolve(p, splits, tiles_m, tiles_n, nk);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (nk == 0) {
    (void)hipMemsetAsync(p->C, 0, (size_t)p->M * p->N * 4, s);
    return MC_OK;
  }
  const size_t ws_need = splits > 1 ? (size_t)splits * p->M * p->N * 4 : 0;
  MC_CHECK(ws_need == 0 || (p->workspace && p->workspace_bytes >= ws_need && aligned16(p->workspace)), MC_ERR_WORKSPACE,
           "mc_gemm_wgrad: workspace must be >= %zu bytes, 16-B aligned (got %zu)", ws_need, p->workspace_bytes);
  Args a;
  a.M = p->M; a.N = p->N; a.T = p->T; a.splits = splits; a.tiles_m = tiles_m; a.tiles_n = tiles_n; a.nk = nk;
  a.A = reinterpret_cast<const char*>(p->A); a.B = reinterpret_cast<const char*>(p->B);
  a.lda = p->lda; a.ldb = p->ldb;
  a.C = splits > 1 ? reinterpret_cast<float*>(p->workspace) : p->C;
  a.ldc = p->N;
  a.slab_stride = (int64_t)p->M * p->N;
  const bool afm = p->a_layout == MC_WGRAD_FEATURE_MAJOR, bfm = p->b_layout == MC_WGRAD_FEATURE_MAJOR;
  if (p->dtype == MC_DTYPE_BF16) launch_t<bf16_t>(a, afm, bfm, s);
  else launch_t<f16_t>(a, afm, bfm, s);
  hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_gemm_wgrad: launch failed: %s", hipGetErrorString(e));
  if (splits > 1) return mc_sum_slabs(splits, (int64_t)p->M * p->N, a.C, a.slab_stride, p->C, stream);
  return MC_OK;
}

// ------------------------------------------------------------------ mc_linear
// Y = X W^T on wgrad4p_kernel with both operands feature-major in its terms (A = W: row m = output
// feature, B = X: row n = token, unit stride along K) and a 16-bit epilogue; one workgroup per
// 256 x 256 output tile (K <= a few thousand: no split).
template <typename T, bool kStag>
static void launch_linear_s(const Args& a, int epi, hipStream_t s) {
  const dim3 grid(a.tiles_m * a.tiles_n), block(kThreads);
  switch (epi) {
    case MC_LINEAR_EPI_NONE: hipLaunchKernelGGL((wgrad4p_kernel<T, true, true, kStag, kEpiStore>), grid, block, 0, s, a); break;
    case MC_LINEAR_EPI_BIAS: hipLaunchKernelGGL((wgrad4p_kernel<T, true, true, kStag, kEpiBias>), grid, block, 0, s, a); break;
    case MC_LINEAR_EPI_BIAS_GELU:
      hipLaunchKernelGGL((wgrad4p_kernel<T, true, true, kStag, kEpiBiasGelu>), grid, block, 0, s, a);
      break;
    default: hipLaunchKernelGGL((wgrad4p_kernel<T, true, true, kStag, kEpiGeluGrad>), grid, block, 0, s, a); break;
  }
}
// MC_LINEAR_STAGGER=0: wave rows in step (A/B of the staggered schedule at these short K loops)
template <typename T>
static void launch_linear(const Args& a, int epi, hipStream_t s) {
  const char* e = getenv("MC_LINEAR_STAGGER");
  if (e && atoi(e) == 0) launch_linear_s<T, false>(a, epi, s);
  else launch_linear_s<T, true>(a, epi, s);
}

static int linear_check(const mc_linear_params* p) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_linear: null params");
  MC_CHECK(p->rows >= 0 && p->cols > 0 && p->K > 0 && p->cols % 8 == 0 && p->K % kBK == 0, MC_ERR_SHAPE,
           "mc_linear: bad shape rows %d cols %d (%% 8) K %d (%% %d)", p->rows, p->cols, p->K, kBK);
  MC_CHECK(p->dtype == MC_DTYPE_BF16 || p->dtype == MC_DTYPE_F16, MC_ERR_DTYPE, "mc_linear: operands must be bf16 or f16");
  MC_CHECK(p->epilogue >= MC_LINEAR_EPI_NONE && p->epilogue <= MC_LINEAR_EPI_GELU_GRAD, MC_ERR_INVALID,
           "mc_linear: bad epilogue %d", p->epilogue);
  auto ok = [](const void* t, int64_t ld, int64_t width) { return t && aligned16(t) && ld % 8 == 0 && ld >= width; };
  MC_CHECK(ok(p->X, p->ldx, p->K) && ok(p->W, p->ldw, p->K) && ok(p->Y, p->ldy, p->cols), MC_ERR_SHAPE,
           "mc_linear: X, W, Y need 16-B aligned bases and leading dims %% 8 == 0 covering the row");
  MC_CHECK((int64_t)p->rows * std::max(p->ldx, p->ldy) < ((int64_t)1 << 40), MC_ERR_SHAPE, "mc_linear: operand too large");
  if (p->epilogue == MC_LINEAR_EPI_BIAS || p->epilogue == MC_LINEAR_EPI_BIAS_GELU)
    MC_CHECK(p->bias && (reinterpret_cast<uintptr_t>(p->bias) & 7) == 0, MC_ERR_INVALID,
             "mc_linear: the bias epilogues need an 8-B aligned bias (operand dtype)");
  if (p->epilogue == MC_LINEAR_EPI_BIAS_GELU)
    MC_CHECK(ok(p->Y2, p->ldy2, p->cols), MC_ERR_SHAPE, "mc_linear: BIAS_GELU needs Y2 (16-B aligned, ld %% 8 == 0)");
  if (p->epilogue == MC_LINEAR_EPI_GELU_GRAD)
    MC_CHECK(ok(p->H, p->ldh, p->cols), MC_ERR_SHAPE, "mc_linear: GELU_GRAD needs H (16-B aligned, ld %% 8 == 0)");
  return MC_OK;
}

extern "C" size_t mc_linear_workspace_bytes(const mc_linear_params* p) {
  if (linear_check(p) != MC_OK) return 0;
  if (p->epilogue != MC_LINEAR_EPI_GELU_GRAD || p->colsum == nullptr) return 0;
  return (size_t)((p->rows + kBN - 1) / kBN) * p->cols * 4;
}

extern "C" int mc_linear(const mc_linear_params* p, void* stream) {
  int rc = linear_check(p);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const bool sums = p->epilogue == MC_LINEAR_EPI_GELU_GRAD && p->colsum != nullptr;
  const int tiles_n = (p->rows + kBN - 1) / kBN;
  if (sums) {
    const size_t need = (size_t)tiles_n * p->cols * 4;
    MC_CHECK(need == 0 || (p->workspace && p->workspace_bytes >= need && aligned16(p->workspace)), MC_ERR_WORKSPACE,
             "mc_linear: workspace must be >= %zu bytes, 16-B aligned (got %zu)", need, p->workspace_bytes);
  }
  if (p->rows == 0) {
    if (sums) (void)hipMemsetAsync(p->colsum, 0, (size_t)p->cols * 4, s);
    return MC_OK;
  }
  Args a{};
  a.M = p->cols; a.N = p->rows; a.T = p->K; a.splits = 1;
  a.tiles_m = (p->cols + kBM - 1) / kBM; a.tiles_n = tiles_n; a.nk = p->K / kBK;
  a.A = reinterpret_cast<const char*>(p->W); a.lda = p->ldw;
  a.B = reinterpret_cast<const char*>(p->X); a.ldb = p->ldx;
  a.Y = p->Y; a.ldy = p->ldy; a.Y2 = p->Y2; a.ldy2 = p->ldy2; a.bias = p->bias;
  a.H = p->H; a.ldh = p->ldh; a.colpart = sums ? reinterpret_cast<float*>(p->workspace) : nullptr;
  if (p->dtype == MC_DTYPE_BF16) launch_linear<bf16_t>(a, p->epilogue, s);
  else launch_linear<f16_t>(a, p->epilogue, s);
  hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_linear: launch failed: %s", hipGetErrorString(e));
  // the per-tile partial rows: many (197 at C2) short rows -> the slice fold, 8 slices in flight per column
  if (sums) return mc_colsum_fold(tiles_n, p->cols, a.colpart, p->colsum, stream);
  return MC_OK;
}

// ------------------------------------------------------------------ mc_gemm_small_k
// Y (M x T) = W (M x K) X (K x T) for a short reduction (K <= 64, K % 16 == 0) and a long, unit-stride
// token dimension: the Mamba mixer's dt_proj forward, delta = W_dt dt_raw (reference model.py:519-528:
// the einsum with dt_projs_weight; Mamba's dt_proj Linear) -- the library runs it at ~1/3 of the
// output-write rate.  One workgroup = 256 tokens x 64 rows of Y; X's K x 256 tile is staged in LDS
// (rows padded to 544 B: the transposed reads of 8 rows hit distinct banks) and read back as MFMA A
// operands with ds_read_b64_tr_b16 (the k-strided direction); W's rows are the B operands straight
// from global memory (8-B pieces, L2-resident); the Y^T tiles (4 consecutive tokens per lane) are
// staged back through the LDS and leave as whole 512-B row pieces.  v_mfma_f32_16x16x16_{bf16,f16}, fp32 accumulation, one rounding.
namespace mc {
namespace skinny {
constexpr int kTT = 256, kTM = 64, kRow = 544;   // tokens / rows per workgroup, LDS row bytes
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

template <typename T>
__device__ __forceinline__ f32x4 mfma16(s16x4_t a, s16x4_t b, f32x4 c) {
  if constexpr (std::is_same<T, bf16_t>::value) return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
  else {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(h4, a), __builtin_bit_cast(h4, b), c, 0, 0, 0);
  }
}

template <typename T, int K>
__global__ __launch_bounds__(256) void small_k_kernel(int M, int Tn, const T* __restrict__ W, int64_t ldw,
                                                      const T* __restrict__ X, int64_t ldx, T* __restrict__ Y,
                                                      int64_t ldy) {
  constexpr int kORow = 528;   // output image row: 256 tokens + 16 B pad (the 16 rows of a store hit distinct banks)
  constexpr int kLds = K * kRow > kTM * kORow ? K * kRow : kTM * kORow;
  __shared__ __attribute__((aligned(16))) char xs[kLds];   // X tile, then the output tile
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tiles_t = (Tn + kTT - 1) / kTT;
  const int t0 = (blockIdx.x % tiles_t) * kTT, m0 = (blockIdx.x / tiles_t) * kTM;
  // X tile -> LDS: K rows x 256 tokens, 16-B vectors (tokens past Tn read as 0)
  constexpr int kVecs = K * kTT / 8;
#pragma unroll
  for (int j = 0; j < (kVecs + 255) / 256; ++j) {
    const int q = tid + 256 * j;
    if (q < kVecs) {
      const int r = q / (kTT / 8), c = (q % (kTT / 8)) * 8;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (t0 + c < Tn) v = ld16(X + (int64_t)r * ldx + t0 + c);   // Tn % 8 == 0: whole vectors
      *reinterpret_cast<uint4*>(xs + r * kRow + c * 2) = v;
    }
  }
  // B operands: W[m0 + 16 cb + i][16 kk + 4 g .. + 3] (rows past M clamped; their columns are not stored)
  const int g = lane >> 4, i = lane & 15;
  s16x4_t bfr[4][K / 16];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int m = min(m0 + 16 * cb + i, M - 1);
#pragma unroll
    for (int kk = 0; kk < K / 16; ++kk)
      bfr[cb][kk] = *reinterpret_cast<const s16x4_t*>(W + (int64_t)m * ldw + 16 * kk + 4 * g);
  }
  __syncthreads();
  // A operands by transposed reads: lane 4q + p of group g addresses row 16 kk + 4 g + q, tokens tb + 4 p
  const int q = i >> 2, p = i & 3;
  f32x4 acc[4][4];
#pragma unroll
  for (int tb = 0; tb < 4; ++tb)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[tb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < K / 16; ++kk)
#pragma unroll
    for (int tb = 0; tb < 4; ++tb) {
      const int tl = w * 64 + tb * 16 + 4 * p;
      const s16x4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4_t*)((__attribute__((address_space(3))) char*)(xs) + (16 * kk + 4 * g + q) * kRow + tl * 2));
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) acc[tb][cb] = mfma16<T>(a, bfr[cb][kk], acc[tb][cb]);
    }
  // C (16 tokens x 16 rows): lane holds tokens 4 g .. 4 g + 3 of row i -> the LDS output image
  // [64 rows][256 tokens], then whole 512-B row pieces of Y (16-B stores, a wave per two rows)
  __syncthreads();   // every wave's transposed reads of the X tile are done
#pragma unroll
  for (int tb = 0; tb < 4; ++tb)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const f32x4 v = acc[tb][cb];
      *reinterpret_cast<uint2*>(xs + (16 * cb + i) * kORow + (w * 64 + tb * 16 + 4 * g) * 2) =
          make_uint2(cvt_pk2<T>(v[0], v[1]), cvt_pk2<T>(v[2], v[3]));
    }
  __syncthreads();
  const int cv = tid & 31, rr = tid >> 5;
#pragma unroll
  for (int j = 0; j < kTM / 8; ++j) {
    const int r = 8 * j + rr, m = m0 + r, t = t0 + cv * 8;
    if (m < M && t < Tn) st16(Y + (int64_t)m * ldy + t, *reinterpret_cast<const uint4*>(xs + r * kORow + cv * 16));
  }
}
}  // namespace skinny
}  // namespace mc

extern "C" int mc_gemm_small_k(int32_t M, int32_t K, int32_t T, int32_t dtype, const void* W, int64_t ldw, const void* X,
                               int64_t ldx, void* Y, int64_t ldy, void* stream) {
  MC_CHECK(dtype == MC_DTYPE_BF16 || dtype == MC_DTYPE_F16, MC_ERR_DTYPE, "mc_gemm_small_k: bf16 / f16 only");
  MC_CHECK(M > 0 && T >= 0 && (K == 16 || K == 32 || K == 48 || K == 64) && T % 8 == 0, MC_ERR_SHAPE,
           "mc_gemm_small_k: M %d > 0, K %d in {16, 32, 48, 64}, T %d %% 8 == 0", M, K, T);
  MC_CHECK(W && X && Y && aligned16(X) && aligned16(Y) && (reinterpret_cast<uintptr_t>(W) & 7) == 0 && ldw % 4 == 0 &&
               ldw >= K && ldx % 8 == 0 && ldx >= T && ldy % 8 == 0 && ldy >= T,
           MC_ERR_SHAPE, "mc_gemm_small_k: 16-B aligned X / Y rows (ld %% 8), 8-B aligned W rows");
  if (T == 0) return MC_OK;
  const dim3 grid(((T + skinny::kTT - 1) / skinny::kTT) * ((M + skinny::kTM - 1) / skinny::kTM)), block(256);
  hipStream_t s = (hipStream_t)stream;
#define MC_SMALLK(TT, KK) hipLaunchKernelGGL((skinny::small_k_kernel<TT, KK>), grid, block, 0, s, M, T, (const TT*)W, ldw, \
                                             (const TT*)X, ldx, (TT*)Y, ldy)
  if (dtype == MC_DTYPE_BF16) {
    if (K == 16) MC_SMALLK(bf16_t, 16); else if (K == 32) MC_SMALLK(bf16_t, 32); else if (K == 48) MC_SMALLK(bf16_t, 48); else MC_SMALLK(bf16_t, 64);
  } else {
    if (K == 16) MC_SMALLK(f16_t, 16); else if (K == 32) MC_SMALLK(f16_t, 32); else if (K == 48) MC_SMALLK(f16_t, 48); else MC_SMALLK(f16_t, 64);
  }
#undef MC_SMALLK
  hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_gemm_small_k: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

// ------------------------------------------------------------------ mc_gemm_skinny_m
// Y (M x T) = W (M x K) X (K x T) for a few output rows (M <= 96) and a long reduction over X's rows
// (K % 256 == 0): the Mamba mixer's x_proj forward, x_dbl = W_x x (80 x 1536 @ 1536 x B*L; reference:
// Mamba's x_proj Linear, the SS2D form at model.py:519-528).  It is an HBM stream of X; the library
// runs it at ~1/3 of that rate.  One workgroup = 64 tokens; its 4 waves split K four ways (each walks
// its quarter in 64-row chunks: the next chunk's X rows and W fragments load into registers while the
// current chunk's MFMAs run from the wave's own LDS image), then the four partial tiles are summed in a
// fixed order ((w0 + w2) + (w1 + w3)) through the LDS and wave 0 writes Y in 128-B row pieces.
namespace mc {
namespace skinny {
constexpr int kST = 64, kSC = 64, kSXRow = 160, kSORow = 144;   // tokens, K rows per chunk, LDS row bytes

template <typename T, int MB>
__global__ __launch_bounds__(256) void skinny_m_kernel(int M, int K, int Tn, const T* __restrict__ W, int64_t ldw,
                                                       const T* __restrict__ X, int64_t ldx, T* __restrict__ Y,
                                                       int64_t ldy) {
  constexpr int kAcc = MB * 4;                          // f32x4 accumulators per lane
  constexpr int kRed = 2 * kAcc * 4 * 64 * 4;           // two waves' partial tiles (bytes)
  constexpr int kImg = 4 * kSC * kSXRow;                // the four waves' X images
  constexpr int kOut = MB * 16 * kSORow;
  constexpr int kLds = (kImg > kRed ? kImg : kRed) > kOut ? (kImg > kRed ? kImg : kRed) : kOut;
  __shared__ __attribute__((aligned(16))) char lds[kLds];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int t0 = blockIdx.x * kST;
  const int kq = K / 4, nchunk = kq / kSC, kw0 = w * kq;
  char* img = lds + w * kSC * kSXRow;
  // X chunk rows -> registers: vector v = lane + 64 j is row v / 8, tokens 8 (v % 8) .. + 7 (0 past Tn)
  uint4 xr[8];
  s16x4_t wn[MB][4];
  auto load = [&](int c) __attribute__((always_inline)) {
    const int k0 = kw0 + c * kSC;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int v = lane + 64 * j, r = v >> 3, col = (v & 7) * 8;
      xr[j] = t0 + col < Tn ? ld16(X + (int64_t)(k0 + r) * ldx + t0 + col) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int cb = 0; cb < MB; ++cb) {
      const int m = min(16 * cb + i, M - 1);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) wn[cb][kk] = *reinterpret_cast<const s16x4_t*>(W + (int64_t)m * ldw + k0 + 16 * kk + 4 * g);
    }
  };
  f32x4 acc[MB][4];
#pragma unroll
  for (int cb = 0; cb < MB; ++cb)
#pragma unroll
    for (int tb = 0; tb < 4; ++tb) acc[cb][tb] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int c = 0; c < nchunk; ++c) {
    // this wave's image only: a wave's LDS accesses complete in issue order, so no barrier
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int v = lane + 64 * j;
      *reinterpret_cast<uint4*>(img + (v >> 3) * kSXRow + (v & 7) * 16) = xr[j];
    }
    s16x4_t wc[MB][4];
#pragma unroll
    for (int cb = 0; cb < MB; ++cb)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) wc[cb][kk] = wn[cb][kk];
    if (c + 1 < nchunk) load(c + 1);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int tb = 0; tb < 4; ++tb) {
        // B operand (k x t) by a transposed read: lane 4q + p addresses row 16 kk + 4 g + q, tokens 16 tb + 4 p
        const s16x4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4_t*)((__attribute__((address_space(3))) char*)(img) + (16 * kk + 4 * g + q) * kSXRow + (16 * tb + 4 * p) * 2));
#pragma unroll
        for (int cb = 0; cb < MB; ++cb) acc[cb][tb] = mfma16<T>(wc[cb][kk], b, acc[cb][tb]);
      }
  }
  // fixed-order sum of the four waves' partial tiles: (w0 + w2) + (w1 + w3)
  float* red = reinterpret_cast<float*>(lds);
  __syncthreads();
  if (w >= 2) {
#pragma unroll
    for (int cb = 0; cb < MB; ++cb)
#pragma unroll
      for (int tb = 0; tb < 4; ++tb)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[(((w - 2) * kAcc + cb * 4 + tb) * 4 + j) * 64 + lane] = acc[cb][tb][j];
  }
  __syncthreads();
  if (w < 2) {
#pragma unroll
    for (int cb = 0; cb < MB; ++cb)
#pragma unroll
      for (int tb = 0; tb < 4; ++tb)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[cb][tb][j] += red[((w * kAcc + cb * 4 + tb) * 4 + j) * 64 + lane];
  }
  __syncthreads();
  if (w == 1) {
#pragma unroll
    for (int cb = 0; cb < MB; ++cb)
#pragma unroll
      for (int tb = 0; tb < 4; ++tb)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[((cb * 4 + tb) * 4 + j) * 64 + lane] = acc[cb][tb][j];
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int cb = 0; cb < MB; ++cb)
#pragma unroll
      for (int tb = 0; tb < 4; ++tb)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[cb][tb][j] += red[((cb * 4 + tb) * 4 + j) * 64 + lane];
  }
  __syncthreads();
  if (w == 0) {
    // C: lane holds rows 16 cb + 4 g + j of token 16 tb + i -> output image [rows][64 tokens] -> Y rows
    T* out = reinterpret_cast<T*>(lds);
#pragma unroll
    for (int cb = 0; cb < MB; ++cb)
#pragma unroll
      for (int tb = 0; tb < 4; ++tb)
#pragma unroll
        for (int j = 0; j < 4; ++j) out[(16 * cb + 4 * g + j) * (kSORow / 2) + 16 * tb + i] = from_f<T>(acc[cb][tb][j]);
#pragma unroll
    for (int j = 0; j < (MB * 16 * 8 + 63) / 64; ++j) {
      const int v = lane + 64 * j, r = v >> 3, col = (v & 7) * 8;
      if (r < MB * 16 && r < M && t0 + col < Tn)
        st16(Y + (int64_t)r * ldy + t0 + col, *reinterpret_cast<const uint4*>(lds + r * kSORow + col * 2));
    }
  }
}
}  // namespace skinny
}  // namespace mc

extern "C" int mc_gemm_skinny_m(int32_t M, int32_t K, int32_t T, int32_t dtype, const void* W, int64_t ldw, const void* X,
                                int64_t ldx, void* Y, int64_t ldy, void* stream) {
  MC_CHECK(dtype == MC_DTYPE_BF16 || dtype == MC_DTYPE_F16, MC_ERR_DTYPE, "mc_gemm_skinny_m: bf16 / f16 only");
  MC_CHECK(M > 0 && M <= 96 && K > 0 && K % 256 == 0 && T >= 0 && T % 8 == 0, MC_ERR_SHAPE,
           "mc_gemm_skinny_m: 0 < M %d <= 96, K %d %% 256 == 0, T %d %% 8 == 0", M, K, T);
  MC_CHECK(W && X && Y && aligned16(X) && aligned16(Y) && (reinterpret_cast<uintptr_t>(W) & 7) == 0 && ldw % 4 == 0 &&
               ldw >= K && ldx % 8 == 0 && ldx >= T && ldy % 8 == 0 && ldy >= T,
           MC_ERR_SHAPE, "mc_gemm_skinny_m: 16-B aligned X / Y rows (ld %% 8), 8-B aligned W rows");
  MC_CHECK((int64_t)K * ldx < ((int64_t)1 << 40), MC_ERR_SHAPE, "mc_gemm_skinny_m: X too large");
  if (T == 0) return MC_OK;
  const dim3 grid((T + skinny::kST - 1) / skinny::kST), block(256);
  hipStream_t s = (hipStream_t)stream;
  const int mb = (M + 15) / 16;
#define MC_SKM(TT, MBV) hipLaunchKernelGGL((skinny::skinny_m_kernel<TT, MBV>), grid, block, 0, s, M, K, T, (const TT*)W, ldw, \
                                           (const TT*)X, ldx, (TT*)Y, ldy)
#define MC_SKM_T(TT) \
  switch (mb) { case 1: MC_SKM(TT, 1); break; case 2: MC_SKM(TT, 2); break; case 3: MC_SKM(TT, 3); break; \
                case 4: MC_SKM(TT, 4); break; case 5: MC_SKM(TT, 5); break; default: MC_SKM(TT, 6); break; }
  if (dtype == MC_DTYPE_BF16) { MC_SKM_T(bf16_t) } else { MC_SKM_T(f16_t) }
#undef MC_SKM_T
#undef MC_SKM
  hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_gemm_skinny_m: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}
