// scan_common.h -- pieces shared by the selective-scan forward and backward.
#pragma once

#include "mc_common.h"
#include "../../include/mc_scan.h"

namespace mc {
namespace scan {

constexpr int kT = 32;             // sequence positions per forward tile
constexpr int kS = MC_SCAN_CHUNK;  // positions per saved chunk state (32)
constexpr int kFineS = MC_SCAN_STATE_INTERVAL_FINE;   // the fine saved-state interval (8)
constexpr int kRows = 64;          // channels per workgroup: one wave

// B/C as the recurrence consumes them: fp32, position-major, [b][g][l][2*kNp]
// (B states 0..kNp-1 then C states; states >= dstate are zero).  Every lane of
// a wave reads the same position, so one chunk of it is a contiguous block
// that is staged in LDS once per wave and broadcast-read.

inline int padded_dstate(int dstate) { return dstate <= 8 ? 8 : (dstate <= 16 ? 16 : 32); }

inline size_t bct_bytes(int batch, int seqlen, int dstate, int n_groups) {
  return (size_t)batch * n_groups * seqlen * 2 * padded_dstate(dstate) * sizeof(float);
}

// LDS hand-off between the lanes of a ONE-WAVE workgroup.  A wave's LDS
// instructions are performed in program order, so a compiler barrier is all
// the ordering a cross-lane exchange needs.  __syncthreads() would also lower
// to a vmcnt(0)/lgkmcnt(0) drain: every chunk would wait for the previous
// chunk's global stores and for prefetch loads still in flight (measured in
// the backward: ~2/3 of the wave's cycles sat in those drains).
static_assert(kRows == 64, "wave_lds_sync() is only valid for one-wave workgroups");
__device__ __forceinline__ void wave_lds_sync() { asm volatile("" ::: "memory"); }

// Workgroup barrier for LDS hand-offs only: this wave's LDS operations are
// complete, global loads / stores stay in flight (gfx950 has the back-off
// barrier, so s_barrier itself forces no vmcnt drain; __syncthreads()'s fence
// would wait for every prefetch still in flight).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Lane id the compiler cannot hoist or CSE (asm volatile): values derived from
// it are rebuilt where used instead of occupying VGPRs across a hot loop.
__device__ __forceinline__ int opaque_lane_id() {
  int v;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
  return v;
}

// Bijective blockIdx remap so that consecutive logical blocks (same batch /
// group, sharing B/C) run on one XCD: hardware deals blocks round-robin over
// the 8 XCDs (speed only -- correctness never depends on placement).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int xcd = bid & 7, q = nblocks >> 3, r = nblocks & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Re-lay B/C (any strides along b/g/n, unit stride along l) into the fp32
// position-major buffer.  One thread per (b, g, l, j<2kNp).
template <typename TW, int kNp>
__global__ __launch_bounds__(256) void bc_relayout_kernel(const TW* __restrict__ B, const TW* __restrict__ C,
                                                         int64_t B_bs, int64_t B_gs, int64_t B_ns, int64_t C_bs,
                                                         int64_t C_gs, int64_t C_ns, int batch, int G, int L,
                                                         int dstate, int rev, float* __restrict__ out) {
  const int64_t total = (int64_t)batch * G * L * 2 * kNp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(i % (2 * kNp));
    const int64_t rest = i / (2 * kNp);
    const int l = (int)(rest % L);
    const int64_t bg = rest / L;
    const int g = (int)(bg % G), b = (int)(bg / G);
    const bool isC = j >= kNp;
    const int n = isC ? j - kNp : j;
    float v = 0.f;
    if (n < dstate) {
      const TW* src = isC ? C + (int64_t)b * C_bs + (int64_t)g * C_gs + (int64_t)n * C_ns
                          : B + (int64_t)b * B_bs + (int64_t)g * B_gs + (int64_t)n * B_ns;
      v = to_f(src[((rev >> g) & 1) ? L - 1 - l : l]);   // reversed groups: mirrored positions
    }
    out[i] = v;
  }
}

// Vector form for 16-bit B/C with 16-B aligned rows, L % 8 == 0 and no reversed groups (every
// long-sequence call): one thread per (b, g, 8-position block, B|C half) reads kNp 16-B row
// vectors and writes its half of 8 position rows as float4s (the element-wise kernel above
// moves 2-B loads and 4-B stores: 31 us at C4).
template <typename TW, int kNp>
__global__ __launch_bounds__(256) void bc_relayout_vec_kernel(const TW* __restrict__ B, const TW* __restrict__ C,
                                                             int64_t B_bs, int64_t B_gs, int64_t B_ns, int64_t C_bs,
                                                             int64_t C_gs, int64_t C_ns, int batch, int G, int L,
                                                             int dstate, float* __restrict__ out) {
  const int nblk = L / 8;
  const int64_t total = (int64_t)batch * G * nblk * 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int half = (int)(i & 1);
    const int64_t rest = i >> 1;
    const int lb = (int)(rest % nblk);
    const int64_t bg = rest / nblk;
    const int g = (int)(bg % G), b = (int)(bg / G);
    const TW* src = half ? C + (int64_t)b * C_bs + (int64_t)g * C_gs : B + (int64_t)b * B_bs + (int64_t)g * B_gs;
    const int64_t ns = half ? C_ns : B_ns;
    uint4 q[kNp];
#pragma unroll
    for (int n = 0; n < kNp; ++n)
      q[n] = n < dstate ? ld16(src + (int64_t)n * ns + 8 * lb) : make_uint4(0u, 0u, 0u, 0u);
    float* dst = out + ((bg * L + 8 * lb) * 2 + half) * kNp;
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int n4 = 0; n4 < kNp / 4; ++n4)
        reinterpret_cast<float4*>(dst + e * 2 * kNp)[n4] =
            make_float4(elem_f<TW>(q[4 * n4], e), elem_f<TW>(q[4 * n4 + 1], e), elem_f<TW>(q[4 * n4 + 2], e),
                        elem_f<TW>(q[4 * n4 + 3], e));
  }
}

template <typename TW>
inline hipError_t launch_bc_relayout(const void* B, const void* C, int64_t B_bs, int64_t B_gs, int64_t B_ns,
                                     int64_t C_bs, int64_t C_gs, int64_t C_ns, int batch, int G, int L, int dstate,
                                     int rev, float* out, hipStream_t s) {
  const int np = padded_dstate(dstate);
  const TW* b = reinterpret_cast<const TW*>(B);
  const TW* c = reinterpret_cast<const TW*>(C);
  if constexpr (sizeof(TW) == 2) {
    auto al = [](const void* p, int64_t s0, int64_t s1, int64_t s2) {
      return aligned16(p) && s0 % 8 == 0 && s1 % 8 == 0 && s2 % 8 == 0;
    };
    if (rev == 0 && L % 8 == 0 && al(B, B_bs, B_gs, B_ns) && al(C, C_bs, C_gs, C_ns) && np >= 8) {
      const int64_t tv = (int64_t)batch * G * (L / 8) * 2;
      const int gv = (int)std::min<int64_t>((tv + 255) / 256, 16384);
      if (np == 8)
        hipLaunchKernelGGL((bc_relayout_vec_kernel<TW, 8>), gv, 256, 0, s, b, c, B_bs, B_gs, B_ns, C_bs, C_gs, C_ns,
                           batch, G, L, dstate, out);
      else if (np == 16)
        hipLaunchKernelGGL((bc_relayout_vec_kernel<TW, 16>), gv, 256, 0, s, b, c, B_bs, B_gs, B_ns, C_bs, C_gs, C_ns,
                           batch, G, L, dstate, out);
      else
        hipLaunchKernelGGL((bc_relayout_vec_kernel<TW, 32>), gv, 256, 0, s, b, c, B_bs, B_gs, B_ns, C_bs, C_gs, C_ns,
                           batch, G, L, dstate, out);
      return hipGetLastError();
    }
  }
  const int64_t total = (int64_t)batch * G * L * 2 * np;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
  if (np == 8)
    hipLaunchKernelGGL((bc_relayout_kernel<TW, 8>), grid, 256, 0, s, b, c, B_bs, B_gs, B_ns, C_bs, C_gs, C_ns, batch,
                       G, L, dstate, rev, out);
  else if (np == 16)
    hipLaunchKernelGGL((bc_relayout_kernel<TW, 16>), grid, 256, 0, s, b, c, B_bs, B_gs, B_ns, C_bs, C_gs, C_ns,
                       batch, G, L, dstate, rev, out);
  else
    hipLaunchKernelGGL((bc_relayout_kernel<TW, 32>), grid, 256, 0, s, b, c, B_bs, B_gs, B_ns, C_bs, C_gs, C_ns,
                       batch, G, L, dstate, rev, out);
  return hipGetLastError();
}

inline hipError_t relayout_bc(int wtype, const void* B, const void* C, int64_t B_bs, int64_t B_gs, int64_t B_ns,
                              int64_t C_bs, int64_t C_gs, int64_t C_ns, int batch, int G, int L, int dstate,
                              int rev, float* out, hipStream_t s) {
  if (wtype == MC_DTYPE_F32)
    return launch_bc_relayout<float>(B, C, B_bs, B_gs, B_ns, C_bs, C_gs, C_ns, batch, G, L, dstate, rev, out, s);
  if (wtype == MC_DTYPE_BF16)
    return launch_bc_relayout<bf16_t>(B, C, B_bs, B_gs, B_ns, C_bs, C_gs, C_ns, batch, G, L, dstate, rev, out, s);
  return launch_bc_relayout<f16_t>(B, C, B_bs, B_gs, B_ns, C_bs, C_gs, C_ns, batch, G, L, dstate, rev, out, s);
}

// LDS row of one channel for one chunk: kT / VI blocks; block k = {u vector k
// (16 B = VI steps), delta vector k (16 B)}.  After consuming block k the
// thread writes y for those VI steps (fp32, 4*VI <= 32 B) over the block, so
// the y tile costs no extra LDS.  Row stride = data + 16 B: conflict-free
// ds_read_b128 when every lane reads its own row.
template <typename TI>
struct RowLayout {
  static constexpr int VI = ElemTraits<TI>::kVec;
  static constexpr int kBlock = 32;
  static constexpr int kBlocks = kT / VI;
  static constexpr int kBytes = kBlocks * kBlock;
  static constexpr int kStride = kBytes + 16;
};

// Packed (two positions) softplus and silu (the lane-pair kernels, scan_fwd_pair.hip / scan_bwd_pair.hip): the arithmetic around the transcendental
// ops runs as v_pk_* (one issue for two positions).
__device__ __forceinline__ f32x2 softplus2_log1p(f32x2 x) {
  // softplus(x) = max(x, 0) + log1p(exp(-|x|)): exp never overflows, and above 20 the log1p
  // term is below half an ulp of x, which is torch's threshold (x > 20 -> x) exactly.
  // -|arg| is a free VOP3 input modifier on v_exp_f32.
  const f32x2 arg = x * kLog2e;
  const f32x2 t = f32x2{fast_exp2(-fabsf(arg.x)), fast_exp2(-fabsf(arg.y))};
  const f32x2 tp = t + 1.f;
  const f32x2 lg = f32x2{fast_log2(tp.x), fast_log2(tp.y)};
  return lg * kLn2 + f32x2{fmaxf(x.x, 0.f), fmaxf(x.y, 0.f)};
}
// MC_ASM_TAIL / MC_ASM_HEAD: appended / prepended to the arithmetic inline asm of the scan kernels.  Empty
// in the product build; "s_nop 4" in the hazard-audit builds (make ASM_AUDIT=1: tail, ASM_AUDIT=2: both),
// which give every asm result (and every asm operand) 5 wait states whatever the compiler's hazard
// recognizer assumed about the opaque block.
#ifndef MC_ASM_TAIL
#define MC_ASM_TAIL ""
#endif
#ifndef MC_ASM_HEAD
#define MC_ASM_HEAD ""
#endif
// Packed / transcendental arithmetic of the pair backward's sweeps.  Plain expressions in the product
// build; with MC_PK_PAD / MC_EXP_PAD (diagnostic) each is an asm op followed by "s_nop N", so
// every result has that many extra wait states before its first consumer whatever the compiler scheduled.
#if defined(MC_SCALAR_PK)   // diagnostic: every sweep product as two scalar VALU ops, no packed math
__device__ __forceinline__ f32x2 pmul(f32x2 a, f32x2 b) {
  float x, y;
  asm("v_mul_f32 %0, %2, %3\n\tv_mul_f32 %1, %4, %5" : "=&v"(x), "=&v"(y) : "v"(a.x), "v"(b.x), "v"(a.y), "v"(b.y));
  return f32x2{x, y};
}
__device__ __forceinline__ f32x2 pfma(f32x2 a, f32x2 b, f32x2 c) {
  float x, y;
  asm("v_fma_f32 %0, %2, %3, %4\n\tv_fma_f32 %1, %5, %6, %7" : "=&v"(x), "=&v"(y)
      : "v"(a.x), "v"(b.x), "v"(c.x), "v"(a.y), "v"(b.y), "v"(c.y));
  return f32x2{x, y};
}
#elif defined(MC_PK_PAD)
__device__ __forceinline__ f32x2 pmul(f32x2 a, f32x2 b) {
  f32x2 r;
  asm("v_pk_mul_f32 %0, %1, %2\n\ts_nop " MC_PK_PAD : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f32x2 pfma(f32x2 a, f32x2 b, f32x2 c) {
  f32x2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3\n\ts_nop " MC_PK_PAD : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
#else
__device__ __forceinline__ f32x2 pmul(f32x2 a, f32x2 b) { return a * b; }
__device__ __forceinline__ f32x2 pfma(f32x2 a, f32x2 b, f32x2 c) { return a * b + c; }
#endif
#ifdef MC_EXP_PAD   // (the leading nop covers the VALU -> trans operand read the compiler cannot see into)
__device__ __forceinline__ float pexp2(float a) {
  float r;
  asm("s_nop 1\n\tv_exp_f32 %0, %1\n\ts_nop " MC_EXP_PAD : "=v"(r) : "v"(a));
  return r;
}
#else
__device__ __forceinline__ float pexp2(float a) { return fast_exp2(a); }
#endif
// MC_DIAG_OPSEL_HI (diagnostic build only) restores the round-5 form of the high-half broadcasts (the
// packed op_sel:[0,1] ops below) so that the determinism A/B variants can be rebuilt; the
// product build rejects that form at compile time.
#ifdef MC_DIAG_OPSEL_HI
constexpr bool kDiagOpselHi = true;
#else
constexpr bool kDiagOpselHi = false;
#endif
// a * {s.lo, s.lo} (kHi = 0) or a * {s.hi, s.hi} (kHi = 1, diagnostic only): one v_pk_mul_f32 with
// op_sel (the compiler otherwise moves an odd-register scalar to an even register first)
template <int kHi>
__device__ __forceinline__ f32x2 pk_mul_bcast(f32x2 a, f32x2 s) {
  static_assert(kHi == 0 || kDiagOpselHi, "the op_sel high-half broadcast is diagnostic only (DESIGN 4.9): "
                                          "use pk_mul_bcast_safe");
#ifdef MC_SCALAR_PK
  return pmul(a, f32x2{kHi ? s.y : s.x, kHi ? s.y : s.x});
#endif
#ifdef MC_BCAST_C
  return a * f32x2{kHi ? s.y : s.x, kHi ? s.y : s.x};
#endif
  f32x2 r;
  if constexpr (kHi) asm(MC_ASM_HEAD "v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" MC_ASM_TAIL : "=v"(r) : "v"(a), "v"(s));
  else asm(MC_ASM_HEAD "v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" MC_ASM_TAIL : "=v"(r) : "v"(a), "v"(s));
  return r;
}
// a * s.{lo|hi} + c: one v_pk_fma_f32 with op_sel (same reason; kHi = 1 diagnostic only)
template <int kHi>
__device__ __forceinline__ f32x2 pk_fma_bcast(f32x2 a, f32x2 s, f32x2 c) {
  static_assert(kHi == 0 || kDiagOpselHi, "the op_sel high-half broadcast is diagnostic only (DESIGN 4.9): "
                                          "use pk_fma_bcast_safe");
#ifdef MC_SCALAR_PK
  return pfma(a, f32x2{kHi ? s.y : s.x, kHi ? s.y : s.x}, c);
#endif
#ifdef MC_BCAST_C
  return a * f32x2{kHi ? s.y : s.x, kHi ? s.y : s.x} + c;
#endif
  f32x2 r;
  if constexpr (kHi) asm(MC_ASM_HEAD "v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" MC_ASM_TAIL : "=v"(r) : "v"(a), "v"(s), "v"(c));
  else asm(MC_ASM_HEAD "v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" MC_ASM_TAIL : "=v"(r) : "v"(a), "v"(s), "v"(c));
  return r;
}
// The same products without the op_sel[src] = 1 form (the LOW result reading a source's HIGH half):
// in that form, issued from our inline asm, gfx950 returned wrong low-half results for lanes 48-63 of
// v_pk_mul_f32 / v_pk_fma_f32 now and then while another kernel ran beside it (run-to-run differences of
// the two-stream training step).  kHi = 1 is two scalar ops reading s.hi directly; kHi = 0
// keeps the packed op (op_sel_hi only: the HIGH result reads s.lo).  Where one s.hi feeds several
// products, hi_to_lo() moves it to a low half once and the packed kHi = 0 form broadcasts it.
__device__ __forceinline__ f32x2 hi_to_lo(f32x2 s) {   // {s.hi, unspecified}: one v_mov, no op_sel
  f32x2 r = __builtin_nondeterministic_value(r);
  r.x = s.y;
  return r;
}
template <int kHi>
__device__ __forceinline__ f32x2 pk_mul_bcast_safe(f32x2 a, f32x2 s) {
  if constexpr (kHi && kDiagOpselHi) {
    return pk_mul_bcast<1>(a, s);
  } else if constexpr (kHi) {
    float x, y;
    asm("v_mul_f32 %0, %2, %4\n\tv_mul_f32 %1, %3, %4" : "=&v"(x), "=&v"(y) : "v"(a.x), "v"(a.y), "v"(s.y));
    return f32x2{x, y};
  } else {
    return pk_mul_bcast<0>(a, s);
  }
}
template <int kHi>
__device__ __forceinline__ f32x2 pk_fma_bcast_safe(f32x2 a, f32x2 s, f32x2 c) {
  if constexpr (kHi && kDiagOpselHi) {
    return pk_fma_bcast<1>(a, s, c);
  } else if constexpr (kHi) {
    float x, y;
    asm("v_fma_f32 %0, %2, %4, %5\n\tv_fma_f32 %1, %3, %4, %6" : "=&v"(x), "=&v"(y)
        : "v"(a.x), "v"(a.y), "v"(s.y), "v"(c.x), "v"(c.y));
    return f32x2{x, y};
  } else {
    return pk_fma_bcast<0>(a, s, c);
  }
}
// exp2 of two values on the packed-FMA pipe (no transcendental): round-to-nearest split x = j + f
// with the 1.5 * 2^23 shifter, a degree-6 near-minimax polynomial for 2^f on [-0.5, 0.5] (relative
// error 9.6e-8), j added into the exponent field.  For x in [-126, 126].  A/B lever for the forward
// recurrence (MC_FWD_POLY_PAIRS, scan_fwd_pair.hip): 15 VALU ops for two values against two v_exp_f32.
__device__ __forceinline__ f32x2 exp2_poly2(f32x2 x) {
  x = f32x2{fmaxf(x.x, -126.f), fmaxf(x.y, -126.f)};
  const f32x2 t = x + 12582912.f;
  const f32x2 f = x - (t - 12582912.f);
  f32x2 p = f * 1.534579787403345e-4f + 1.3399930903688073e-3f;
  p = p * f + 9.618489071726799e-3f;
  p = p * f + 5.550328642129898e-2f;
  p = p * f + 2.4022646248340607e-1f;
  p = p * f + 6.931471824645996e-1f;
  p = p * f + 1.f;
  return f32x2{__int_as_float(__float_as_int(p.x) + (__float_as_int(t.x) << 23)),
               __int_as_float(__float_as_int(p.y) + (__float_as_int(t.y) << 23))};
}
__device__ __forceinline__ f32x2 silu2(f32x2 z) {
  const f32x2 arg = z * -kLog2e;
  const f32x2 ep = f32x2{fast_exp2(arg.x), fast_exp2(arg.y)} + 1.f;
  return z * f32x2{fast_rcp(ep.x), fast_rcp(ep.y)};
}

// Forward kernel arguments (scan_fwd.hip, scan_fwd_pair.hip).
// MFMA operand vectors of the projected-delta tile (4 16-bit values per lane)
template <typename TI> struct Mfma16;
template <> struct Mfma16<bf16_t> {
  typedef short v4 __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ f32x4 mma(v4 a, v4 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0); }
};
template <> struct Mfma16<f16_t> {
  typedef _Float16 v4 __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ f32x4 mma(v4 a, v4 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0); }
};

struct FwdArgs {
  int batch, dim, seqlen, dstate, n_groups, n_chunks, n_states, nblk, total_blocks;
  int softplus;
  int64_t u_bs, u_ds, dt_bs, dt_ds, z_bs, z_ds, o_bs, o_ds;
  const void* u; const void* delta; const float* A; const float* bct;
  const float* D; const void* z; const float* delta_bias;
  void* out; float* chunk_states; float* last_state;
  void* out_y; int64_t y_bs, y_ds;   // nullable: pre-gate y + D u (training with z: the backward's dz input)
  int rev_groups, u_groups;          // grouped directions (0 = off; element-wise path only)
  // projected delta (pair kernel only): delta = dpw (dim x rank) . dpx^T, formed per chunk on MFMA
  const void* dpx; const void* dpw; int rank;
  int64_t dpx_bs, dpx_ts, dpw_ds;
  void* delta_out;                   // nullable: the formed delta, strides dt_bs / dt_ds
  // B / C rows as given (the pair kernel reads them directly; the others read the relaid bct)
  const void* B; const void* C;
  int64_t B_bs, B_gs, B_ns, C_bs, C_gs, C_ns;
  int state_interval;                // positions per saved state (pair kernel: 8 or 32; others 32)
};

int validate_common(int batch, int dim, int seqlen, int dstate, int n_groups, int itype, int wtype, const char* who);
bool vec_ok(const void* p, int64_t s0, int64_t s1, int64_t s2, int elem_bytes);

}  // namespace scan
}  // namespace mc
