// mc_common.h -- shared device/host helpers for the MI355X (gfx950) kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>
#include <string>

namespace mc {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// ---------------------------------------------------------------- dtypes
// Element types as they sit in HBM.  bf16 and f16 travel as raw 16-bit words
// and are widened in registers; all arithmetic is fp32.
using bf16_t = __bf16;
using f16_t = _Float16;

// packed fp32 vectors: arithmetic on f32x2 lowers to v_pk_*_f32
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct ElemTraits;
template <> struct ElemTraits<float> { static constexpr int kVec = 4; };   // 16 B = 4 elems
template <> struct ElemTraits<bf16_t> { static constexpr int kVec = 8; };  // 16 B = 8 elems
template <> struct ElemTraits<f16_t> { static constexpr int kVec = 8; };

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16_t x) { return (float)x; }
__device__ __forceinline__ float to_f(f16_t x) { return (float)x; }

template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float x) { return (bf16_t)x; }  // RNE, v_cvt_pk_bf16_f32
template <> __device__ __forceinline__ f16_t from_f<f16_t>(float x) { return (f16_t)x; }

// ---------------------------------------------------------------- 16-byte vectors
// A 16-B vector of 4 (fp32) or 8 (16-bit) elements lives in a uint4; element
// access uses compile-time indices only (no addressable arrays, so nothing is
// demoted to scratch).
__device__ __forceinline__ uint32_t word_of(const uint4& q, int i) {
  return i == 0 ? q.x : (i == 1 ? q.y : (i == 2 ? q.z : q.w));
}

template <typename T> __device__ __forceinline__ float elem_f(const uint4& q, int i);
template <> __device__ __forceinline__ float elem_f<float>(const uint4& q, int i) {
  return __uint_as_float(word_of(q, i));
}
template <> __device__ __forceinline__ float elem_f<bf16_t>(const uint4& q, int i) {
  const uint32_t w = word_of(q, i >> 1);
  return __uint_as_float((i & 1) ? (w & 0xffff0000u) : (w << 16));
}
template <> __device__ __forceinline__ float elem_f<f16_t>(const uint4& q, int i) {
  const uint32_t w = word_of(q, i >> 1);
  return (float)__builtin_bit_cast(f16_t, (uint16_t)((i & 1) ? (w >> 16) : (w & 0xffffu)));
}

template <typename T> __device__ __forceinline__ uint32_t bits16(float x) {
  return (uint32_t)__builtin_bit_cast(uint16_t, from_f<T>(x));
}
// pack kVec fp32 values into the element type
template <typename T> __device__ __forceinline__ uint4 pack_f(const float (&v)[ElemTraits<T>::kVec]);
template <> __device__ __forceinline__ uint4 pack_f<float>(const float (&v)[4]) {
  return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
}
template <typename T>
__device__ __forceinline__ uint4 pack16_impl(const float (&v)[8]) {
  return make_uint4(bits16<T>(v[0]) | (bits16<T>(v[1]) << 16), bits16<T>(v[2]) | (bits16<T>(v[3]) << 16),
                    bits16<T>(v[4]) | (bits16<T>(v[5]) << 16), bits16<T>(v[6]) | (bits16<T>(v[7]) << 16));
}
// 16-bit outputs convert two values per instruction (v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32, RNE)
template <typename T>
__device__ __forceinline__ uint32_t cvt_pk2(float a, float b) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{a, b}), t2));
}
template <typename T>
__device__ __forceinline__ uint4 pack16_pk(const float (&v)[8]) {
  return make_uint4(cvt_pk2<T>(v[0], v[1]), cvt_pk2<T>(v[2], v[3]), cvt_pk2<T>(v[4], v[5]), cvt_pk2<T>(v[6], v[7]));
}
template <> __device__ __forceinline__ uint4 pack_f<bf16_t>(const float (&v)[8]) { return pack16_pk<bf16_t>(v); }
template <> __device__ __forceinline__ uint4 pack_f<f16_t>(const float (&v)[8]) { return pack16_pk<f16_t>(v); }

// raw 16-bit/32-bit element bits
template <typename T> __device__ __forceinline__ uint32_t ld_bits(const T* p) {
  if constexpr (sizeof(T) == 4) return *reinterpret_cast<const uint32_t*>(p);
  else return (uint32_t)*reinterpret_cast<const uint16_t*>(p);
}
template <typename T> __device__ __forceinline__ void st_bits(T* p, uint32_t b) {
  if constexpr (sizeof(T) == 4) *reinterpret_cast<uint32_t*>(p) = b;
  else *reinterpret_cast<uint16_t*>(p) = (uint16_t)b;
}

// Vector load of elements [0, nvalid) from p, zero-filled above; nvalid in [0, kVec].
template <typename T>
__device__ __forceinline__ uint4 ld16_masked(const T* __restrict__ p, int nvalid) {
  constexpr int N = ElemTraits<T>::kVec;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t b = (i < nvalid) ? ld_bits(p + i) : 0u;
    if constexpr (sizeof(T) == 4) w[i] = b;
    else w[i >> 1] |= b << (16 * (i & 1));
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}
template <typename T>
__device__ __forceinline__ void st16_masked(T* __restrict__ p, const uint4& q, int nvalid) {
  constexpr int N = ElemTraits<T>::kVec;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (i < nvalid) {
      if constexpr (sizeof(T) == 4) st_bits(p + i, word_of(q, i));
      else st_bits(p + i, (word_of(q, i >> 1) >> (16 * (i & 1))) & 0xffffu);
    }
  }
}

__device__ __forceinline__ uint4 ld16(const void* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ void st16(void* p, const uint4& q) { *reinterpret_cast<uint4*>(p) = q; }

// Mirrored sequence access for reversed scan groups (SS2D's flipped directions,
// reference model.py:510-517 / 553-565).  A reversed group's chunk of steps
// [l0, l0 + kT) lives at positions [L - l0 - kT, L - l0): lane c of a row moves
// the 16-B block at ascending position cm = L - l0 - kT + c * VI (addresses
// keep increasing with the lane, so the accesses coalesce like a forward walk)
// and the block holds the steps of block kVPR - 1 - c in reverse element order.
// ld16_top: that block in MEMORY order (the caller flips it where the values are
// consumed -- flipping right after the load would make the wave wait for it);
// only its top nvalid elements (the steps < L) exist, the rest read as 0.
// st16_rev: step-ordered values -> the block, flipped, top nvalid elements.
// Whole aligned blocks move as one 16-B access, others element by element.
__device__ __forceinline__ uint32_t swap16(uint32_t w) { return (w >> 16) | (w << 16); }
template <typename T>
__device__ __forceinline__ uint4 reverse_elems(const uint4& q) {
  if constexpr (sizeof(T) == 4) return make_uint4(q.w, q.z, q.y, q.x);
  else return make_uint4(swap16(q.w), swap16(q.z), swap16(q.y), swap16(q.x));
}
template <typename T>
__device__ __forceinline__ uint4 ld16_top(const T* __restrict__ row, int cm, int nvalid) {
  constexpr int N = ElemTraits<T>::kVec;
  if (nvalid == N && ((reinterpret_cast<uintptr_t>(row + cm) & 15) == 0)) return ld16(row + cm);
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t b = (i >= N - nvalid) ? ld_bits(row + (cm + i)) : 0u;
    if constexpr (sizeof(T) == 4) w[i] = b;
    else w[i >> 1] |= b << (16 * (i & 1));
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}
template <typename T>
__device__ __forceinline__ void st16_rev(T* __restrict__ row, int cm, const uint4& q, int nvalid) {
  constexpr int N = ElemTraits<T>::kVec;
  if (nvalid == N && ((reinterpret_cast<uintptr_t>(row + cm) & 15) == 0)) {
    st16(row + cm, reverse_elems<T>(q));
    return;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (i < nvalid) {
      T* p = row + (cm + N - 1 - i);
      if constexpr (sizeof(T) == 4) st_bits(p, word_of(q, i));
      else st_bits(p, (word_of(q, i >> 1) >> (16 * (i & 1))) & 0xffffu);
    }
  }
}

// ---------------------------------------------------------------- raw buffer access
// A buffer resource (V#) holds a wave-uniform base and byte range in SGPRs, so
// a lane's address is ONE 32-bit VGPR offset instead of a 64-bit pointer, and
// a read at or past num_records returns 0 instead of faulting: ragged tails are
// loaded branch-free and masked where used.  Word 3 = raw 32-bit access, gfx9.
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 buf_ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ void buf_st16(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, off, 0, 0);
}
// streaming (non-temporal, nt cache policy) store: the line is not kept in L2 for re-use
__device__ __forceinline__ void buf_st16_nt(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, off, 0, 2);
}
// elements [0, nvalid) of a 16-B vector (nvalid wave-uniform)
template <typename T>
__device__ __forceinline__ void buf_st16_masked(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint4& q, int nvalid) {
  constexpr int N = ElemTraits<T>::kVec;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (i < nvalid) {
      if constexpr (sizeof(T) == 4) __builtin_amdgcn_raw_buffer_store_b32(word_of(q, i), r, off + 4 * i, 0, 0);
      else __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(word_of(q, i >> 1) >> (16 * (i & 1))), r,
                                                 off + 2 * i, 0, 0);
    }
  }
}

// exp2 on the transcendental unit (v_exp_f32)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_log2(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// softplus with torch's threshold (F.softplus: x > 20 -> x).  Branch-free
// (selects only) so it does not split the recurrence's basic block.
__device__ __forceinline__ float softplus_f(float x) {
  const float t = fast_exp2(fminf(x, 20.f) * kLog2e);
  const float lg = fast_log2(1.f + t) * kLn2;
  const float series = t * (1.f - 0.5f * t);  // log1p(t) for tiny t (softplus(-30) != 0)
  const float r = t < 1e-4f ? series : lg;
  return x > 20.f ? x : r;
}
// d softplus / dx = sigmoid(x)
__device__ __forceinline__ float sigmoid_f(float x) { return fast_rcp(1.f + fast_exp2(-x * kLog2e)); }

__device__ __forceinline__ float silu_f(float x) { return x * sigmoid_f(x); }

// GELU, exact erf form (torch F.gelu approximate='none': x * 0.5 * (1 + erf(x / sqrt2))) and its derivative
__device__ __forceinline__ float gelu_f(float x) { return x * 0.5f * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad_f(float x) {   // d/dx [x * Phi(x)]
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return fmaf(x, pdf, cdf);
}
// Phi(x) and pdf(x) = exp(-x^2/2)/sqrt(2 pi) from two v_exp_f32 and one v_rcp_f32 (the GEMM epilogues'
// GELU / GELU', where the library erff's instruction count is not hidden behind memory): for
// z = |x|/sqrt2, erfc(z) = t exp(-z^2 + P(t)), t = 1/(1 + z/2), P the degree-9 Chebyshev fit of
// Numerical Recipes' erfcc (fractional error < 1.2e-7 for every z >= 0, so also in Phi's far tail);
// exp(-z^2) is pdf's own exponential.
__device__ __forceinline__ void phi_pdf_f(float x, float& phi, float& pdf) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.f));
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float e = __builtin_amdgcn_exp2f(-0.72134752044448170f * x * x);   // exp(-x^2/2)
  const float erf_abs = 1.f - t * e * __builtin_amdgcn_exp2f(p * 1.4426950408889634f);   // erf(z), fp32
  // torch's form 0.5 (1 + erf(x / sqrt2)), rounding included: for x << 0 the sum cancels exactly as
  // F.gelu's does (e.g. gelu(-6) = -0 there), so the results match torch's, not the exact Phi
  phi = 0.5f * (1.f + (x < 0.f ? -erf_abs : erf_abs));
  pdf = 0.39894228040143268f * e;
}

// phi_pdf_f on two values at once: the fit's FMAs as packed v_pk_fma_f32 (half the issue slots)
__device__ __forceinline__ void phi_pdf_f2(f32x2 x, f32x2& phi, f32x2& pdf) {
  const f32x2 z = f32x2{fabsf(x.x), fabsf(x.y)} * 0.70710678118654752f;
  const f32x2 d = z * 0.5f + 1.f;
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = f32x2{0.17087277f, 0.17087277f};
  p = p * t + -0.82215223f;
  p = p * t + 1.48851587f;
  p = p * t + -1.13520398f;
  p = p * t + 0.27886807f;
  p = p * t + -0.18628806f;
  p = p * t + 0.09678418f;
  p = p * t + 0.37409196f;
  p = p * t + 1.00002368f;
  p = p * t + -1.26551223f;
  const f32x2 ea = x * x * -0.72134752044448170f;
  const f32x2 e = f32x2{__builtin_amdgcn_exp2f(ea.x), __builtin_amdgcn_exp2f(ea.y)};
  const f32x2 pl = p * 1.4426950408889634f;
  const f32x2 erf_abs = 1.f - t * e * f32x2{__builtin_amdgcn_exp2f(pl.x), __builtin_amdgcn_exp2f(pl.y)};
  const f32x2 erf_x = f32x2{x.x < 0.f ? -erf_abs.x : erf_abs.x, x.y < 0.f ? -erf_abs.y : erf_abs.y};
  phi = (erf_x + 1.f) * 0.5f;
  pdf = e * 0.39894228040143268f;
}

// ---------------------------------------------------------------- host error plumbing
void set_error(const char* fmt, ...);
const char* last_error();

#define MC_CHECK(cond, code, ...)      \
  do {                                 \
    if (!(cond)) {                     \
      ::mc::set_error(__VA_ARGS__);    \
      return (code);                   \
    }                                  \
  } while (0)

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace mc
