// ops.hip -- encoder kernels around the scan for MI355X (gfx950): fused
// residual-add + RMSNorm, residual-add + LayerNorm, causal depthwise conv1d
// (+SiLU), patch im2col.  All are HBM-bound streaming ops: 16-B vector accesses along the
// contiguous dimension, one pass over the data, fp32 math, deterministic
// reductions (per-wave partial slabs + fixed-order column sums).
#include <algorithm>

#include "mc_common.h"
#include "../../include/mc_ops.h"

namespace mc {
namespace ops {

// ------------------------------------------------------------------ RMSNorm
// One wave per row, the row in registers between the two passes; NV = 16-B
// vectors per lane per row (cols <= 64 * NV * V).  The weight vectors a lane
// touches are loaded once per wave (hoisted out of the row loop).  Grid-stride
// over rows so the backward's per-wave dw partials stay few (one slab row per
// wave).
constexpr int kMaxVec = 8;  // 16-B vectors per lane per row: cols <= 4096 (16-bit) / 2048 (fp32)

template <int V>
__device__ __forceinline__ void ld_f32v(const float* __restrict__ p, float (&v)[V]) {
#pragma unroll
  for (int e4 = 0; e4 < V; e4 += 4) {
    const float4 q = *reinterpret_cast<const float4*>(p + e4);
    v[e4] = q.x; v[e4 + 1] = q.y; v[e4 + 2] = q.z; v[e4 + 3] = q.w;
  }
}
template <int V>
__device__ __forceinline__ void st_f32v(float* __restrict__ p, const float (&v)[V]) {
#pragma unroll
  for (int e4 = 0; e4 < V; e4 += 4)
    *reinterpret_cast<float4*>(p + e4) = make_float4(v[e4], v[e4 + 1], v[e4 + 2], v[e4 + 3]);
}

// Sum over the 64 lanes, the same bits in every lane: an xor butterfly on VALU only (DPP inside
// 16-lane rows, permlane swaps across rows) instead of six ds_bpermute round trips.
__device__ __forceinline__ float wave_allsum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true));   // lane ^ 1
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true));   // lane ^ 2
  {                                                                                                // lane ^ 4
    const int iv = __float_as_int(v);
    const int lo = __builtin_amdgcn_update_dpp(iv, iv, 0x104, 0xF, 0x5, false);
    v += __int_as_float(__builtin_amdgcn_update_dpp(lo, iv, 0x114, 0xF, 0xA, false));
  }
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, true));  // lane ^ 8
  const auto p16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p16[0]) + __uint_as_float(p16[1]);                                          // lane ^ 16
  const auto p32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(p32[0]) + __uint_as_float(p32[1]);                                       // lane ^ 32
}

template <typename T, int NV>
__global__ __launch_bounds__(256) void add_rmsnorm_fwd_kernel(int rows, int cols, const T* __restrict__ x,
                                                              const float* __restrict__ res_in,
                                                              const float* __restrict__ w, float eps,
                                                              T* __restrict__ y, float* __restrict__ res_out,
                                                              float* __restrict__ rstd) {
  constexpr int V = ElemTraits<T>::kVec;
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int nvec = cols / V;
  float wr[NV][V];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = lane + 64 * i;
    if (v < nvec) ld_f32v<V>(w + v * V, wr[i]);
  }
  // the NEXT row's x / res_in in flight during this row's math (rows <= 1024 wide)
  uint4 qx[NV];
  float qr[NV][V];
  auto load = [&](int row, uint4 (&a)[NV], float (&b)[NV][V]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      a[i] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int e = 0; e < V; ++e) b[i][e] = 0.f;
      if (v < nvec) {
        const int64_t off = (int64_t)row * cols + v * V;
        a[i] = ld16(x + off);
        if (res_in) ld_f32v<V>(res_in + off, b[i]);
      }
    }
  };
  constexpr bool kPrefetch = NV <= 2;
  if (kPrefetch && wave < rows) load(wave, qx, qr);
  for (int row = wave; row < rows; row += nwaves) {
    uint4 nx[NV];
    float nr[NV][V];
    if constexpr (kPrefetch) {
      if (row + nwaves < rows) load(row + nwaves, nx, nr);
    } else {
      load(row, qx, qr);
    }
    float h[NV][V];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      if (v < nvec) {
#pragma unroll
        for (int e = 0; e < V; ++e) h[i][e] = elem_f<T>(qx[i], e) + qr[i][e];
#pragma unroll
        for (int e = 0; e < V; ++e) ss = fmaf(h[i][e], h[i][e], ss);
      }
    }
    ss = wave_allsum(ss);
    const float rs = rsqrtf(ss / cols + eps);
    if (lane == 0) rstd[row] = rs;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      if (v < nvec) {
        const int64_t off = (int64_t)row * cols + v * V;
        float o[V];
#pragma unroll
        for (int e = 0; e < V; ++e) o[e] = h[i][e] * rs * wr[i][e];
        st16(y + off, pack_f<T>(o));
        if (res_out) st_f32v<V>(res_out + off, h[i]);
      }
    }
    if constexpr (kPrefetch) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        qx[i] = nx[i];
#pragma unroll
        for (int e = 0; e < V; ++e) qr[i][e] = nr[i][e];
      }
    }
  }
}

// The 4 waves of a block fold their per-lane column partials in LDS in a fixed order (wave 0 + 1 + 2 + 3)
// and wave 0 writes ONE partial row per block: the column-sum passes then read kNormGrid rows, not
// 4 kNormGrid.  Every wave of the block must call it (it holds two barriers per vector).
template <int NV, int V>
__device__ __forceinline__ void block_fold_store(const float (&acc)[NV][V], int lane, int nvec, float* __restrict__ dst) {
  __shared__ float red[3][64 * V];
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = lane + 64 * i;
    if (w > 0) {
#pragma unroll
      for (int e = 0; e < V; ++e) red[w - 1][lane * V + e] = acc[i][e];
    }
    __syncthreads();
    if (w == 0 && v < nvec) {
      float o[V];
#pragma unroll
      for (int e = 0; e < V; ++e) o[e] = ((acc[i][e] + red[0][lane * V + e]) + red[1][lane * V + e]) + red[2][lane * V + e];
      st_f32v<V>(dst + v * V, o);
    }
    __syncthreads();
  }
}

template <typename T, int NV>
__global__ __launch_bounds__(256) void add_rmsnorm_bwd_kernel(int rows, int cols, const T* __restrict__ dy,
                                                              const float* __restrict__ dres,
                                                              const float* __restrict__ hbuf,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ rstd, T* __restrict__ dx,
                                                              float* __restrict__ dres_in,
                                                              float* __restrict__ dw_part) {
  constexpr int V = ElemTraits<T>::kVec;
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int nvec = cols / V;
  float wr[NV][V], dwacc[NV][V];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = lane + 64 * i;
#pragma unroll
    for (int e = 0; e < V; ++e) dwacc[i][e] = 0.f;
    if (v < nvec) ld_f32v<V>(w + v * V, wr[i]);
  }
  for (int row = wave; row < rows; row += nwaves) {
    const float rs = rstd[row];
    float h[NV][V], g[NV][V];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      if (v < nvec) {
        const int64_t off = (int64_t)row * cols + v * V;
        const uint4 q = ld16(dy + off);
        ld_f32v<V>(hbuf + off, h[i]);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const float d = elem_f<T>(q, e);
          g[i][e] = d * wr[i][e];
          dot = fmaf(g[i][e], h[i][e], dot);
          dwacc[i][e] = fmaf(d, h[i][e] * rs, dwacc[i][e]);
        }
      }
    }
    dot = wave_allsum(dot);
    const float c = dot * rs * rs / cols;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      if (v < nvec) {
        const int64_t off = (int64_t)row * cols + v * V;
        float o[V];
        float r[V];
        if (dres) ld_f32v<V>(dres + off, r);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          o[e] = rs * (g[i][e] - h[i][e] * c);
          if (dres) o[e] += r[e];
        }
        if (dx) st16(dx + off, pack_f<T>(o));
        if (dres_in) st_f32v<V>(dres_in + off, o);
      }
    }
  }
  block_fold_store<NV, V>(dwacc, lane, nvec, dw_part + (int64_t)blockIdx.x * cols);
}

// Deterministic column sums of a row-major partial slab in two passes:
//   pass 1: grid (ceil(cols/256), kColSlices); thread = one column over a
//           fixed row slice (coalesced across the block) -> tmp[slice][c]
//   pass 2: thread = one column, sums the kColSlices partials in order.
// Columns [0, split) land in out0, [split, cols) in out1 (out1 may be null).
constexpr int kColSlices = 32;

__global__ __launch_bounds__(256) void colsum_pass1_kernel(const float* __restrict__ in, int nrows, int cols,
                                                           float* __restrict__ tmp) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  const int per = (nrows + kColSlices - 1) / kColSlices;
  const int r0 = blockIdx.y * per, r1 = min(nrows, r0 + per);
  float s = 0.f;
#pragma unroll 8   // loads in flight; the summation order is unchanged
  for (int r = r0; r < r1; ++r) s += in[(int64_t)r * cols + c];
  tmp[(int64_t)blockIdx.y * cols + c] = s;
}

__global__ __launch_bounds__(256) void colsum_pass2_kernel(const float* __restrict__ tmp, int cols, int split,
                                                           float* __restrict__ out0, float* __restrict__ out1,
                                                           float* __restrict__ out2) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
#pragma unroll 8
  for (int k = 0; k < kColSlices; ++k) s += tmp[(int64_t)k * cols + c];
  if (c < split) out0[c] = s;
  else if (c < 2 * split) { if (out1) out1[c - split] = s; }
  else if (out2) out2[c - 2 * split] = s;
}

// columns [0, split) -> out0, [split, 2 split) -> out1, [2 split, cols) -> out2 (out1 / out2 nullable)
static void colsum_two_pass(const float* in, int nrows, int cols, int split, float* out0, float* out1, float* tmp,
                            hipStream_t s, float* out2 = nullptr) {
  const int gx = (cols + 255) / 256;
  hipLaunchKernelGGL(colsum_pass1_kernel, dim3(gx, kColSlices), dim3(256), 0, s, in, nrows, cols, tmp);
  hipLaunchKernelGGL(colsum_pass2_kernel, dim3(gx), dim3(256), 0, s, tmp, cols, split, out0, out1, out2);
}

constexpr int kNormGrid = 512;  // blocks of 4 waves: 2048 waves -> 2048 dw partial rows

// ------------------------------------------------------------------ residual-add + LayerNorm
// ViT/BERT pre-LN blocks: h = x + res (stored in the activation dtype, the
// same rounding as the autocast residual add), y = (h - mean) * rstd * w + b
// in fp32 math, stored in the activation dtype.  One wave per row, the row in
// registers, weights hoisted per wave; the backward recomputes xhat from h
// and emits per-wave dw/db partials reduced by colsum_two_pass
// (deterministic).
template <typename T, int NV>
__global__ __launch_bounds__(256) void add_layernorm_fwd_kernel(int rows, int cols, const T* __restrict__ x,
                                                                const T* __restrict__ res,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ bias, float eps,
                                                                T* __restrict__ y, T* __restrict__ h_out,
                                                                float* __restrict__ mean_out,
                                                                float* __restrict__ rstd_out) {
  constexpr int V = ElemTraits<T>::kVec;
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int nvec = cols / V;
  float wr[NV][V], br[NV][V];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = lane + 64 * i;
    if (v < nvec) {
      ld_f32v<V>(w + v * V, wr[i]);
      if (bias) ld_f32v<V>(bias + v * V, br[i]);
      else
#pragma unroll
        for (int e = 0; e < V; ++e) br[i][e] = 0.f;
    }
  }
  // the NEXT row's x / res in flight during this row's math (as the backward; rows <= 1024 wide)
  uint4 qx[NV], qr[NV];
  auto load = [&](int row, uint4 (&a)[NV], uint4 (&b)[NV]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      a[i] = b[i] = make_uint4(0u, 0u, 0u, 0u);
      if (v < nvec) {
        const int64_t off = (int64_t)row * cols + v * V;
        a[i] = ld16(x + off);
        if (res) b[i] = ld16(res + off);
      }
    }
  };
  constexpr bool kPrefetch = NV <= 2;
  if (kPrefetch && wave < rows) load(wave, qx, qr);
  for (int row = wave; row < rows; row += nwaves) {
    uint4 nx[NV], nr[NV];
    if constexpr (kPrefetch) {
      if (row + nwaves < rows) load(row + nwaves, nx, nr);
    } else {
      load(row, qx, qr);
    }
    float h[NV][V];
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      if (v < nvec) {
        const int64_t off = (int64_t)row * cols + v * V;
        const uint4 q = qx[i];
        if (res) {
          const uint4 r = qr[i];
#pragma unroll
          for (int e = 0; e < V; ++e) h[i][e] = to_f(from_f<T>(elem_f<T>(q, e) + elem_f<T>(r, e)));
          if (h_out) st16(h_out + off, pack_f<T>(h[i]));
        } else {
#pragma unroll
          for (int e = 0; e < V; ++e) h[i][e] = elem_f<T>(q, e);
        }
#pragma unroll
        for (int e = 0; e < V; ++e) sum += h[i][e];
      }
    }
    sum = wave_allsum(sum);
    const float mu = sum / cols;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      if (v < nvec)
#pragma unroll
        for (int e = 0; e < V; ++e) { const float c = h[i][e] - mu; ss = fmaf(c, c, ss); }
    }
    ss = wave_allsum(ss);
    const float rs = rsqrtf(ss / cols + eps);
    if (lane == 0) { mean_out[row] = mu; rstd_out[row] = rs; }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      if (v < nvec) {
        float o[V];
#pragma unroll
        for (int e = 0; e < V; ++e) o[e] = fmaf((h[i][e] - mu) * rs, wr[i][e], br[i][e]);
        st16(y + (int64_t)row * cols + v * V, pack_f<T>(o));
      }
    }
    if constexpr (kPrefetch) {
#pragma unroll
      for (int i = 0; i < NV; ++i) { qx[i] = nx[i]; qr[i] = nr[i]; }
    }
  }
}

// dh_total = dh + rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * w
// dx (= dres) = dh_total;  part rows (one per block, its 4 waves folded in order): [block][0..cols) dw, [block][cols..2cols) db and, with kDxSum,
// [block][2cols..3cols) the column sums of dx as stored: the bias gradient of the layer whose output
// entered as x (fc2 / attention proj), taken in this pass instead of a second read of dx
template <typename T, int NV, bool kDxSum>
__global__ __launch_bounds__(256) void add_layernorm_bwd_kernel(int rows, int cols, const T* __restrict__ dy,
                                                                const T* __restrict__ dh,
                                                                const T* __restrict__ hbuf,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd,
                                                                T* __restrict__ dx, float* __restrict__ part) {
  constexpr int V = ElemTraits<T>::kVec;
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int nvec = cols / V;
  float wr[NV][V], dwacc[NV][V], dbacc[NV][V], dxacc[kDxSum ? NV : 1][V];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = lane + 64 * i;
#pragma unroll
    for (int e = 0; e < V; ++e) { dwacc[i][e] = 0.f; dbacc[i][e] = 0.f; if constexpr (kDxSum) dxacc[i][e] = 0.f; }
    if (v < nvec) ld_f32v<V>(w + v * V, wr[i]);
  }
  // one wave per row, the NEXT row's dy / h / dh in flight during this row's math (the kernel is
  // latency-bound at two waves per SIMD otherwise: two dependent HBM round trips per row)
  uint4 qd[NV], qh[NV], qr[NV];
  auto load = [&](int row, uint4 (&a)[NV], uint4 (&b)[NV], uint4 (&c)[NV]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      a[i] = b[i] = c[i] = make_uint4(0u, 0u, 0u, 0u);
      if (v < nvec) {
        const int64_t off = (int64_t)row * cols + v * V;
        a[i] = ld16(dy + off);
        b[i] = ld16(hbuf + off);
        if (dh) c[i] = ld16(dh + off);
      }
    }
  };
  constexpr bool kPrefetch = NV <= 2;   // wider rows: registers for one row only (no spills)
  if (kPrefetch && wave < rows) load(wave, qd, qh, qr);
  for (int row = wave; row < rows; row += nwaves) {
    const float mu = mean[row], rs = rstd[row];
    uint4 nd[NV], nh[NV], nr[NV];
    if constexpr (kPrefetch) {
      if (row + nwaves < rows) load(row + nwaves, nd, nh, nr);
    } else {
      load(row, qd, qh, qr);
    }
    float xh[NV][V], g[NV][V];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      if (v < nvec) {
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const float d = elem_f<T>(qd[i], e);
          xh[i][e] = (elem_f<T>(qh[i], e) - mu) * rs;
          g[i][e] = d * wr[i][e];
          sg += g[i][e];
          sgx = fmaf(g[i][e], xh[i][e], sgx);
          dwacc[i][e] = fmaf(d, xh[i][e], dwacc[i][e]);
          dbacc[i][e] += d;
        }
      }
    }
    sg = wave_allsum(sg);
    sgx = wave_allsum(sgx);
    const float mg = sg / cols, mgx = sgx / cols;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = lane + 64 * i;
      if (v < nvec) {
        const int64_t off = (int64_t)row * cols + v * V;
        float o[V];
#pragma unroll
        for (int e = 0; e < V; ++e) {
          o[e] = rs * (g[i][e] - mg - xh[i][e] * mgx);
          if (dh) o[e] += elem_f<T>(qr[i], e);
        }
        const uint4 oq = pack_f<T>(o);
        st16(dx + off, oq);
        if constexpr (kDxSum) {
#pragma unroll
          for (int e = 0; e < V; ++e) dxacc[i][e] += elem_f<T>(oq, e);
        }
      }
    }
    if constexpr (kPrefetch) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        qd[i] = nd[i];
        qh[i] = nh[i];
        qr[i] = nr[i];
      }
    }
  }
  constexpr int kW = kDxSum ? 3 : 2;   // partial columns per block row
  float* row = part + (int64_t)blockIdx.x * kW * cols;
  block_fold_store<NV, V>(dwacc, lane, nvec, row);
  block_fold_store<NV, V>(dbacc, lane, nvec, row + cols);
  if constexpr (kDxSum) block_fold_store<NV, V>(dxacc, lane, nvec, row + 2 * cols);
}

// vectors per lane per row -> template instance
static inline int norm_nv(int cols, int V) {
  const int per = (cols / V + 63) / 64;
  return per <= 1 ? 1 : per <= 2 ? 2 : per <= 4 ? 4 : 8;
}
#define MC_DISPATCH_NV(nv, ...)                                   \
  do {                                                            \
    if ((nv) == 1) { constexpr int NV = 1; __VA_ARGS__; }         \
    else if ((nv) == 2) { constexpr int NV = 2; __VA_ARGS__; }    \
    else if ((nv) == 4) { constexpr int NV = 4; __VA_ARGS__; }    \
    else { constexpr int NV = 8; __VA_ARGS__; }                   \
  } while (0)

// ------------------------------------------------------------------ causal conv1d
// Vector tiles along the sequence: each work item owns VEC consecutive
// positions t0 .. t0+VEC-1 of one (b, d) row (one 16-B load), and reads the
// K-1 positions before it from the neighbouring vector(s) (cache hits), so
// the row is streamed once, coalesced along L.  VEC = 1 is the generic path
// for unaligned strides / ragged L.
constexpr int kMaxK = 8;

template <typename T, int VEC>
__device__ __forceinline__ void load_vec(const T* __restrict__ p, float (&v)[VEC]) {
  if constexpr (VEC == 1) {
    v[0] = to_f(*p);
  } else {
    const uint4 q = ld16(p);
#pragma unroll
    for (int e = 0; e < VEC; ++e) v[e] = elem_f<T>(q, e);
  }
}

template <typename T, int VEC>
__device__ __forceinline__ void store_vec(T* __restrict__ p, const float (&v)[VEC]) {
  if constexpr (VEC == 1) {
    *p = from_f<T>(v[0]);
  } else {
    st16(p, pack_f<T>(v));
  }
}

// Window of x[t0 - NP*VEC .. t0 + (1+NN)*VEC - 1] in registers (zero outside [0, L)).
template <typename T, int VEC, int NP, int NN>
__device__ __forceinline__ void load_window(const T* __restrict__ xr, int t0, int L,
                                            float (&win)[(NP + 1 + NN) * VEC]) {
#pragma unroll
  for (int j = -NP; j <= NN; ++j) {
    const int t = t0 + j * VEC;
    float v[VEC];
    if (t >= 0 && t < L) {
      load_vec<T, VEC>(xr + t, v);
    } else {
#pragma unroll
      for (int e = 0; e < VEC; ++e) v[e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) win[(j + NP) * VEC + e] = v[e];
  }
}

// KC: the tap count as a compile-time constant (4: Mamba's d_conv) or 0 = runtime K <= kMaxK.
// Items walk the rows in memory order: with the mixer's channel-major views (x_bs = L < x_ds) the
// batch index varies fastest, so a wave's 64 16-B vectors are one contiguous 1 KiB span (ordering
// by channel first touched 160-B rows 40 KiB apart, each straddling two 128-B lines).  32-bit
// index math (the launcher checks the item count).
template <typename T, int VEC, int KC>
__global__ __launch_bounds__(256) void conv1d_fwd_kernel(int batch, int dim, int L, int K_, const T* __restrict__ x,
                                                         int64_t x_bs, int64_t x_ds, const float* __restrict__ w,
                                                         const float* __restrict__ bias, int silu,
                                                         T* __restrict__ y, int64_t y_bs, int64_t y_ds, int bfast) {
  constexpr int KM = KC ? KC : kMaxK;
  const int K = KC ? KC : K_;
  constexpr int NP = (KM - 1 + VEC - 1) / VEC;   // previous vectors covering the K-1 halo
  const unsigned nchunk = (unsigned)(L + VEC - 1) / VEC;
  const unsigned item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= (unsigned)batch * (unsigned)dim * nchunk) return;
  const unsigned row = item / nchunk;
  const int t0 = (int)(item - row * nchunk) * VEC;
  int b, d;
  if (bfast) { d = (int)(row / (unsigned)batch); b = (int)(row - (unsigned)d * batch); }
  else { b = (int)(row / (unsigned)dim); d = (int)(row - (unsigned)b * dim); }
  const T* xr = x + (int64_t)b * x_bs + (int64_t)d * x_ds;
  float win[(NP + 1) * VEC];
  load_window<T, VEC, NP, 0>(xr, t0, L, win);
  float wk[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) wk[k] = k < K ? w[d * K + k] : 0.f;
  const float bv = bias ? bias[d] : 0.f;
  float out[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    float acc = bv;
#pragma unroll
    for (int k = 0; k < KM; ++k)   // tap k reads position t0 + i - (K-1) + k
      if (k < K) acc = fmaf(wk[k], win[NP * VEC + i - (K - 1) + k], acc);
    out[i] = silu ? silu_f(acc) : acc;
  }
  store_vec<T, VEC>(y + (int64_t)b * y_bs + (int64_t)d * y_ds + t0, out);
}

// Backward.  One wave per (channel d, slice of the channel's batch x chunk
// items): per item it recomputes the pre-activation over t0 .. t0+VEC+K-2,
// forms g = dy * act'(pre), writes dx for its VEC positions and accumulates
// dw / dbias in registers; a wave reduction then writes one partial per
// (slice, d) -- deterministic, no atomics.
template <typename T, int VEC, int KC>
__global__ __launch_bounds__(256) void conv1d_bwd_kernel(int batch, int dim, int L, int K_, const T* __restrict__ x,
                                                         int64_t x_bs, int64_t x_ds, const float* __restrict__ w,
                                                         const float* __restrict__ bias, int silu,
                                                         const T* __restrict__ dy, int64_t dy_bs, int64_t dy_ds,
                                                         T* __restrict__ dx, int64_t dx_bs, int64_t dx_ds,
                                                         int items_per_slice, float* __restrict__ part) {
  constexpr int KM = KC ? KC : kMaxK;
  const int K = KC ? KC : K_;
  constexpr int NP = (KM - 1 + VEC - 1) / VEC;
  constexpr int NN = NP;                             // following vectors covering t0+VEC .. t0+VEC+K-2
  constexpr int W = (NP + 1 + NN) * VEC;
  constexpr int G = VEC + KM - 1;                    // g positions t0 .. t0+VEC+K-2
  const int lane = threadIdx.x & 63;
  const int d = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d >= dim) return;
  const int slice = blockIdx.y;
  const int nchunk = (L + VEC - 1) / VEC;
  const int total = batch * nchunk;
  const int i_begin = slice * items_per_slice;
  const int i_end = min(total, i_begin + items_per_slice);
  float wk[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) wk[k] = k < K ? w[d * K + k] : 0.f;
  const float bv = bias ? bias[d] : 0.f;
  float dwk[KM], db = 0.f;
#pragma unroll
  for (int k = 0; k < KM; ++k) dwk[k] = 0.f;
  for (int item = i_begin + lane; item < i_end; item += 64) {
    const int b = item / nchunk;
    const int t0 = (item - b * nchunk) * VEC;
    const T* xr = x + (int64_t)b * x_bs + (int64_t)d * x_ds;
    const T* gyr = dy + (int64_t)b * dy_bs + (int64_t)d * dy_ds;
    T* dxr = dx + (int64_t)b * dx_bs + (int64_t)d * dx_ds;
    float win[W];
    load_window<T, VEC, NP, NN>(xr, t0, L, win);
    float gy[(1 + NN) * VEC];
#pragma unroll
    for (int j = 0; j <= NN; ++j) {
      const int t = t0 + j * VEC;
      float v[VEC];
      if (t < L) {
        load_vec<T, VEC>(gyr + t, v);
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) v[e] = 0.f;
      }
#pragma unroll
      for (int e = 0; e < VEC; ++e) gy[j * VEC + e] = v[e];
    }
    float g[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      float pre = bv;
#pragma unroll
      for (int k = 0; k < KM; ++k)
        if (k < K) pre = fmaf(wk[k], win[NP * VEC + j - (K - 1) + k], pre);
      float gj = gy[j];                               // zero beyond L (loaded as 0)
      if (silu) {
        const float s = sigmoid_f(pre);
        gj *= s * (1.f + pre * (1.f - s));
      }
      g[j] = (t0 + j < L) ? gj : 0.f;
    }
    float out[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < KM; ++k)                  // dx[t] = sum_k w[k] g[t + K-1-k]
        if (k < K) acc = fmaf(wk[k], g[i + (K - 1) - k], acc);
      out[i] = acc;
      db += g[i];
#pragma unroll
      for (int k = 0; k < KM; ++k)
        if (k < K) dwk[k] = fmaf(g[i], win[NP * VEC + i - (K - 1) + k], dwk[k]);
    }
    store_vec<T, VEC>(dxr + t0, out);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
    for (int k = 0; k < KM; ++k) dwk[k] += __shfl_xor(dwk[k], o);
    db += __shfl_xor(db, o);
  }
  if (lane == 0) {
    float* pr = part + ((int64_t)slice * dim + d) * (kMaxK + 1);
#pragma unroll
    for (int k = 0; k < KM; ++k) pr[k] = dwk[k];   // slots >= K are never read
    pr[kMaxK] = db;
  }
}

// Backward for vector rows and Mamba's K = 4 (K - 1 <= VEC): lane l takes item base + l, so lane
// l + 1 holds the next VEC positions of the same row.  Each lane forms g = dy * act'(pre) for its own
// VEC positions only and takes the K - 1 halo values g[t0 + VEC ..] from lane l + 1 (one shuffle
// each); the wave advances by 63 items, lane 63 forming g only as lane 62's halo.  Against the
// generic kernel: 8 instead of 11 sigmoids per item, and neither the x vector after the item nor
// the next dy vector is loaded.  Same sums, same order (g values are bit-identical either way).
template <typename T, int VEC>
__global__ __launch_bounds__(256) void conv1d_bwd_halo_kernel(int batch, int dim, int L, const T* __restrict__ x,
                                                              int64_t x_bs, int64_t x_ds, const float* __restrict__ w,
                                                              const float* __restrict__ bias, int silu,
                                                              const T* __restrict__ dy, int64_t dy_bs, int64_t dy_ds,
                                                              T* __restrict__ dx, int64_t dx_bs, int64_t dx_ds,
                                                              int items_per_slice, float* __restrict__ part) {
  constexpr int K = 4;
  static_assert(K - 1 <= VEC, "halo from one neighbour");
  const int lane = threadIdx.x & 63;
  const int d = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d >= dim) return;   // whole wave: the shuffles below see all 64 lanes
  const int slice = blockIdx.y;
  const int nchunk = (L + VEC - 1) / VEC;
  const int total = batch * nchunk;
  const int i_begin = slice * items_per_slice;
  const int i_end = min(total, i_begin + items_per_slice);
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[d * K + k];
  const float bv = bias ? bias[d] : 0.f;
  float dwk[K] = {0.f, 0.f, 0.f, 0.f}, db = 0.f;
  for (int base = i_begin; base < i_end; base += 63) {
    const int item = base + lane;
    const bool live = item < total;                      // forms g (lane 63: lane 62's halo)
    const bool own = lane < 63 && item < i_end;          // writes dx, accumulates dw / db
    const int it = live ? item : total - 1;
    const int b = it / nchunk;
    const int t0 = (it - b * nchunk) * VEC;
    const T* xr = x + (int64_t)b * x_bs + (int64_t)d * x_ds;
    float win[2 * VEC];
    load_window<T, VEC, 1, 0>(xr, t0, L, win);
    float gy[VEC];
    load_vec<T, VEC>(dy + (int64_t)b * dy_bs + (int64_t)d * dy_ds + t0, gy);
    float g[VEC + K - 1];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float pre = bv;
#pragma unroll
      for (int k = 0; k < K; ++k) pre = fmaf(wk[k], win[VEC + j - (K - 1) + k], pre);
      float gj = gy[j];
      if (silu) {
        const float s = sigmoid_f(pre);
        gj *= s * (1.f + pre * (1.f - s));
      }
      g[j] = live ? gj : 0.f;
    }
#pragma unroll
    for (int j = 0; j < K - 1; ++j) {
      const float h = __shfl_down(g[j], 1);
      g[VEC + j] = (t0 + VEC + j < L) ? h : 0.f;         // past the row's end: zero (as the generic kernel)
    }
    if (own) {
      float out[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) acc = fmaf(wk[k], g[i + (K - 1) - k], acc);
        out[i] = acc;
        db += g[i];
#pragma unroll
        for (int k = 0; k < K; ++k) dwk[k] = fmaf(g[i], win[VEC + i - (K - 1) + k], dwk[k]);
      }
      store_vec<T, VEC>(dx + (int64_t)b * dx_bs + (int64_t)d * dx_ds + t0, out);
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
    for (int k = 0; k < K; ++k) dwk[k] += __shfl_xor(dwk[k], o);
    db += __shfl_xor(db, o);
  }
  if (lane == 0) {
    float* pr = part + ((int64_t)slice * dim + d) * (kMaxK + 1);
#pragma unroll
    for (int k = 0; k < K; ++k) pr[k] = dwk[k];
    pr[kMaxK] = db;
  }
}

// dw[d, k] = sum_s part[s, d, k]; dbias[d] = sum_s part[s, d, kMaxK]   (fixed order)
__global__ __launch_bounds__(256) void conv1d_reduce_kernel(const float* __restrict__ part, int nslice, int dim, int K,
                                                            float* __restrict__ dw, float* __restrict__ dbias) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= dim * (K + 1)) return;
  const int d = i / (K + 1), k = i % (K + 1);
  const int slot = k < K ? k : kMaxK;
  float s = 0.f;
  for (int b = 0; b < nslice; ++b) s += part[((int64_t)b * dim + d) * (kMaxK + 1) + slot];
  if (k < K) dw[d * K + k] = s;
  else if (dbias) dbias[d] = s;
}

// batch x chunk items per backward wave: ~4 items per lane
// (step: items a wave advances per iteration -- 63 for the halo kernel; slices are whole iterations
// there, so no iteration runs a handful of items)
static inline int conv1d_items_per_slice(int batch, int L, int vec, int step = 64) {
  const int nchunk = (L + vec - 1) / vec;
  const int total = batch * nchunk;
  const int target = step * 4;          // 4 items per lane: enough waves to hide the load latency
  const int nslice = std::max(1, (total + target - 1) / target);
  const int per = (total + nslice - 1) / nslice;
  return step == 64 ? per : (per + step - 1) / step * step;
}

// ------------------------------------------------------------------ patch im2col
template <typename T>
__global__ __launch_bounds__(256) void im2col_kernel(int batch, int C, int H, int W, int P, const T* __restrict__ img,
                                                     T* __restrict__ out) {
  const int ph = H / P, pw = W / P;
  const int64_t cols = (int64_t)C * P * P;
  const int64_t total = (int64_t)batch * ph * pw * cols;
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += (int64_t)gridDim.x * blockDim.x) {
    const int64_t prow = o / cols;
    const int col = (int)(o % cols);
    const int kx = col % P, ky = (col / P) % P, c = col / (P * P);
    const int j = (int)(prow % pw), i = (int)((prow / pw) % ph);
    const int b = (int)(prow / ((int64_t)ph * pw));
    out[o] = img[(((int64_t)b * C + c) * H + i * P + ky) * W + j * P + kx];
  }
}

}  // namespace ops
// ------------------------------------------------------------------ fused bias-gradient passes
// Both kernels stream a (rows x cols) gradient once, coalesced along the row
// (a wave = 64 consecutive 16-B column vectors of one row), write it, and sum
// its columns on the way -- the bias gradient the unfused path gets from a
// second full read.  Block = 64 column vectors x 4 row lanes over one row
// slice; the 4 lanes meet in LDS and one fp32 partial per (slice, column)
// goes to the workspace; colsum_slices_kernel folds the slices in order
// (deterministic, no atomics).  The sums are of the values as stored (rounded
// to the activation dtype), like the unfused reduction.
constexpr int kGradSlices = 512;


template <typename T>
__global__ __launch_bounds__(256) void gelu_bwd_colsum_kernel(int rows, int cols, const T* __restrict__ h, int64_t ldh,
                                                              const T* __restrict__ ga, int64_t ldga, T* __restrict__ gh,
                                                              int64_t ldgh, float* __restrict__ part) {
  constexpr int V = ElemTraits<T>::kVec;
  __shared__ float red[3][64 * V];
  const int lane = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int cv = blockIdx.x * 64 + lane;
  const bool ok = cv < cols / V;
  const int per = (rows + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
  float acc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = 0.f;
  if (ok) {
    // two rows per step: both rows' loads are in flight before the first use
    for (int r = r0 + rl; r < r1; r += 8) {
      const int r2 = min(r + 4, r1 - 1);
      const bool two = r + 4 < r1;
      const uint4 hq = ld16(h + (int64_t)r * ldh + cv * V);
      const uint4 gq = ld16(ga + (int64_t)r * ldga + cv * V);
      const uint4 hq2 = ld16(h + (int64_t)r2 * ldh + cv * V);
      const uint4 gq2 = ld16(ga + (int64_t)r2 * ldga + cv * V);
      float o[V], o2[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        o[e] = elem_f<T>(gq, e) * gelu_grad_f(elem_f<T>(hq, e));
        o2[e] = elem_f<T>(gq2, e) * gelu_grad_f(elem_f<T>(hq2, e));
      }
      const uint4 oq = pack_f<T>(o), oq2 = pack_f<T>(o2);
      st16(gh + (int64_t)r * ldgh + cv * V, oq);
      if (two) st16(gh + (int64_t)r2 * ldgh + cv * V, oq2);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] += elem_f<T>(oq, e) + (two ? elem_f<T>(oq2, e) : 0.f);
    }
  }
  if (rl > 0) {
#pragma unroll
    for (int e = 0; e < V; ++e) red[rl - 1][lane * V + e] = acc[e];
  }
  __syncthreads();
  if (rl == 0 && ok) {
#pragma unroll
    for (int e = 0; e < V; ++e)
      part[(int64_t)blockIdx.y * cols + cv * V + e] = ((acc[e] + red[0][lane * V + e]) + red[1][lane * V + e]) +
                                                      red[2][lane * V + e];
  }
}

// Attention q/k/v gradients -> the packed (B*N, 3*H*D) gradient of the qkv
// projection output (the layout of its (B, N, 3, H, D) view) + its column sums.
struct QkvSrc {
  const void* p[3];
  int64_t sb[3], sn[3], sh[3];   // element strides of (batch, token, head); head_dim stride 1
};

template <typename T>
__global__ __launch_bounds__(256) void qkv_pack_colsum_kernel(int batch, int seq, int heads, int hd, const QkvSrc src,
                                                              T* __restrict__ out, int64_t ldo, float* __restrict__ part) {
  constexpr int V = ElemTraits<T>::kVec;
  __shared__ float red[3][64 * V];
  const int lane = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int cols = 3 * heads * hd;
  const int cv = blockIdx.x * 64 + lane;
  const bool ok = cv < cols / V;
  const int vph = hd / V;                         // vectors per head
  const int s3 = ok ? cv / (heads * vph) : 0;
  const int hh = ok ? (cv / vph) % heads : 0;
  const int dv = ok ? cv % vph : 0;
  const T* base = reinterpret_cast<const T*>(s3 == 0 ? src.p[0] : (s3 == 1 ? src.p[1] : src.p[2]));
  const int64_t sb = s3 == 0 ? src.sb[0] : (s3 == 1 ? src.sb[1] : src.sb[2]);
  const int64_t sn = s3 == 0 ? src.sn[0] : (s3 == 1 ? src.sn[1] : src.sn[2]);
  const int64_t sh = s3 == 0 ? src.sh[0] : (s3 == 1 ? src.sh[1] : src.sh[2]);
  base += (int64_t)hh * sh + dv * V;
  const int rows = batch * seq;
  const int per = (rows + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
  float acc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = 0.f;
  if (ok) {
    for (int r = r0 + rl; r < r1; r += 4) {
      const int b = r / seq, n = r - b * seq;
      const uint4 q = ld16(base + (int64_t)b * sb + (int64_t)n * sn);
      st16(out + (int64_t)r * ldo + cv * V, q);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] += elem_f<T>(q, e);
    }
  }
  if (rl > 0) {
#pragma unroll
    for (int e = 0; e < V; ++e) red[rl - 1][lane * V + e] = acc[e];
  }
  __syncthreads();
  if (rl == 0 && ok && part) {
#pragma unroll
    for (int e = 0; e < V; ++e)
      part[(int64_t)blockIdx.y * cols + cv * V + e] = ((acc[e] + red[0][lane * V + e]) + red[1][lane * V + e]) +
                                                      red[2][lane * V + e];
  }
}

// out[c] = sum_k part[k][c]: a block = 32 columns x 8 slice lanes (independent loads in flight),
// the 8 lane sums meet in LDS in a fixed order
__global__ __launch_bounds__(256) void colsum_slices_kernel(const float* __restrict__ part, int nslices, int cols,
                                                            float* __restrict__ out) {
  __shared__ float red[8][33];
  const int cx = threadIdx.x & 31, q = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cx;
  float s = 0.f;
  if (c < cols)
#pragma unroll 8   // loads in flight; the summation order is unchanged
    for (int k = q; k < nslices; k += 8) s += part[(int64_t)k * cols + c];
  red[q][cx] = s;
  __syncthreads();
  if (q == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][cx];
    out[c] = t;
  }
}


// ------------------------------------------------------------------ column sums and row L2-normalize
// The reductions the towers' glue would otherwise leave to torch: torch's cross-
// workgroup reductions (a staging buffer and a per-output ticket combine partials from several
// workgroups) returned wrong sums for ~0.1 % of the outputs while library GEMMs ran on the other
// stream (tools/sum_under_load.py).  These kernels never hand data between workgroups of one launch:
// pass 1 writes one partial row per fixed row slice, pass 2 (colsum_slices_kernel) folds the slices
// in order -- deterministic and independent of what else runs on the device.

// part[slice][c] = sum over rows [slice * per, (slice + 1) * per) of x[r][c]; block = 4 row lanes x 64
// column vectors of V elements, the 4 lanes meet in LDS in a fixed order.
template <typename T, int V>
__global__ __launch_bounds__(256) void colsum_rows_kernel(int rows, int cols, const T* __restrict__ x, int64_t ld,
                                                          float* __restrict__ part) {
  __shared__ float red[3][64 * V];
  const int lane = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int cv = blockIdx.x * 64 + lane;
  const bool ok = cv * V < cols;
  const int per = (rows + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
  float acc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = 0.f;
  if (ok) {
    if constexpr (V > 1) {
#pragma unroll 4
      for (int r = r0 + rl; r < r1; r += 4) {
        const uint4 q = ld16(x + (int64_t)r * ld + cv * V);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += elem_f<T>(q, e);
      }
    } else {
#pragma unroll 4
      for (int r = r0 + rl; r < r1; r += 4) acc[0] += to_f(x[(int64_t)r * ld + cv]);
    }
  }
  if (rl > 0) {
#pragma unroll
    for (int e = 0; e < V; ++e) red[rl - 1][lane * V + e] = acc[e];
  }
  __syncthreads();
  if (rl == 0 && ok) {
#pragma unroll
    for (int e = 0; e < V; ++e)
      part[(int64_t)blockIdx.y * cols + cv * V + e] = ((acc[e] + red[0][lane * V + e]) + red[1][lane * V + e]) +
                                                      red[2][lane * V + e];
  }
}

// y = x / max(||x||, eps) per row (torch.nn.functional.normalize, p = 2); one wave per row, fp32 out,
// norm[r] = ||x_r|| (unclamped) saved for the backward.
template <typename T>
__global__ __launch_bounds__(256) void l2norm_fwd_kernel(int rows, int cols, const T* __restrict__ x, int64_t ldx,
                                                         float eps, float* __restrict__ y, int64_t ldy,
                                                         float* __restrict__ norm) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const T* xr = x + (int64_t)r * ldx;
  float ss = 0.f;
  for (int c = lane; c < cols; c += 64) {
    const float v = to_f(xr[c]);
    ss += v * v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  const float n = sqrtf(ss);
  const float inv = 1.f / fmaxf(n, eps);
  float* yr = y + (int64_t)r * ldy;
  for (int c = lane; c < cols; c += 64) yr[c] = to_f(xr[c]) * inv;
  if (lane == 0) norm[r] = n;
}

// dx = (g - y (y . g)) / ||x|| where ||x|| > eps, else g / eps (the clamp passes no gradient to the
// norm); y recomputed from x.  dx in x's dtype.
template <typename T>
__global__ __launch_bounds__(256) void l2norm_bwd_kernel(int rows, int cols, const T* __restrict__ x, int64_t ldx,
                                                         const float* __restrict__ norm, float eps,
                                                         const float* __restrict__ g, int64_t ldg,
                                                         T* __restrict__ dx, int64_t lddx) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const T* xr = x + (int64_t)r * ldx;
  const float* gr = g + (int64_t)r * ldg;
  const float n = norm[r];
  const bool clamped = !(n > eps);
  const float c_ = clamped ? eps : n;
  float dot = 0.f;
  if (!clamped) {
    for (int c = lane; c < cols; c += 64) dot += to_f(xr[c]) * gr[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
  }
  const float inv = 1.f / c_;
  const float k = clamped ? 0.f : dot * inv * inv * inv;   // (y . g) / c with y = x / c
  T* dr = dx + (int64_t)r * lddx;
  for (int c = lane; c < cols; c += 64) dr[c] = from_f<T>(gr[c] * inv - to_f(xr[c]) * k);
}

}  // namespace mc

using namespace mc;
using namespace mc::ops;

#define MC_DISPATCH_T(dtype, ...)                                   \
  do {                                                              \
    if ((dtype) == MC_DTYPE_F32) { using T = float; __VA_ARGS__; }  \
    else if ((dtype) == MC_DTYPE_BF16) { using T = bf16_t; __VA_ARGS__; } \
    else { using T = f16_t; __VA_ARGS__; }                          \
  } while (0)

static int check_launch(const char* who) {
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "%s: launch failed: %s", who, hipGetErrorString(e));
  return MC_OK;
}

extern "C" int mc_add_rmsnorm_fwd(int32_t rows, int32_t cols, int32_t dtype, const void* x, const float* res_in,
                                  const float* w, float eps, void* y, float* res_out, float* rstd, void* stream) {
  MC_CHECK(dtype >= MC_DTYPE_F32 && dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_add_rmsnorm_fwd: bad dtype");
  const int V = dtype == MC_DTYPE_F32 ? 4 : 8;
  MC_CHECK(rows >= 0 && cols > 0 && cols % V == 0 && cols / V <= 64 * kMaxVec, MC_ERR_SHAPE,
           "mc_add_rmsnorm_fwd: cols=%d must be a multiple of %d and <= %d", cols, V, 64 * kMaxVec * V);
  if (rows == 0) return MC_OK;
  MC_CHECK(x && w && y && rstd && aligned16(x) && aligned16(y), MC_ERR_INVALID,
           "mc_add_rmsnorm_fwd: x, w, y, rstd required (x, y 16-B aligned)");
  const int grid = std::min((rows + 3) / 4, 4096);
  MC_DISPATCH_T(dtype, MC_DISPATCH_NV(norm_nv(cols, V), hipLaunchKernelGGL((add_rmsnorm_fwd_kernel<T, NV>), dim3(grid),
      dim3(256), 0, (hipStream_t)stream, rows, cols, (const T*)x, res_in, w, eps, (T*)y, res_out, rstd)));
  return check_launch("mc_add_rmsnorm_fwd");
}

extern "C" size_t mc_add_rmsnorm_bwd_workspace_bytes(int32_t rows, int32_t cols) {
  (void)rows;
  return ((size_t)kNormGrid * 4 + kColSlices) * cols * sizeof(float);   // per-wave partials + column-sum slices
}

extern "C" int mc_add_rmsnorm_bwd(int32_t rows, int32_t cols, int32_t dtype, const void* dy, const float* dres,
                                  const float* h, const float* w, const float* rstd, void* dx, float* dres_in,
                                  float* dw, void* workspace, size_t workspace_bytes, void* stream) {
  MC_CHECK(dtype >= MC_DTYPE_F32 && dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_add_rmsnorm_bwd: bad dtype");
  const int V = dtype == MC_DTYPE_F32 ? 4 : 8;
  MC_CHECK(rows >= 0 && cols > 0 && cols % V == 0 && cols / V <= 64 * kMaxVec, MC_ERR_SHAPE,
           "mc_add_rmsnorm_bwd: bad cols=%d", cols);
  MC_CHECK(dy && h && w && rstd && dw, MC_ERR_INVALID, "mc_add_rmsnorm_bwd: dy, h, w, rstd, dw required");
  MC_CHECK(workspace && workspace_bytes >= mc_add_rmsnorm_bwd_workspace_bytes(rows, cols), MC_ERR_WORKSPACE,
           "mc_add_rmsnorm_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  float* part = reinterpret_cast<float*>(workspace);
  MC_DISPATCH_T(dtype, MC_DISPATCH_NV(norm_nv(cols, V), hipLaunchKernelGGL((add_rmsnorm_bwd_kernel<T, NV>),
      dim3(kNormGrid), dim3(256), 0, s, rows, cols, (const T*)dy, dres, h, w, rstd, (T*)dx, dres_in, part)));
  colsum_two_pass(part, kNormGrid, cols, cols, dw, nullptr, part + (size_t)kNormGrid * 4 * cols, s);
  return check_launch("mc_add_rmsnorm_bwd");
}

extern "C" int mc_add_layernorm_fwd(int32_t rows, int32_t cols, int32_t dtype, const void* x, const void* res,
                                    const float* w, const float* bias, float eps, void* y, void* h_out, float* mean,
                                    float* rstd, void* stream) {
  MC_CHECK(dtype >= MC_DTYPE_F32 && dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_add_layernorm_fwd: bad dtype");
  const int V = dtype == MC_DTYPE_F32 ? 4 : 8;
  MC_CHECK(rows >= 0 && cols > 0 && cols % V == 0 && cols / V <= 64 * kMaxVec, MC_ERR_SHAPE,
           "mc_add_layernorm_fwd: cols=%d must be a multiple of %d and <= %d", cols, V, 64 * kMaxVec * V);
  if (rows == 0) return MC_OK;
  MC_CHECK(x && w && y && mean && rstd && aligned16(x) && aligned16(y) && (!res || aligned16(res)) &&
               (!h_out || aligned16(h_out)),
           MC_ERR_INVALID, "mc_add_layernorm_fwd: x, w, y, mean, rstd required (16-B aligned rows)");
  const int grid = std::min((rows + 3) / 4, 4096);
  MC_DISPATCH_T(dtype, MC_DISPATCH_NV(norm_nv(cols, V), hipLaunchKernelGGL((add_layernorm_fwd_kernel<T, NV>),
      dim3(grid), dim3(256), 0, (hipStream_t)stream, rows, cols, (const T*)x, (const T*)res, w, bias, eps, (T*)y,
      (T*)h_out, mean, rstd)));
  return check_launch("mc_add_layernorm_fwd");
}

extern "C" size_t mc_add_layernorm_bwd_workspace_bytes(int32_t rows, int32_t cols) {
  (void)rows;
  return ((size_t)kNormGrid * 4 + kColSlices) * 3 * cols * sizeof(float);   // per-wave dw|db|dxsum partials + slices
}

extern "C" int mc_add_layernorm_bwd(int32_t rows, int32_t cols, int32_t dtype, const void* dy, const void* dh,
                                    const void* h, const float* w, const float* mean, const float* rstd, void* dx,
                                    float* dw, float* dbias, float* dx_colsum, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  MC_CHECK(dtype >= MC_DTYPE_F32 && dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_add_layernorm_bwd: bad dtype");
  const int V = dtype == MC_DTYPE_F32 ? 4 : 8;
  MC_CHECK(rows >= 0 && cols > 0 && cols % V == 0 && cols / V <= 64 * kMaxVec, MC_ERR_SHAPE,
           "mc_add_layernorm_bwd: bad cols=%d", cols);
  MC_CHECK(dy && h && w && mean && rstd && dx && dw, MC_ERR_INVALID,
           "mc_add_layernorm_bwd: dy, h, w, mean, rstd, dx, dw required");
  MC_CHECK(workspace && workspace_bytes >= mc_add_layernorm_bwd_workspace_bytes(rows, cols), MC_ERR_WORKSPACE,
           "mc_add_layernorm_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  float* part = reinterpret_cast<float*>(workspace);
  const int kw = dx_colsum ? 3 : 2;
  if (dx_colsum)
    MC_DISPATCH_T(dtype, MC_DISPATCH_NV(norm_nv(cols, V), hipLaunchKernelGGL((add_layernorm_bwd_kernel<T, NV, true>),
        dim3(kNormGrid), dim3(256), 0, s, rows, cols, (const T*)dy, (const T*)dh, (const T*)h, w, mean, rstd, (T*)dx,
        part)));
  else
    MC_DISPATCH_T(dtype, MC_DISPATCH_NV(norm_nv(cols, V), hipLaunchKernelGGL((add_layernorm_bwd_kernel<T, NV, false>),
        dim3(kNormGrid), dim3(256), 0, s, rows, cols, (const T*)dy, (const T*)dh, (const T*)h, w, mean, rstd, (T*)dx,
        part)));
  // part is [block][kw * cols]: dw in columns [0, cols), dbias in [cols, 2 cols), dx sums in [2 cols, 3 cols)
  colsum_two_pass(part, kNormGrid, kw * cols, cols, dw, dbias, part + (size_t)kNormGrid * 4 * kw * cols, s,
                  dx_colsum);
  return check_launch("mc_add_layernorm_bwd");
}

// VEC path when every row start is 16-B aligned and L is a whole number of vectors.
static bool conv1d_vec_ok(const void* p, int64_t bs, int64_t ds, int V) {
  return aligned16(p) && bs % V == 0 && ds % V == 0;
}

#define MC_DISPATCH_VEC(vec, ...)                                      \
  do {                                                                 \
    if ((vec) == 1) { constexpr int VEC = 1; __VA_ARGS__; }            \
    else if ((vec) == 4) { constexpr int VEC = 4; __VA_ARGS__; }       \
    else { constexpr int VEC = 8; __VA_ARGS__; }                       \
  } while (0)

extern "C" int mc_causal_conv1d_fwd(int32_t batch, int32_t dim, int32_t seqlen, int32_t K, int32_t dtype,
                                    const void* x, int64_t x_bs, int64_t x_ds, const float* w, const float* bias,
                                    int32_t silu, void* y, int64_t y_bs, int64_t y_ds, void* stream) {
  MC_CHECK(dtype >= MC_DTYPE_F32 && dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_causal_conv1d_fwd: bad dtype");
  MC_CHECK(batch >= 0 && dim > 0 && seqlen >= 0 && K >= 1 && K <= kMaxK, MC_ERR_SHAPE,
           "mc_causal_conv1d_fwd: bad shape (K must be in [1, %d])", kMaxK);
  if (batch == 0 || seqlen == 0) return MC_OK;
  MC_CHECK(x && w && y, MC_ERR_INVALID, "mc_causal_conv1d_fwd: x, w, y required");
  const int V = dtype == MC_DTYPE_F32 ? 4 : 8;
  const int vec = seqlen % V == 0 && conv1d_vec_ok(x, x_bs, x_ds, V) && conv1d_vec_ok(y, y_bs, y_ds, V) ? V : 1;
  const int64_t items = (int64_t)batch * dim * ((seqlen + vec - 1) / vec);
  MC_CHECK(items < (int64_t(1) << 31), MC_ERR_SHAPE, "mc_causal_conv1d_fwd: %lld vector items exceed 2^31",
           (long long)items);
  const dim3 grid((unsigned)((items + 255) / 256));
  const int bfast = x_bs < x_ds;   // rows adjacent in memory along the batch (channel-major views)
  MC_DISPATCH_T(dtype, MC_DISPATCH_VEC(vec, if constexpr (VEC == 1 || VEC == ElemTraits<T>::kVec) {
    if (K == 4)
      hipLaunchKernelGGL((conv1d_fwd_kernel<T, VEC, 4>), grid, dim3(256), 0, (hipStream_t)stream, batch, dim, seqlen,
                         K, (const T*)x, x_bs, x_ds, w, bias, silu, (T*)y, y_bs, y_ds, bfast);
    else
      hipLaunchKernelGGL((conv1d_fwd_kernel<T, VEC, 0>), grid, dim3(256), 0, (hipStream_t)stream, batch, dim, seqlen,
                         K, (const T*)x, x_bs, x_ds, w, bias, silu, (T*)y, y_bs, y_ds, bfast);
  }));
  return check_launch("mc_causal_conv1d_fwd");
}

extern "C" size_t mc_causal_conv1d_bwd_workspace_bytes(int32_t batch, int32_t dim, int32_t seqlen, int32_t K) {
  (void)K;
  const int items = conv1d_items_per_slice(batch, seqlen, 1);          // VEC = 1 has the most slices
  const int64_t total = (int64_t)batch * std::max(seqlen, 1);
  const int64_t nslice = std::max<int64_t>(1, (total + items - 1) / items);
  return (size_t)nslice * dim * (kMaxK + 1) * sizeof(float);
}

extern "C" int mc_causal_conv1d_bwd(int32_t batch, int32_t dim, int32_t seqlen, int32_t K, int32_t dtype,
                                    const void* x, int64_t x_bs, int64_t x_ds, const float* w, const float* bias,
                                    int32_t silu, const void* dy, int64_t dy_bs, int64_t dy_ds, void* dx,
                                    int64_t dx_bs, int64_t dx_ds, float* dw, float* dbias, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  MC_CHECK(dtype >= MC_DTYPE_F32 && dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_causal_conv1d_bwd: bad dtype");
  MC_CHECK(batch >= 0 && dim > 0 && seqlen >= 0 && K >= 1 && K <= kMaxK, MC_ERR_SHAPE, "mc_causal_conv1d_bwd: bad shape");
  hipStream_t s = (hipStream_t)stream;
  if (batch == 0 || seqlen == 0) {
    if (dw) (void)hipMemsetAsync(dw, 0, (size_t)dim * K * 4, s);
    if (dbias) (void)hipMemsetAsync(dbias, 0, (size_t)dim * 4, s);
    return MC_OK;
  }
  MC_CHECK(x && w && dy && dx && dw, MC_ERR_INVALID, "mc_causal_conv1d_bwd: x, w, dy, dx, dw required");
  MC_CHECK(workspace && workspace_bytes >= mc_causal_conv1d_bwd_workspace_bytes(batch, dim, seqlen, K),
           MC_ERR_WORKSPACE, "mc_causal_conv1d_bwd: workspace too small");
  float* part = reinterpret_cast<float*>(workspace);
  const int V = dtype == MC_DTYPE_F32 ? 4 : 8;
  const int vec = seqlen % V == 0 && conv1d_vec_ok(x, x_bs, x_ds, V) && conv1d_vec_ok(dy, dy_bs, dy_ds, V) &&
                          conv1d_vec_ok(dx, dx_bs, dx_ds, V) ? V : 1;
  const int per = conv1d_items_per_slice(batch, seqlen, vec, (vec > 1 && K == 4) ? 63 : 64);
  const int total = batch * ((seqlen + vec - 1) / vec);
  const int nslice = (total + per - 1) / per;
  const dim3 grid((unsigned)((dim + 3) / 4), (unsigned)nslice);
  MC_DISPATCH_T(dtype, MC_DISPATCH_VEC(vec, if constexpr (VEC == 1 || VEC == ElemTraits<T>::kVec) {
    bool done = false;
    if constexpr (VEC > 1) {
      if (K == 4) {   // Mamba's d_conv on vector rows: halo g from the neighbouring lane
        hipLaunchKernelGGL((conv1d_bwd_halo_kernel<T, VEC>), grid, dim3(256), 0, s, batch, dim, seqlen, (const T*)x,
                           x_bs, x_ds, w, bias, silu, (const T*)dy, dy_bs, dy_ds, (T*)dx, dx_bs, dx_ds, per, part);
        done = true;
      }
    }
    if (done) {
    } else if (K == 4)   // taps unrolled at compile time
      hipLaunchKernelGGL((conv1d_bwd_kernel<T, VEC, 4>), grid, dim3(256), 0, s, batch, dim, seqlen, K, (const T*)x,
                         x_bs, x_ds, w, bias, silu, (const T*)dy, dy_bs, dy_ds, (T*)dx, dx_bs, dx_ds, per, part);
    else
      hipLaunchKernelGGL((conv1d_bwd_kernel<T, VEC, 0>), grid, dim3(256), 0, s, batch, dim, seqlen, K, (const T*)x,
                         x_bs, x_ds, w, bias, silu, (const T*)dy, dy_bs, dy_ds, (T*)dx, dx_bs, dx_ds, per, part);
  }));
  const int n = dim * (K + 1);
  hipLaunchKernelGGL(conv1d_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, s, part, nslice, dim, K, dw, dbias);
  return check_launch("mc_causal_conv1d_bwd");
}

extern "C" size_t mc_grad_colsum_workspace_bytes(int32_t rows, int32_t cols) {
  (void)rows;
  return (size_t)kGradSlices * (size_t)std::max(cols, 0) * sizeof(float);
}

static int grad_slices(int rows) { return std::max(1, std::min(kGradSlices, (rows + 31) / 32)); }

extern "C" int mc_gelu_bwd(int32_t rows, int32_t cols, int32_t dtype, const void* h, int64_t ldh, const void* ga,
                           int64_t ldga, void* gh, int64_t ldgh, float* dbias, void* workspace,
                           size_t workspace_bytes, void* stream) {
  MC_CHECK(dtype >= MC_DTYPE_F32 && dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_gelu_bwd: bad dtype");
  const int V = dtype == MC_DTYPE_F32 ? 4 : 8;
  MC_CHECK(rows >= 0 && cols > 0 && cols % V == 0, MC_ERR_SHAPE, "mc_gelu_bwd: cols must be a multiple of %d", V);
  if (rows == 0) {
    if (dbias) (void)hipMemsetAsync(dbias, 0, (size_t)cols * 4, (hipStream_t)stream);
    return MC_OK;
  }
  MC_CHECK(h && ga && gh && dbias, MC_ERR_INVALID, "mc_gelu_bwd: h, ga, gh, dbias required");
  MC_CHECK(aligned16(h) && aligned16(ga) && aligned16(gh) && ldh % V == 0 && ldga % V == 0 && ldgh % V == 0,
           MC_ERR_SHAPE, "mc_gelu_bwd: rows must be 16-B aligned");
  MC_CHECK(workspace && workspace_bytes >= mc_grad_colsum_workspace_bytes(rows, cols), MC_ERR_WORKSPACE,
           "mc_gelu_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  float* part = reinterpret_cast<float*>(workspace);
  const int ns = grad_slices(rows);
  const dim3 grid((unsigned)((cols / V + 63) / 64), (unsigned)ns);
  MC_DISPATCH_T(dtype, hipLaunchKernelGGL((gelu_bwd_colsum_kernel<T>), grid, dim3(256), 0, s, rows, cols,
                                          (const T*)h, ldh, (const T*)ga, ldga, (T*)gh, ldgh, part));
  hipLaunchKernelGGL(colsum_slices_kernel, dim3((cols + 31) / 32), dim3(256), 0, s, part, ns, cols, dbias);
  return check_launch("mc_gelu_bwd");
}

extern "C" int mc_qkv_grad_pack(const mc_qkv_pack_params* p, void* stream) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_qkv_grad_pack: null params");
  MC_CHECK(p->dtype >= MC_DTYPE_F32 && p->dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_qkv_grad_pack: bad dtype");
  const int V = p->dtype == MC_DTYPE_F32 ? 4 : 8;
  MC_CHECK(p->batch >= 0 && p->seq >= 0 && p->heads > 0 && p->head_dim > 0 && p->head_dim % V == 0, MC_ERR_SHAPE,
           "mc_qkv_grad_pack: head_dim must be a multiple of %d", V);
  const int rows = p->batch * p->seq, cols = 3 * p->heads * p->head_dim;
  if (rows == 0) {
    if (p->dbias) (void)hipMemsetAsync(p->dbias, 0, (size_t)cols * 4, (hipStream_t)stream);
    return MC_OK;
  }
  QkvSrc src;
  for (int i = 0; i < 3; ++i) {
    MC_CHECK(p->src[i] && aligned16(p->src[i]) && p->sb[i] % V == 0 && p->sn[i] % V == 0 && p->sh[i] % V == 0,
             MC_ERR_SHAPE, "mc_qkv_grad_pack: source %d must be non-null with 16-B aligned head rows", i);
    src.p[i] = p->src[i]; src.sb[i] = p->sb[i]; src.sn[i] = p->sn[i]; src.sh[i] = p->sh[i];
  }
  MC_CHECK(p->out && aligned16(p->out) && p->ld_out % V == 0 && p->ld_out >= cols, MC_ERR_SHAPE,
           "mc_qkv_grad_pack: out must be 16-B aligned with ld_out >= 3 * heads * head_dim");
  MC_CHECK(!p->dbias || (p->workspace && p->workspace_bytes >= mc_grad_colsum_workspace_bytes(rows, cols)),
           MC_ERR_WORKSPACE, "mc_qkv_grad_pack: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  float* part = p->dbias ? reinterpret_cast<float*>(p->workspace) : nullptr;
  const int ns = grad_slices(rows);
  const dim3 grid((unsigned)((cols / V + 63) / 64), (unsigned)ns);
  MC_DISPATCH_T(p->dtype, hipLaunchKernelGGL((qkv_pack_colsum_kernel<T>), grid, dim3(256), 0, s, p->batch, p->seq,
                                             p->heads, p->head_dim, src, (T*)p->out, p->ld_out, part));
  if (p->dbias)
    hipLaunchKernelGGL(colsum_slices_kernel, dim3((cols + 31) / 32), dim3(256), 0, s, part, ns, cols, p->dbias);
  return check_launch("mc_qkv_grad_pack");
}

extern "C" int mc_patch_im2col(int32_t batch, int32_t C, int32_t H, int32_t W, int32_t P, int32_t dtype,
                               const void* img, void* patches, void* stream) {
  MC_CHECK(dtype >= MC_DTYPE_F32 && dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_patch_im2col: bad dtype");
  MC_CHECK(batch >= 0 && C > 0 && P > 0 && H % P == 0 && W % P == 0, MC_ERR_SHAPE,
           "mc_patch_im2col: H and W must be multiples of P");
  if (batch == 0) return MC_OK;
  MC_CHECK(img && patches, MC_ERR_INVALID, "mc_patch_im2col: null pointer");
  const int64_t total = (int64_t)batch * C * H * W;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 65536);
  MC_DISPATCH_T(dtype, hipLaunchKernelGGL((im2col_kernel<T>), dim3(grid), dim3(256), 0, (hipStream_t)stream, batch,
                                          C, H, W, P, (const T*)img, (T*)patches));
  return check_launch("mc_patch_im2col");
}

// ------------------------------------------------------------------ achievable HBM rate (measurement)
// float4 streaming copy: each thread moves kU 16-B vectors per pass (loads first, then stores, so
// kU loads are in flight per lane); up to 65536 blocks (tools/ubench/hbm_rw.hip: the larger grid
// streams fastest, 5.85 TB/s at 2 GiB vs 5.1 at 1024 blocks).
namespace {
constexpr int kCopyU = 4;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void stream_copy_kernel(const u32x4_t* __restrict__ src, u32x4_t* __restrict__ dst,
                                                          int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256 * kCopyU;
  for (int64_t base = (int64_t)blockIdx.x * 256 * kCopyU + threadIdx.x; base < n16; base += stride) {
    u32x4_t v[kCopyU];
#pragma unroll
    for (int k = 0; k < kCopyU; ++k) {
      const int64_t i = base + (int64_t)k * 256;
      v[k] = i < n16 ? __builtin_nontemporal_load(src + i) : u32x4_t{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int k = 0; k < kCopyU; ++k) {
      const int64_t i = base + (int64_t)k * 256;
      if (i < n16) __builtin_nontemporal_store(v[k], dst + i);
    }
  }
}
}  // namespace

extern "C" int mc_stream_copy(const void* src, void* dst, size_t nbytes, void* stream) {
  MC_CHECK(nbytes % 16 == 0 && aligned16(src) && aligned16(dst), MC_ERR_SHAPE,
           "mc_stream_copy: 16-B aligned buffers and a multiple of 16 bytes required");
  if (nbytes == 0) return MC_OK;
  const int64_t n16 = (int64_t)(nbytes / 16);
  const int grid = (int)std::min<int64_t>((n16 + 256 * kCopyU - 1) / (256 * kCopyU), 65536);
  hipLaunchKernelGGL(stream_copy_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const u32x4_t*>(src), reinterpret_cast<u32x4_t*>(dst), n16);
  return check_launch("mc_stream_copy");
}

// ---------------------------------------------------------------------------- many fp32 -> 16-bit casts, one launch
namespace {
template <typename TO>
__global__ __launch_bounds__(256) void cast_many_kernel(const mc_cast_chunk* __restrict__ chunks, TO* __restrict__ base) {
  const mc_cast_chunk c = chunks[blockIdx.x];
  TO* __restrict__ dst = base + c.dst_off;
  const bool vec = ((reinterpret_cast<uintptr_t>(c.src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0 && (c.n & 7) == 0;
  if (vec) {
    for (int64_t i = 8 * (int64_t)threadIdx.x; i < c.n; i += 8 * 256) {
      const float4 a = *reinterpret_cast<const float4*>(c.src + i);
      const float4 b = *reinterpret_cast<const float4*>(c.src + i + 4);
      const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      *reinterpret_cast<uint4*>(dst + i) = pack_f<TO>(v);
    }
  } else {
    for (int64_t i = threadIdx.x; i < c.n; i += 256) dst[i] = from_f<TO>(c.src[i]);
  }
}
}  // namespace

extern "C" int mc_cast_f32_many(int32_t n_chunks, const mc_cast_chunk* chunks, void* dst_base, int32_t dst_dtype,
                                void* stream) {
  MC_CHECK(n_chunks >= 0 && (n_chunks == 0 || (chunks && dst_base)), MC_ERR_INVALID, "mc_cast_f32_many: bad chunk table");
  MC_CHECK(dst_dtype == MC_DTYPE_BF16 || dst_dtype == MC_DTYPE_F16, MC_ERR_DTYPE,
           "mc_cast_f32_many: dst dtype %d (bf16 / f16 only)", dst_dtype);
  if (n_chunks == 0) return MC_OK;
  if (dst_dtype == MC_DTYPE_BF16)
    hipLaunchKernelGGL(cast_many_kernel<bf16_t>, dim3(n_chunks), dim3(256), 0, (hipStream_t)stream, chunks,
                       reinterpret_cast<bf16_t*>(dst_base));
  else
    hipLaunchKernelGGL(cast_many_kernel<f16_t>, dim3(n_chunks), dim3(256), 0, (hipStream_t)stream, chunks,
                       reinterpret_cast<f16_t*>(dst_base));
  return check_launch("mc_cast_f32_many");
}

// ---------------------------------------------------------------------------- transposed weight casts
namespace {
template <typename TO>
__global__ __launch_bounds__(256) void cast_transpose_kernel(const mc_cast_t_tile* __restrict__ tiles, TO* __restrict__ base) {
  __shared__ float tile[64][65];
  const mc_cast_t_tile t = tiles[blockIdx.x];
  // loads: thread (r = tid >> 2, a = tid & 3) reads float4 a + 4k of source row r, so the four lanes of a
  // row cover 64 contiguous bytes per instruction
  const int tid = threadIdx.x, r = tid >> 2, a = tid & 3;
  const bool full = t.rows == 64 && t.cols == 64 && (t.src_ld & 3) == 0 && (reinterpret_cast<uintptr_t>(t.src) & 15) == 0;
  if (full) {
    float4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const float4*>(t.src + (int64_t)r * t.src_ld + 4 * (a + 4 * k));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 4 * (a + 4 * k);
      tile[r][c] = v[k].x; tile[r][c + 1] = v[k].y; tile[r][c + 2] = v[k].z; tile[r][c + 3] = v[k].w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 4 * (a + 4 * k) + e;
        tile[r][c] = (r < t.rows && c < t.cols) ? t.src[(int64_t)r * t.src_ld + c] : 0.f;
      }
  }
  __syncthreads();
  // stores: output row j (= source column), 8-element groups a and a + 4 (source rows 8 g .. 8 g + 7): the
  // four lanes of a row write 64 contiguous bytes per instruction
  const int j = tid >> 2;
  TO* dst = base + t.dst_off + (int64_t)j * t.dst_ld;
  const bool vec = full && (t.dst_ld & 7) == 0 && (reinterpret_cast<uintptr_t>(base + t.dst_off) & 15) == 0;
#pragma unroll
  for (int hlf = 0; hlf < 2; ++hlf) {
    const int g = a + 4 * hlf;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = tile[8 * g + e][j];
    if (vec) {
      *reinterpret_cast<uint4*>(dst + 8 * g) = pack_f<TO>(v);
    } else if (j < t.cols) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (8 * g + e < t.rows) dst[8 * g + e] = from_f<TO>(v[e]);
    }
  }
}
}  // namespace

extern "C" int mc_cast_transpose_f32_many(int32_t n_tiles, const mc_cast_t_tile* tiles, void* dst_base, int32_t dst_dtype,
                                          void* stream) {
  MC_CHECK(n_tiles >= 0 && (n_tiles == 0 || (tiles && dst_base)), MC_ERR_INVALID, "mc_cast_transpose_f32_many: bad tile table");
  MC_CHECK(dst_dtype == MC_DTYPE_BF16 || dst_dtype == MC_DTYPE_F16, MC_ERR_DTYPE,
           "mc_cast_transpose_f32_many: dst dtype %d (bf16 / f16 only)", dst_dtype);
  if (n_tiles == 0) return MC_OK;
  if (dst_dtype == MC_DTYPE_BF16)
    hipLaunchKernelGGL(cast_transpose_kernel<bf16_t>, dim3(n_tiles), dim3(256), 0, (hipStream_t)stream, tiles,
                       reinterpret_cast<bf16_t*>(dst_base));
  else
    hipLaunchKernelGGL(cast_transpose_kernel<f16_t>, dim3(n_tiles), dim3(256), 0, (hipStream_t)stream, tiles,
                       reinterpret_cast<f16_t*>(dst_base));
  return check_launch("mc_cast_transpose_f32_many");
}

// ---------------------------------------------------------------------------- AdamW over many tensors
namespace {
__device__ __forceinline__ void adamw_elem(float& p, float& m, float& v, float g, const mc_adamw_group& h) {
  p *= h.decay;
  m = h.beta1 * m + (1.f - h.beta1) * g;
  v = h.beta2 * v + (1.f - h.beta2) * g * g;
  const float denom = sqrtf(v) / h.bc2_sqrt + h.eps;
  p -= h.step_size * m / denom;
}

__global__ __launch_bounds__(256) void adamw_kernel(const mc_adamw_chunk* __restrict__ chunks,
                                                    const mc_adamw_tensor* __restrict__ tensors, const mc_adamw_hyper hy) {
  const mc_adamw_chunk c = chunks[blockIdx.x];
  const mc_adamw_tensor t = tensors[c.tensor];
  const mc_adamw_group h = hy.group[c.group];
  float* __restrict__ p = t.p + c.off;
  float* __restrict__ m = t.m + c.off;
  float* __restrict__ v = t.v + c.off;
  const float* __restrict__ g = t.g + c.off;
  const bool vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v) |
                     reinterpret_cast<uintptr_t>(g)) & 15) == 0;
  const int64_t n4 = vec ? c.n / 4 : 0;
  for (int64_t i = threadIdx.x; i < n4; i += 256) {
    float4 pp = reinterpret_cast<float4*>(p)[i], mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    adamw_elem(pp.x, mm.x, vv.x, gg.x, h);
    adamw_elem(pp.y, mm.y, vv.y, gg.y, h);
    adamw_elem(pp.z, mm.z, vv.z, gg.z, h);
    adamw_elem(pp.w, mm.w, vv.w, gg.w, h);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  for (int64_t i = 4 * n4 + threadIdx.x; i < c.n; i += 256) {
    float pp = p[i], mm = m[i], vv = v[i];
    adamw_elem(pp, mm, vv, g[i], h);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}
}  // namespace

extern "C" int mc_adamw_step(int32_t n_chunks, const mc_adamw_chunk* chunks, const mc_adamw_tensor* tensors,
                             const mc_adamw_hyper* hyper, void* stream) {
  MC_CHECK(n_chunks >= 0 && hyper, MC_ERR_INVALID, "mc_adamw_step: bad arguments");
  MC_CHECK(hyper->n_groups >= 1 && hyper->n_groups <= MC_ADAMW_MAX_GROUPS, MC_ERR_INVALID,
           "mc_adamw_step: n_groups %d (1..%d)", hyper->n_groups, MC_ADAMW_MAX_GROUPS);
  if (n_chunks == 0) return MC_OK;
  MC_CHECK(chunks && tensors, MC_ERR_INVALID, "mc_adamw_step: null chunk / tensor table");
  hipLaunchKernelGGL(adamw_kernel, dim3(n_chunks), dim3(256), 0, (hipStream_t)stream, chunks, tensors, *hyper);
  return check_launch("mc_adamw_step");
}

// ---------------------------------------------------------------------------- split-K slab sums
namespace {
template <bool kVec>
__global__ __launch_bounds__(256) void sum_slabs_kernel(int s, int64_t n, const float* __restrict__ src, int64_t stride,
                                                        float* __restrict__ dst) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * (kVec ? 4 : 1);
  if (i0 >= n) return;
  if constexpr (kVec) {
    float4 acc = *reinterpret_cast<const float4*>(src + i0);
    for (int k = 1; k < s; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)k * stride + i0);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    *reinterpret_cast<float4*>(dst + i0) = acc;
  } else {
    float acc = src[i0];
    for (int k = 1; k < s; ++k) acc += src[(int64_t)k * stride + i0];
    dst[i0] = acc;
  }
}
}  // namespace

extern "C" int mc_sum_slabs(int32_t s, int64_t n, const float* src, int64_t slab_stride, float* dst, void* stream) {
  MC_CHECK(s >= 1 && n >= 0 && slab_stride >= n, MC_ERR_SHAPE, "mc_sum_slabs: bad shape (s %d, n %lld, stride %lld)", s,
           (long long)n, (long long)slab_stride);
  if (n == 0) return MC_OK;
  MC_CHECK(src && dst, MC_ERR_INVALID, "mc_sum_slabs: null pointer");
  const bool vec = n % 4 == 0 && slab_stride % 4 == 0 && aligned16(src) && aligned16(dst);
  const int64_t items = vec ? n / 4 : n;
  const dim3 grid((unsigned)((items + 255) / 256));
  if (vec) hipLaunchKernelGGL(sum_slabs_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, s, n, src, slab_stride, dst);
  else hipLaunchKernelGGL(sum_slabs_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, s, n, src, slab_stride, dst);
  return check_launch("mc_sum_slabs");
}

// ------------------------------------------------------------------ column sums, row L2-normalize (C-ABI)
static int colsum_slices(int rows) { return std::max(1, std::min(kGradSlices, (rows + 31) / 32)); }

extern "C" size_t mc_colsum_workspace_bytes(int32_t rows, int32_t cols) {
  return (size_t)colsum_slices(std::max(rows, 0)) * (size_t)std::max(cols, 0) * sizeof(float);
}

extern "C" int mc_colsum(int32_t rows, int32_t cols, int32_t dtype, const void* x, int64_t ld, float* out,
                         void* workspace, size_t workspace_bytes, void* stream) {
  MC_CHECK(dtype >= MC_DTYPE_F32 && dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_colsum: bad dtype");
  MC_CHECK(rows >= 0 && cols >= 0 && ld >= cols, MC_ERR_SHAPE, "mc_colsum: bad shape (rows %d, cols %d, ld %lld)",
           rows, cols, (long long)ld);
  hipStream_t s = (hipStream_t)stream;
  if (cols == 0) return MC_OK;
  MC_CHECK(out, MC_ERR_INVALID, "mc_colsum: null output");
  if (rows == 0) {
    (void)hipMemsetAsync(out, 0, (size_t)cols * 4, s);
    return check_launch("mc_colsum");
  }
  MC_CHECK(x && workspace && workspace_bytes >= mc_colsum_workspace_bytes(rows, cols), MC_ERR_WORKSPACE,
           "mc_colsum: x and a workspace of mc_colsum_workspace_bytes required");
  float* part = reinterpret_cast<float*>(workspace);
  const int ns = colsum_slices(rows);
  const int V = dtype == MC_DTYPE_F32 ? 4 : 8;
  const bool vec = cols % V == 0 && ld % V == 0 && aligned16(x);
  MC_DISPATCH_T(dtype, {
    if (vec)
      hipLaunchKernelGGL((colsum_rows_kernel<T, ElemTraits<T>::kVec>), dim3((unsigned)((cols / V + 63) / 64), ns),
                         dim3(256), 0, s, rows, cols, (const T*)x, ld, part);
    else
      hipLaunchKernelGGL((colsum_rows_kernel<T, 1>), dim3((unsigned)((cols + 63) / 64), ns), dim3(256), 0, s, rows,
                         cols, (const T*)x, ld, part);
  });
  hipLaunchKernelGGL(colsum_slices_kernel, dim3((cols + 31) / 32), dim3(256), 0, s, part, ns, cols, out);
  return check_launch("mc_colsum");
}

extern "C" int mc_l2norm_fwd(int32_t rows, int32_t cols, int32_t dtype, const void* x, int64_t ldx, float eps,
                             float* y, int64_t ldy, float* norm, void* stream) {
  MC_CHECK(dtype >= MC_DTYPE_F32 && dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_l2norm_fwd: bad dtype");
  MC_CHECK(rows >= 0 && cols > 0 && ldx >= cols && ldy >= cols, MC_ERR_SHAPE, "mc_l2norm_fwd: bad shape");
  if (rows == 0) return MC_OK;
  MC_CHECK(x && y && norm, MC_ERR_INVALID, "mc_l2norm_fwd: x, y, norm required");
  MC_DISPATCH_T(dtype, hipLaunchKernelGGL((l2norm_fwd_kernel<T>), dim3((rows + 3) / 4), dim3(256), 0,
                                          (hipStream_t)stream, rows, cols, (const T*)x, ldx, eps, y, ldy, norm));
  return check_launch("mc_l2norm_fwd");
}

extern "C" int mc_l2norm_bwd(int32_t rows, int32_t cols, int32_t dtype, const void* x, int64_t ldx, const float* norm,
                             float eps, const float* g, int64_t ldg, void* dx, int64_t lddx, void* stream) {
  MC_CHECK(dtype >= MC_DTYPE_F32 && dtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "mc_l2norm_bwd: bad dtype");
  MC_CHECK(rows >= 0 && cols > 0 && ldx >= cols && ldg >= cols && lddx >= cols, MC_ERR_SHAPE,
           "mc_l2norm_bwd: bad shape");
  if (rows == 0) return MC_OK;
  MC_CHECK(x && norm && g && dx, MC_ERR_INVALID, "mc_l2norm_bwd: x, norm, g, dx required");
  MC_DISPATCH_T(dtype, hipLaunchKernelGGL((l2norm_bwd_kernel<T>), dim3((rows + 3) / 4), dim3(256), 0,
                                          (hipStream_t)stream, rows, cols, (const T*)x, ldx, norm, eps, g, ldg,
                                          (T*)dx, lddx));
  return check_launch("mc_l2norm_bwd");
}

// out[c] = sum over k of part[k][c], in a fixed order (colsum_slices_kernel): the fold of per-tile /
// per-slice column partials (mc_linear's GELU' epilogue writes one row per 256-token tile).
extern "C" int mc_colsum_fold(int32_t nslices, int32_t cols, const float* part, float* out, void* stream) {
  MC_CHECK(nslices >= 1 && cols >= 0, MC_ERR_SHAPE, "mc_colsum_fold: bad shape (nslices %d, cols %d)", nslices, cols);
  if (cols == 0) return MC_OK;
  MC_CHECK(part && out, MC_ERR_INVALID, "mc_colsum_fold: null pointer");
  hipLaunchKernelGGL(colsum_slices_kernel, dim3((cols + 31) / 32), dim3(256), 0, (hipStream_t)stream, part, nslices, cols,
                     out);
  return check_launch("mc_colsum_fold");
}
