// gelu.hip -- microbenchmark (no torch) of the ViT MLP activation passes at the C2 shape
// (rows = 256 * 197 = 50432, cols = 3072, bf16): where does gelu_bwd_colsum's time go?
//   bwd modes: 0 exact erff + exp (the shipped math), 1 no math (gh = ga * h: the memory floor),
//              2 erfc-based Phi with one shared exp (fractional error ~1e-7)
//   rows in flight per thread: 2 (shipped) or 4
//   fwd: y = h * Phi(h), exact erff (mode 0) / shared-exp form (mode 2) / y = h (mode 1)
//   hipcc --offload-arch=gfx950 -O3 -I mamba-clip_amd/csrc tools/ubench/gelu.hip -o /tmp/gelu_ub
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mc_common.h"

using namespace mc;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

__device__ __forceinline__ float phi_exact(float x) { return 0.5f * (1.f + erff(x * 0.70710678118654752f)); }

// Phi(x) and pdf(x) from one exp: for z = |x|/sqrt2, erfc(z) = t * exp(-z^2 + P(t)), t = 1/(1 + z/2)
// (Chebyshev fit, fractional error < 1.2e-7 for all z >= 0); exp(-z^2 + P) = exp(-x^2/2) * exp(P).
__device__ __forceinline__ void phi_pdf_fast(float x, float& phi, float& pdf) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = fast_rcp(fmaf(0.5f, z, 1.f));
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
  const float e = fast_exp2(-0.5f * x * x * kLog2e);        // exp(-x^2/2)
  const float erfc_z = t * e * fast_exp2(p * kLog2e);
  const float half = 0.5f * erfc_z;                          // Phi(-|x|)
  phi = x < 0.f ? half : 1.f - half;
  pdf = 0.39894228040143268f * e;
}

template <int MODE>
__device__ __forceinline__ float gelu_grad(float x) {
  if constexpr (MODE == 0) {
    const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
    return fmaf(x, pdf, phi_exact(x));
  } else if constexpr (MODE == 1) {
    return x;
  } else {
    float phi, pdf;
    phi_pdf_fast(x, phi, pdf);
    return fmaf(x, pdf, phi);
  }
}
template <int MODE>
__device__ __forceinline__ float gelu_fwd(float x) {
  if constexpr (MODE == 0) return x * phi_exact(x);
  else if constexpr (MODE == 1) return x;
  else { float phi, pdf; phi_pdf_fast(x, phi, pdf); return x * phi; }
}

template <int MODE, int RPI>
__global__ __launch_bounds__(256) void bwd_kernel(int rows, int cols, const bf16_t* __restrict__ h, const bf16_t* __restrict__ ga,
                                                  bf16_t* __restrict__ gh, float* __restrict__ part) {
  constexpr int V = 8;
  __shared__ float red[3][64 * V];
  const int lane = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int cv = blockIdx.x * 64 + lane;
  const int per = (rows + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
  float acc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = 0.f;
  for (int r = r0 + rl; r < r1; r += 4 * RPI) {
    uint4 hq[RPI], gq[RPI];
#pragma unroll
    for (int k = 0; k < RPI; ++k) {
      const int rr = min(r + 4 * k, r1 - 1);
      hq[k] = ld16(h + (int64_t)rr * cols + cv * V);
      gq[k] = ld16(ga + (int64_t)rr * cols + cv * V);
    }
#pragma unroll
    for (int k = 0; k < RPI; ++k) {
      float o[V];
#pragma unroll
      for (int e = 0; e < V; ++e) o[e] = elem_f<bf16_t>(gq[k], e) * gelu_grad<MODE>(elem_f<bf16_t>(hq[k], e));
      const uint4 oq = pack_f<bf16_t>(o);
      if (r + 4 * k < r1) {
        st16(gh + (int64_t)(r + 4 * k) * cols + cv * V, oq);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += elem_f<bf16_t>(oq, e);
      }
    }
  }
  if (rl > 0) {
#pragma unroll
    for (int e = 0; e < V; ++e) red[rl - 1][lane * V + e] = acc[e];
  }
  __syncthreads();
  if (rl == 0) {
#pragma unroll
    for (int e = 0; e < V; ++e)
      part[(int64_t)blockIdx.y * cols + cv * V + e] = ((acc[e] + red[0][lane * V + e]) + red[1][lane * V + e]) + red[2][lane * V + e];
  }
}

// flat elementwise forward: grid-stride over 16-B vectors, UNR vectors in flight per thread
template <int MODE, int UNR>
__global__ __launch_bounds__(256) void fwd_kernel(int64_t nvec, const bf16_t* __restrict__ h, bf16_t* __restrict__ y) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += stride * UNR) {
    uint4 q[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) q[k] = i + k * stride < nvec ? ld16(h + (i + k * stride) * 8) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = gelu_fwd<MODE>(elem_f<bf16_t>(q[k], e));
      if (i + k * stride < nvec) st16(y + (i + k * stride) * 8, pack_f<bf16_t>(o));
    }
  }
}

__global__ void init_kernel(int64_t n, bf16_t* p, unsigned seed, float scale) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    unsigned s = (unsigned)i * 2654435761u ^ seed;
    s ^= s >> 13; s *= 0x5bd1e995u; s ^= s >> 15;
    const float u1 = ((s & 0xffffu) + 0.5f) / 65536.f, u2 = ((s >> 16) + 0.5f) / 65536.f;
    p[i] = (bf16_t)(scale * sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2));
  }
}

template <typename F>
float time_it(F f, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / iters;
}

int main() {
  const int rows = 50432, cols = 3072, ns = 512;
  const int64_t n = (int64_t)rows * cols;
  bf16_t *h, *ga, *gh;
  float* part;
  CK(hipMalloc(&h, n * 2)); CK(hipMalloc(&ga, n * 2)); CK(hipMalloc(&gh, n * 2));
  CK(hipMalloc(&part, (size_t)ns * cols * 4));
  hipLaunchKernelGGL(init_kernel, dim3(4096), dim3(256), 0, 0, n, h, 1u, 1.f);
  hipLaunchKernelGGL(init_kernel, dim3(4096), dim3(256), 0, 0, n, ga, 7u, 1e-3f);
  CK(hipDeviceSynchronize());
  const double bwd_bytes = 3.0 * n * 2, fwd_bytes = 2.0 * n * 2;
  const dim3 g(cols / 8 / 64, ns);
#define BWD(M, R) { float us = time_it([&] { hipLaunchKernelGGL((bwd_kernel<M, R>), g, dim3(256), 0, 0, rows, cols, h, ga, gh, part); }, 20); \
    printf("{\"pass\": \"bwd\", \"mode\": %d, \"rows_in_flight\": %d, \"us\": %.1f, \"GBps\": %.0f}\n", M, R, us, bwd_bytes / us / 1e3); }
  BWD(0, 2) BWD(1, 2) BWD(2, 2) BWD(0, 4) BWD(1, 4) BWD(2, 4)
  const int64_t nvec = n / 8;
#define FWD(M, U, G) { float us = time_it([&] { hipLaunchKernelGGL((fwd_kernel<M, U>), dim3(G), dim3(256), 0, 0, nvec, h, gh); }, 20); \
    printf("{\"pass\": \"fwd\", \"mode\": %d, \"unroll\": %d, \"grid\": %d, \"us\": %.1f, \"GBps\": %.0f}\n", M, U, G, us, fwd_bytes / us / 1e3); }
  FWD(0, 2, 4096) FWD(1, 2, 4096) FWD(2, 2, 4096) FWD(0, 4, 2048) FWD(2, 4, 2048) FWD(2, 4, 8192) FWD(1, 4, 2048)
  return 0;
}
