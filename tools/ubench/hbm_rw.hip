// HBM streaming rates on MI355X: write-only (fill), read-only (sum) and copy, 16-B vectors,
// plain and non-temporal stores, over a 268 MB buffer (the C5 fp32 logit matrix, 8192^2 x 4 B)
// and a 2 GiB one.  Bounds the C5 similarity kernel, whose HBM side is a pure write stream.
//   hipcc --offload-arch=gfx950 -O3 hbm_rw.hip -o hbm_rw
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef unsigned u4 __attribute__((ext_vector_type(4)));

template <bool kNT>
__global__ __launch_bounds__(256) void fill(u4* __restrict__ d, size_t n, unsigned v) {
  const size_t stride = (size_t)gridDim.x * 256 * 4;
  for (size_t b = (size_t)blockIdx.x * 256 * 4 + threadIdx.x; b < n; b += stride)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t i = b + (size_t)k * 256;
      if (i < n) {
        const u4 x = {v, v + 1, v + 2, (unsigned)i};
        if (kNT) __builtin_nontemporal_store(x, d + i); else d[i] = x;
      }
    }
}
__global__ __launch_bounds__(256) void sum(const u4* __restrict__ s, size_t n, unsigned* out) {
  const size_t stride = (size_t)gridDim.x * 256 * 4;
  unsigned acc = 0;
  for (size_t b = (size_t)blockIdx.x * 256 * 4 + threadIdx.x; b < n; b += stride) {
    u4 x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { const size_t i = b + (size_t)k * 256; x[k] = i < n ? __builtin_nontemporal_load(s + i) : u4{0, 0, 0, 0}; }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += x[k].x ^ x[k].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ __launch_bounds__(256) void copy(const u4* __restrict__ s, u4* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256 * 4;
  for (size_t b = (size_t)blockIdx.x * 256 * 4 + threadIdx.x; b < n; b += stride) {
    u4 x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { const size_t i = b + (size_t)k * 256; x[k] = i < n ? __builtin_nontemporal_load(s + i) : u4{0, 0, 0, 0}; }
#pragma unroll
    for (int k = 0; k < 4; ++k) { const size_t i = b + (size_t)k * 256; if (i < n) __builtin_nontemporal_store(x[k], d + i); }
  }
}

int main() {
  const size_t sizes[2] = {(size_t)8192 * 8192 * 4, (size_t)2 << 30};
  u4 *a, *b; unsigned* o;
  hipMalloc(&a, sizes[1]); hipMalloc(&b, sizes[1]); hipMalloc(&o, 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int si = 0; si < 2; ++si) {
    const size_t bytes = sizes[si], n = bytes / 16;
    for (int grid : {1024, 2048, 8192, 32768}) {
      float ms;
      auto time = [&](auto fn) { fn(); fn(); hipEventRecord(e0); for (int it = 0; it < 10; ++it) fn(); hipEventRecord(e1);
                                 hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1); return ms / 10; };
      const float tf = time([&] { hipLaunchKernelGGL(fill<false>, grid, 256, 0, 0, a, n, 7u); });
      const float tn = time([&] { hipLaunchKernelGGL(fill<true>, grid, 256, 0, 0, a, n, 7u); });
      const float tr = time([&] { hipLaunchKernelGGL(sum, grid, 256, 0, 0, a, n, o); });
      const float tc = time([&] { hipLaunchKernelGGL(copy, grid, 256, 0, 0, a, b, n); });
      printf("%5.0f MB grid %5d: write %.0f GB/s (nt %.0f), read %.0f GB/s, copy %.0f GB/s (r+w)\n", bytes / 1e6, grid,
             bytes / tf / 1e6, bytes / tn / 1e6, bytes / tr / 1e6, 2 * bytes / tc / 1e6);
    }
  }
  return 0;
}
