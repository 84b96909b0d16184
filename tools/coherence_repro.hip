// coherence_repro.hip -- standalone test (no torch): do reductions whose partial results pass through
// global memory read exactly what was written, while another stream (its own hardware queue) runs
// kernels?  (the two-stream training step differs from run to run in a few reductions'
// results; one hardware queue, or a host wait after every launch, makes it deterministic.)
//
// Per iteration the data changes (seed it), so a stale read of an earlier iteration's partials shows.
// Stream A:
//   fill      x[i] = f(i, it)                                    (n floats)
//   two-kernel reduction: partial_kernel writes per-block column partials to a slab,
//                         combine_kernel sums the slab in a fixed order (the scan backward's pattern)
//   last-block reduction: one kernel; blocks write partials, __threadfence, atomicAdd a ticket; the
//                         last block sums every partial in a fixed order (torch's global reduce)
//   check     both results vs a host-side expected sum computed from f (exact: integer-valued data)
// Stream B (mode "load"): a long streaming kernel plus short launches, re-issued every iteration.
//   hipcc --offload-arch=gfx950 -O3 tools/coherence_repro.hip -o tools/coherence_repro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

constexpr int kRows = 4096, kCols = 1536, kBlocks = 512;   // rows split over kBlocks blocks

__host__ __device__ inline float f(int r, int c, int it) { return (float)(((r * 131 + c * 7 + it * 977) % 61) - 30); }

__global__ void fill(float* x, int it) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kRows * kCols; i += gridDim.x * blockDim.x)
    x[i] = f(i / kCols, i % kCols, it);
}

// two kernels: per-block column partials -> slab, then a fixed-order combine
__global__ void partial_kernel(const float* x, float* slab) {
  const int rpb = kRows / kBlocks;
  for (int c = threadIdx.x; c < kCols; c += blockDim.x) {
    float s = 0.f;
    for (int r = blockIdx.x * rpb; r < (blockIdx.x + 1) * rpb; ++r) s += x[(size_t)r * kCols + c];
    slab[(size_t)blockIdx.x * kCols + c] = s;
  }
}
__global__ void combine_kernel(const float* slab, float* out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= kCols) return;
  float s = 0.f;
  for (int b = 0; b < kBlocks; ++b) s += slab[(size_t)b * kCols + c];
  out[c] = s;
}

// one kernel, last block combines (fence + ticket)
__global__ void lastblock_kernel(const float* x, float* slab, unsigned* ticket, float* out) {
  const int rpb = kRows / kBlocks;
  for (int c = threadIdx.x; c < kCols; c += blockDim.x) {
    float s = 0.f;
    for (int r = blockIdx.x * rpb; r < (blockIdx.x + 1) * rpb; ++r) s += x[(size_t)r * kCols + c];
    slab[(size_t)blockIdx.x * kCols + c] = s;
  }
  __threadfence();
  __shared__ bool last;
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == kBlocks - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  for (int c = threadIdx.x; c < kCols; c += blockDim.x) {
    float s = 0.f;
    for (int b = 0; b < kBlocks; ++b) s += slab[(size_t)b * kCols + c];
    out[c] = s;
  }
  if (threadIdx.x == 0) *ticket = 0;
}

// torch's global reduce: grid (gx, 2), the two CTAs of a column block each sum half the rows into a
// staging buffer, fence, bump a per-column-block semaphore (zeroed by a memset before every launch);
// the second to arrive adds both partials
__global__ void torchlike_reduce(const float* x, float* staging, unsigned* sem, float* out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int half = kRows / 2;
  float s = 0.f;
  if (c < kCols)
    for (int r = blockIdx.y * half; r < (blockIdx.y + 1) * half; ++r) s += x[(size_t)r * kCols + c];
  if (c < kCols) staging[(size_t)blockIdx.y * kCols + c] = s;
  __threadfence();
  __shared__ bool last;
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(&sem[blockIdx.x], 1u) == 1u;
  __syncthreads();
  if (!last) return;
  __threadfence();
  if (c < kCols) out[c] = staging[c] + staging[kCols + c];
}

__global__ void check(const float* o1, const float* o2, const float* expect, unsigned long long* bad) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= kCols) return;
  if (o1[c] != expect[c]) atomicAdd(bad, 1ull);
  if (o2[c] != expect[c]) atomicAdd(bad + 1, 1ull);
}

__global__ void stream_load(float* y, size_t n, int k) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = y[i] * 0.999f + (float)k;
}

// a load kernel whose waves issue device-scope fences (acquire part: L2 invalidate) in a loop, as a
// reduction's "last block" handshake does (torch's global reduce, __threadfence + ticket)
__global__ void fence_load(float* y, int reps) {
  float v = y[blockIdx.x * blockDim.x + threadIdx.x];
  for (int r = 0; r < reps; ++r) {
    v = v * 0.999f + 1.f;
    // the device-scope fence __threadfence() emits (release: L2 write-back, acquire: L2 invalidate),
    // kept inside the loop (the compiler hoists the builtin out of it)
    asm volatile("buffer_wbl2 sc1\n\ts_waitcnt vmcnt(0)\n\tbuffer_inv sc1" : "+v"(v) :: "memory");
  }
  y[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 300;
  float *x, *slab1, *slab2, *o1, *o2, *ex, *ly;
  unsigned* ticket;
  unsigned long long* bad;
  const size_t ln = (size_t)256 << 20;   // 1 GB of load traffic per pass
  CK(hipMalloc(&x, (size_t)kRows * kCols * 4));
  CK(hipMalloc(&slab1, (size_t)kBlocks * kCols * 4));
  CK(hipMalloc(&slab2, (size_t)kBlocks * kCols * 4));
  CK(hipMalloc(&o1, kCols * 4));
  CK(hipMalloc(&o2, kCols * 4));
  CK(hipMalloc(&ex, (size_t)iters * kCols * 4));
  CK(hipMalloc(&ly, ln * 4));
  CK(hipMalloc(&ticket, 4));
  CK(hipMalloc(&bad, 16));
  CK(hipMemset(ticket, 0, 4));
  CK(hipMemset(ly, 0, ln * 4));
  // expected column sums (exact: small integers)
  std::vector<float> h((size_t)iters * kCols);
  for (int it = 0; it < iters; ++it)
    for (int c = 0; c < kCols; ++c) {
      double s = 0;
      for (int r = 0; r < kRows; ++r) s += f(r, c, it);
      h[(size_t)it * kCols + c] = (float)s;
    }
  CK(hipMemcpy(ex, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  unsigned* sem;
  float* stg;
  CK(hipMalloc(&sem, 64 * 4));
  CK(hipMalloc(&stg, 2 * kCols * 4));
  const char* names[] = {"no_load", "load_stream_b", "fence_load_stream_b", "torchlike_null_stream_no_load",
                         "torchlike_null_stream_load", "torchlike_stream_a_load"};
  for (int mode = 0; mode < 6; ++mode) {
    if (mode >= 3) {
      hipStream_t sa = mode == 5 ? a : (hipStream_t)0;
      CK(hipDeviceSynchronize());
      CK(hipMemset(bad, 0, 16));
      for (int it = 0; it < iters; ++it) {
        if (mode != 3) {
          hipLaunchKernelGGL(stream_load, dim3(1024), dim3(256), 0, b, ly, ln, it);
          for (int k = 0; k < 8; ++k) hipLaunchKernelGGL(stream_load, dim3(32), dim3(256), 0, b, ly, (size_t)1 << 16, k);
        }
        hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, sa, x, it);
        CK(hipMemsetAsync(sem, 0, 64 * 4, sa));
        hipLaunchKernelGGL(torchlike_reduce, dim3((kCols + 255) / 256, 2), dim3(256), 0, sa, x, stg, sem, o2);
        hipLaunchKernelGGL(check, dim3((kCols + 255) / 256), dim3(256), 0, sa, o2, o2, ex + (size_t)it * kCols, bad);
      }
      CK(hipDeviceSynchronize());
      unsigned long long hb[2];
      CK(hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost));
      printf("{\"mode\": \"%s\", \"iters\": %d, \"bad\": %llu}\n", names[mode], iters, hb[0]);
      fflush(stdout);
      continue;
    }
    CK(hipMemset(bad, 0, 16));
    for (int it = 0; it < iters; ++it) {
      if (mode == 1) {
        hipLaunchKernelGGL(stream_load, dim3(1024), dim3(256), 0, b, ly, ln, it);
        for (int k = 0; k < 8; ++k) hipLaunchKernelGGL(stream_load, dim3(32), dim3(256), 0, b, ly, (size_t)1 << 16, k);
      }
      if (mode == 2) hipLaunchKernelGGL(fence_load, dim3(256), dim3(256), 0, b, ly, 2000);
      hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, a, x, it);
      hipLaunchKernelGGL(partial_kernel, dim3(kBlocks), dim3(256), 0, a, x, slab1);
      hipLaunchKernelGGL(combine_kernel, dim3((kCols + 255) / 256), dim3(256), 0, a, slab1, o1);
      hipLaunchKernelGGL(lastblock_kernel, dim3(kBlocks), dim3(256), 0, a, x, slab2, ticket, o2);
      hipLaunchKernelGGL(check, dim3((kCols + 255) / 256), dim3(256), 0, a, o1, o2, ex + (size_t)it * kCols, bad);
    }
    CK(hipDeviceSynchronize());
    unsigned long long hb[2];
    CK(hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost));
    printf("{\"mode\": \"%s\", \"iters\": %d, \"two_kernel_bad\": %llu, \"last_block_bad\": %llu}\n",
           names[mode], iters, hb[0], hb[1]);
    fflush(stdout);
  }
  return 0;
}
