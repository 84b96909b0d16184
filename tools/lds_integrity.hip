// lds_integrity.hip -- standalone test (no torch): does a workgroup's LDS (and its VGPRs) keep what the
// workgroup wrote while kernels of a second stream -- its own hardware queue -- compete for the CUs?
// (the two-stream training step's run-to-run differences sit in results that pass through
// LDS -- the scan backward's dA / dbias, not its register-only dD -- and vanish with one hardware queue.)
//
// checker (stream A): every workgroup fills 64 KB of LDS with a pattern of (workgroup, word) and keeps
// a register copy of its words, then re-reads and compares them `rounds` times with some VALU work in
// between; any difference is counted (LDS vs expected, and register vs expected separately).
// load (stream B): kernels that use 96 KB of LDS each and overwrite it continuously, many workgroups.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_integrity.hip -o tools/lds_integrity
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

constexpr int kWords = 16384;   // 64 KB

__device__ __forceinline__ unsigned pat(unsigned wg, unsigned i, unsigned seed) { return (wg * 2654435761u) ^ (i * 40503u) ^ seed; }

__global__ __launch_bounds__(256) void checker(int rounds, unsigned seed, unsigned long long* bad) {
  __shared__ unsigned lds[kWords];
  const unsigned wg = blockIdx.x;
  unsigned reg[kWords / 256];
#pragma unroll
  for (int k = 0; k < kWords / 256; ++k) {
    const unsigned i = threadIdx.x + 256 * k;
    lds[i] = pat(wg, i, seed);
    reg[k] = pat(wg, i, seed);
  }
  __syncthreads();
  unsigned long long bl = 0, br = 0;
  float spin = (float)threadIdx.x;
  for (int r = 0; r < rounds; ++r) {
#pragma unroll
    for (int k = 0; k < kWords / 256; ++k) {
      const unsigned i = threadIdx.x + 256 * k;
      bl += lds[i] != pat(wg, i, seed);
      br += reg[k] != pat(wg, i, seed);
    }
    for (int j = 0; j < 64; ++j) spin = __fmaf_rn(spin, 1.0001f, 0.5f);
    __syncthreads();
  }
  if (spin == 1.2345f) bl += 1;   // keep the spin
  if (bl) atomicAdd(bad, bl);
  if (br) atomicAdd(bad + 1, br);
}

__global__ __launch_bounds__(256) void lds_hog(int rounds, unsigned* sink) {
  extern __shared__ unsigned buf[];
  const int words = 96 * 1024 / 4;
  unsigned acc = 0;
  for (int r = 0; r < rounds; ++r) {
    for (int i = threadIdx.x; i < words; i += 256) buf[i] = i * 7u + r + blockIdx.x;
    __syncthreads();
    for (int i = threadIdx.x; i < words; i += 256) acc += buf[(i * 13) % words];
    __syncthreads();
  }
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  unsigned long long* bad;
  unsigned* sink;
  CK(hipMalloc(&bad, 16));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipFuncSetAttribute((const void*)lds_hog, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  for (int mode = 0; mode < 2; ++mode) {
    CK(hipMemset(bad, 0, 16));
    for (int it = 0; it < iters; ++it) {
      if (mode == 1)
        for (int k = 0; k < 6; ++k) hipLaunchKernelGGL(lds_hog, dim3(4096), dim3(256), 96 * 1024, b, 40, sink);
      hipLaunchKernelGGL(checker, dim3(4096), dim3(256), 0, a, 200, 0x9E3779B9u * (it + 1), bad);
    }
    CK(hipDeviceSynchronize());
    unsigned long long h[2];
    CK(hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost));
    printf("{\"mode\": \"%s\", \"iters\": %d, \"lds_words_bad\": %llu, \"reg_words_bad\": %llu}\n",
           mode ? "lds_hog_on_stream_b" : "alone", iters, h[0], h[1]);
    fflush(stdout);
  }
  return 0;
}
