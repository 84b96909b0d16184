// lds_poison.hip -- test utility (not part of the product library): fill the LDS of every CU with a
// NaN pattern.  Launched on a stream right before a kernel, it leaves that kernel's workgroups an LDS
// whose every byte it did not write itself reads as NaN, so a kernel that consumes LDS it never wrote
// (content left by whatever ran on the CU before) turns its outputs to NaN deterministically instead of
// differing from run to run with the previous occupant.  tools/lds_audit.py drives it.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/lds_poison.hip -o tools/liblds_poison.so
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ __launch_bounds__(1024) void lds_poison_kernel(uint32_t pattern, int words) {
  extern __shared__ uint32_t lds[];
  for (int i = threadIdx.x; i < words; i += blockDim.x) lds[i] = pattern;
  __syncthreads();
  // read one word back so the stores cannot be dropped as dead
  if (lds[(threadIdx.x * 37) % words] == 0x12345678u) lds[0] = 0;
}

extern "C" int lds_poison(uint32_t pattern, int blocks, void* stream) {
  const int bytes = 160 * 1024;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)lds_poison_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) !=
        hipSuccess)
      return 1;
    attr = true;
  }
  hipLaunchKernelGGL(lds_poison_kernel, dim3(blocks), dim3(1024), bytes, (hipStream_t)stream, pattern, bytes / 4);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
