// FETCH_SIZE calibration for the scan forward's load pattern on gfx950: a wave
// owns 64 rows of a (rows, L) bf16 matrix and walks L in 32-position chunks;
// per chunk each lane loads 16 B, lane j -> row j / 4, 16-B block j % 4 (four
// lanes cover one row's 64-B chunk), exactly as scan_fwd_kernel stages u / delta.
// Known bytes read = rows * L * 2.  Compare FETCH_SIZE * 1024 against it.
//   hipcc --offload-arch=gfx950 -O3 fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(64) void k(const uint4* __restrict__ m, int L, float* out) {
  const int lane = threadIdx.x;
  const int row0 = blockIdx.x * 64;
  const int vpr = L / 8;                                   // 16-B vectors per row
  float acc = 0.f;
  for (int c = 0; c < L / 32; ++c) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int j = lane + 64 * kk;
      const int r = j / 4, cc = j % 4;
      const uint4 v = m[(size_t)(row0 + r) * vpr + c * 4 + cc];
      acc += __uint_as_float(v.x) + __uint_as_float(v.w);
    }
  }
  out[blockIdx.x * 64 + lane] = acc;
}

int main() {
  const int rows = 64 * 3072, L = 4096;                   // one C4 array: 64 x 3072 rows of 4096 bf16
  const size_t bytes = (size_t)rows * L * 2;
  uint4* m;
  float* out;
  (void)hipMalloc(&m, bytes);
  (void)hipMemset(m, 0, bytes);
  (void)hipMalloc(&out, rows * 4);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, rows / 64, 64, 0, 0, m, L, out);
  (void)hipDeviceSynchronize();
  printf("calibration kernel read %zu bytes per launch (%.1f KB)\n", bytes, bytes / 1024.0);
  return 0;
}
