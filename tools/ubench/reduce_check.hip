// Check the lane mapping of the cross-lane primitives used by the scan backward.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
  const int lane = threadIdx.x;
  const unsigned a = 1000 + lane, b = 2000 + lane;
  auto r32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  auto r16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  out[lane * 8 + 0] = r32[0];
  out[lane * 8 + 1] = r32[1];
  out[lane * 8 + 2] = r16[0];
  out[lane * 8 + 3] = r16[1];
  out[lane * 8 + 4] = __builtin_amdgcn_update_dpp((int)a, (int)a, 0x128, 0xF, 0xF, false);
  out[lane * 8 + 5] = __builtin_amdgcn_update_dpp((int)a, (int)a, 0x124, 0xF, 0xF, false);
  out[lane * 8 + 6] = __builtin_amdgcn_update_dpp((int)a, (int)a, 0x4E, 0xF, 0xF, false);
  out[lane * 8 + 7] = __builtin_amdgcn_update_dpp((int)a, (int)a, 0xB1, 0xF, 0xF, false);
}
int main() {
  unsigned *d, h[64 * 8];
  hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("lane: p32[0] p32[1] p16[0] p16[1] ror8 ror4 qp2301 qp1032\n");
  for (int l = 0; l < 64; ++l) {
    printf("%2d:", l);
    for (int j = 0; j < 8; ++j) printf(" %u", h[l * 8 + j]);
    printf("\n");
  }
  return 0;
}
