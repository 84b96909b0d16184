// Microbenchmark: VALU issue rates on gfx950 (fp32 fma, packed fma, exp, mul).
// hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate && ./valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 4096
template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float a, float b) {
  float r[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));
      if constexpr (KIND == 1) asm volatile("v_exp_f32 %0, %0" : "+v"(r[i]));
      if constexpr (KIND == 2) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));
      if constexpr (KIND == 4) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(r[i]) : "s"(a), "v"(b));
      if constexpr (KIND == 6) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "s"(a), "v"(b));
      if constexpr (KIND == 7) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));
      if constexpr (KIND == 5) {  // 1 exp + 4 fma, independent registers per slot
        float e = r[i];
        asm volatile("v_exp_f32 %0, %0" : "+v"(e));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[(i + 1) & 7]) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[(i + 2) & 7]) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[(i + 3) & 7]) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[(i + 4) & 7]) : "v"(a), "v"(b));
        r[i] = e;
      }
    }
    if constexpr (KIND == 3) {
      // packed fp32 fma on register pairs
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(double*)&r[0]) : "v"(*(double*)&r[2]), "v"(*(double*)&r[4]));
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(double*)&r[2]) : "v"(*(double*)&r[4]), "v"(*(double*)&r[6]));
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(double*)&r[4]) : "v"(*(double*)&r[6]), "v"(*(double*)&r[0]));
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(double*)&r[6]) : "v"(*(double*)&r[0]), "v"(*(double*)&r[2]));
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
void run(const char* name, float* d, int instr_per_iter) {
  const int blocks = 256 * 8;  // 8 blocks of 256 threads per CU = 32 waves/CU
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<KIND>, blocks, 256, 0, 0, d, 1.0001f, 0.5f);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<KIND>, blocks, 256, 0, 0, d, 1.0001f, 0.5f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double winstr = (double)blocks * 4 * ITERS * instr_per_iter;  // wave-instructions
  const double per_simd = winstr / 1024.0;
  printf("%-12s %.3f ms  %.3f wave-instr/ns/SIMD  -> %.2f cycles per wave-instr at 2.4 GHz\n", name, ms,
         per_simd / (ms * 1e6), (ms * 1e6 * 2.4) / per_simd);
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 8 * 256 * 4);
  run<0>("v_fma_f32", d, 8);
  run<2>("v_mul_f32", d, 8);
  run<4>("v_fmac(sgpr)", d, 8);
  run<3>("v_pk_fma_f32", d, 4);
  run<1>("v_exp_f32", d, 8);
  run<6>("v_fma(sgpr)", d, 8);
  run<7>("v_fmac(vgpr)", d, 8);
  run<5>("1exp+4fma", d, 40);
  hipFree(d);
  return 0;
}
