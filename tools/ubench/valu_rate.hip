// Microbenchmark: VALU issue cost per wave-instruction on gfx950 (fp32 fma,
// packed fma/mul, exp, mixes) at 1, 2 and 8 resident waves per SIMD.
// hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate && ./valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 4096
typedef float f2 __attribute__((ext_vector_type(2)));
template <int KIND>
__global__ __launch_bounds__(64) void k(float* out, float a, float b) {
  float r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));
      if constexpr (KIND == 1) asm volatile("v_exp_f32 %0, %0" : "+v"(r[i]));
      if constexpr (KIND == 2) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[i]) : "v"(a));
      if constexpr (KIND == 3) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(f2*)&r[2 * i]) : "v"(*(f2*)&r[(2 * i + 2) & 15]), "v"(*(f2*)&r[(2 * i + 4) & 15]));
      if constexpr (KIND == 4) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(*(f2*)&r[2 * i]) : "v"(*(f2*)&r[(2 * i + 2) & 15]));
      if constexpr (KIND == 5) asm volatile("v_pk_fma_f32 %0, %1, %0, %2 op_sel_hi:[1,0,1]" : "+v"(*(f2*)&r[2 * i]) : "s"(*(double*)&a), "v"(*(f2*)&r[(2 * i + 4) & 15]));
      if constexpr (KIND == 6) {  // the scan's pair: 2 exp + 4 packed
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(*(f2*)&r[2 * i]) : "v"(*(f2*)&r[(2 * i + 2) & 15]));
        asm volatile("v_exp_f32 %0, %0" : "+v"(r[(2 * i + 6) & 15]));
        asm volatile("v_exp_f32 %0, %0" : "+v"(r[(2 * i + 7) & 15]));
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(*(f2*)&r[(2 * i + 8) & 15]) : "v"(*(f2*)&r[(2 * i + 2) & 15]));
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(f2*)&r[(2 * i + 10) & 15]) : "v"(*(f2*)&r[(2 * i + 2) & 15]), "v"(*(f2*)&r[(2 * i + 4) & 15]));
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(f2*)&r[(2 * i + 12) & 15]) : "v"(*(f2*)&r[(2 * i + 2) & 15]), "v"(*(f2*)&r[(2 * i + 4) & 15]));
      }
      if constexpr (KIND == 7) {  // the same pair in scalar form: 2 exp + 8 scalar
        asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[(i + 1) & 15]) : "v"(a));
        asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[(i + 2) & 15]) : "v"(a));
        asm volatile("v_exp_f32 %0, %0" : "+v"(r[(i + 3) & 15]));
        asm volatile("v_exp_f32 %0, %0" : "+v"(r[(i + 4) & 15]));
        asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[(i + 5) & 15]) : "v"(a));
        asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[(i + 6) & 15]) : "v"(a));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[(i + 7) & 15]) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[(i + 8) & 15]) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[(i + 9) & 15]) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[(i + 10) & 15]) : "v"(a), "v"(b));
      }
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
void run(const char* name, float* d, int instr_per_iter) {
  for (int w : {1, 2, 8}) {
    const int blocks = 1024 * w;  // one-wave workgroups, w per SIMD
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k<KIND>, blocks, 64, 0, 0, d, 1.0001f, 0.5f);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<KIND>, blocks, 64, 0, 0, d, 1.0001f, 0.5f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double per_simd = (double)w * ITERS * instr_per_iter;   // wave-instructions per SIMD
    printf("%-14s waves/SIMD %d: %.3f ms  %.2f SIMD cycles per wave-instr at 2.1 GHz\n", name, w, ms,
           ms * 1e6 * 2.1 / per_simd);
  }
}

int main() {
  float* d;
  (void)hipMalloc(&d, 1024 * 8 * 64 * 4);
  run<0>("v_fma_f32", d, 8);
  run<2>("v_mul_f32", d, 8);
  run<1>("v_exp_f32", d, 8);
  run<3>("v_pk_fma_f32", d, 8);
  run<4>("v_pk_mul_f32", d, 8);
  run<5>("v_pk_fma(sgpr)", d, 8);
  run<6>("pair:2exp+4pk", d, 48);
  run<7>("pair:2exp+8", d, 80);
  (void)hipFree(d);
  return 0;
}
