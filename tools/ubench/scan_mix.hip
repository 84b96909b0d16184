// Microbenchmark: the selective-scan forward's per-position VALU mix on gfx950,
// in isolation (no HBM traffic): per state pair  arg = A*dt, 2x v_exp,
// x = dA*x + B*du, y += C*x, with B/C wave-uniform (SGPRs) and the position's
// dt from a softplus.  Reports SIMD cycles per position per wave at 1..4
// resident waves per SIMD, for packed (v_pk_*_f32) and scalar fp32 forms, with
// and without the exponentials.
//   hipcc --offload-arch=gfx950 -O3 scan_mix.hip -o scan_mix && ./scan_mix
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const f32x4 cf32x4;

constexpr int kL = 4096;

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float softplus_f(float x) {
  const float t = ex2(fminf(x, 20.f) * 1.442695f);
  const float lg = __builtin_amdgcn_logf(1.f + t) * 0.6931472f;
  return x > 20.f ? x : lg;
}

// MODE 0: packed, with exp.  1: scalar fp32, with exp.  2: packed, no exp.  3: packed, exp, no softplus
template <int MODE>
__global__ __launch_bounds__(64) void k(const float* __restrict__ bc, float* out, int L) {
  const int lane = threadIdx.x;
  const cf32x4* bcs = (const cf32x4*)bc;
  f32x2 A2[8], x[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    A2[p] = f32x2{-1.f - 2 * p - lane * 1e-3f, -2.f - 2 * p} * 0.01f;
    x[p] = f32x2{0.f, 0.f};
  }
  float uacc = 0.f;
  float u = lane * 1e-2f, d = lane * 1e-3f - 0.5f;
  for (int t = 0; t < L; ++t) {
    f32x4 cur[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) cur[q] = bcs[(t & 3) * 8 + q];
    const float dt = MODE == 3 ? d : softplus_f(d);
    const float du = dt * u;
    if constexpr (MODE == 1) {
      float ya = 0.f, yb = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int p = 2 * q + h;
          const f32x2 bb = h ? cur[q].hi : cur[q].lo, cc = h ? cur[4 + q].hi : cur[4 + q].lo;
          float xa = x[p].x, xb = x[p].y;
          xa = fmaf(ex2(A2[p].x * dt), xa, bb.x * du);
          xb = fmaf(ex2(A2[p].y * dt), xb, bb.y * du);
          ya = fmaf(cc.x, xa, ya);
          yb = fmaf(cc.y, xb, yb);
          x[p] = f32x2{xa, xb};
        }
      }
      uacc += ya + yb;
    } else {
      f32x2 ya = {0.f, 0.f}, yb = {0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int p = 2 * q + h;
          const f32x2 bb = h ? cur[q].hi : cur[q].lo, cc = h ? cur[4 + q].hi : cur[4 + q].lo;
          const f32x2 arg = A2[p] * dt;
          const f32x2 dA = MODE == 2 ? arg : f32x2{ex2(arg.x), ex2(arg.y)};
          x[p] = dA * x[p] + bb * du;
          if (h) yb = cc * x[p] + yb;
          else ya = cc * x[p] + ya;
        }
      }
      const f32x2 ys = ya + yb;
      uacc += ys.x + ys.y;
    }
    u += 1e-3f;
    d -= 1e-4f;
  }
  out[blockIdx.x * 64 + lane] = uacc + x[0].x + x[7].y;
}

template <int MODE>
void run(const char* name, const float* bc, float* out) {
  for (int w = 1; w <= 4; ++w) {
    const int blocks = 1024 * w;   // 256 CUs x 4 SIMDs x w one-wave workgroups
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k<MODE>, blocks, 64, 0, 0, bc, out, kL);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<MODE>, blocks, 64, 0, 0, bc, out, kL);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // SIMD cycles per position per wave at an assumed 2.1 GHz (read relative, not absolute)
    printf("%-22s waves/SIMD %d: %.3f ms  %.1f cyc/pos/wave (2.1 GHz)  %.1f cyc/pos wall\n", name, w, ms,
           ms * 1e-3 * 2.1e9 / (double)kL / w, ms * 1e-3 * 2.1e9 / (double)kL);
  }
}

int main() {
  float *bc, *out;
  hipMalloc(&bc, 4 * 32 * 4);
  float h[128];
  for (int i = 0; i < 128; ++i) h[i] = 0.01f * (i % 17) - 0.05f;
  hipMemcpy(bc, h, sizeof(h), hipMemcpyHostToDevice);
  hipMalloc(&out, 1024 * 4 * 64 * 4);
  run<0>("packed+exp+softplus", bc, out);
  run<1>("scalar+exp+softplus", bc, out);
  run<2>("packed, no exp", bc, out);
  run<3>("packed+exp, no softpl", bc, out);
  hipFree(bc);
  hipFree(out);
  return 0;
}
