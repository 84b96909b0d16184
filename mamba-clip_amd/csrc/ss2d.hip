// ss2d.hip -- SS2D cross-scan glue for gfx950 (include/mc_ss2d.h).
//
// Reference: src/mamba_clip/model.py SS2D.forward (630-647) and forward_corev0 (503-565).  The
// reference builds u = stack[x, x^T] (then flips) with copies after a permute + conv2d + SiLU, and
// merges the four direction outputs with flips, transposes and adds before LayerNorm and the
// silu(z) gate.  The flips are in the scan kernels' addressing (reverse_groups); here:
//   conv_stack_fwd  channels-last x -> depthwise k x k conv + bias + SiLU -> u[b, 0] (h*W + w) and
//                   u[b, 1] (w*H + h), fp32, through one LDS tile per (batch, 16 x 16 pixels (8 x 8
//                   for small images), 32 channels): no permute copy, no stack, no transposed copy;
//   conv_stack_bwd  g = du[b, 0] + du[b, 1]^T over the tile plus its halo, g * silu'(pre) with pre
//                   recomputed, dx by the transposed depthwise conv, dw / db partials per workgroup
//                   summed in a fixed order (reduce_partials): deterministic;
//   merge_fwd       ((y1 + y2) + y3) + y4 of all channels of a pixel tile in LDS (directions 1, 3
//                   read in their x^T frame), LayerNorm over channels (two-pass mean / variance),
//                   * silu(z), channels-last;
//   merge_bwd       dz, dLN weight / bias partials, and d(merge) written to the four direction
//                   gradients in their own frames (the grouped scan backward reads them as dout).
// One thread owns one pixel and 4 consecutive channels (16-B fp32 / 8-B 16-bit channels-last
// vectors, 8 threads cover a 32-channel block).
#include <type_traits>

#include "mc_common.h"
#include "../../include/mc_ss2d.h"

namespace mc {
namespace ss2d {

constexpr int CB = 32;    // channels per block (conv kernels)
constexpr int NT = 256;   // threads per workgroup
// conv tiles: TS x TS pixels, 16 (8 when the image is at most 8 pixels on a side: 7 x 7 VSSM stage)
inline int conv_ts(int H, int W) { return (H <= 8 || W <= 8) ? 8 : 16; }

// ---- 4 consecutive channels of a channels-last row, as fp32
template <typename T> __device__ __forceinline__ f32x4 ld4(const T* p);
template <> __device__ __forceinline__ f32x4 ld4<float>(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
template <> __device__ __forceinline__ f32x4 ld4<bf16_t>(const bf16_t* p) {
  const uint2 w = *reinterpret_cast<const uint2*>(p);
  return f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
               __uint_as_float(w.y & 0xffff0000u)};
}
template <> __device__ __forceinline__ f32x4 ld4<f16_t>(const f16_t* p) {
  const uint2 w = *reinterpret_cast<const uint2*>(p);
  return f32x4{(float)__builtin_bit_cast(f16_t, (uint16_t)(w.x & 0xffffu)), (float)__builtin_bit_cast(f16_t, (uint16_t)(w.x >> 16)),
               (float)__builtin_bit_cast(f16_t, (uint16_t)(w.y & 0xffffu)), (float)__builtin_bit_cast(f16_t, (uint16_t)(w.y >> 16))};
}
template <typename T> __device__ __forceinline__ void st4(T* p, f32x4 v);
template <> __device__ __forceinline__ void st4<float>(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
template <> __device__ __forceinline__ void st4<bf16_t>(bf16_t* p, f32x4 v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(cvt_pk2<bf16_t>(v.x, v.y), cvt_pk2<bf16_t>(v.z, v.w));
}
template <> __device__ __forceinline__ void st4<f16_t>(f16_t* p, f32x4 v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(cvt_pk2<f16_t>(v.x, v.y), cvt_pk2<f16_t>(v.z, v.w));
}
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

struct ConvArgs {
  int B, H, W, C, tiles_w, tiles;
  int64_t xbs, xhs, xws;
  const void* x;
  const float* w;
  const float* bias;
  float* u;
  const float* du;
  void* dx;
  float* ws;   // [B * tiles][C * (K*K + 1)]: dw partials, then db partials
};

// ------------------------------------------------------------------ conv + SiLU -> u = [x, x^T]
template <typename TX, int K, int TS>
__global__ __launch_bounds__(NT) void conv_stack_fwd_kernel(const ConvArgs a) {
  constexpr int R = K / 2, TPS = TS * TS + 1;
  __shared__ float tile[CB * TPS];
  const int tw = blockIdx.x % a.tiles_w, th = blockIdx.x / a.tiles_w;
  const int c0 = blockIdx.y * CB, b = blockIdx.z;
  const int h0 = th * TS, w0 = tw * TS;
  const int t = threadIdx.x, cg = t & 7, ps = t >> 3;
  const int cc = c0 + 4 * cg;
  const bool cok = cc < a.C;   // C % 4 == 0: a 4-channel group is all in or all out
  const TX* xb = reinterpret_cast<const TX*>(a.x) + (int64_t)b * a.xbs + (cok ? cc : 0);
  f32x4 wk[K * K];
#pragma unroll
  for (int k = 0; k < K * K; ++k)
    wk[k] = cok ? f32x4{a.w[(cc + 0) * K * K + k], a.w[(cc + 1) * K * K + k], a.w[(cc + 2) * K * K + k],
                        a.w[(cc + 3) * K * K + k]}
                : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 bv = (cok && a.bias) ? *reinterpret_cast<const f32x4*>(a.bias + cc) : f32x4{0.f, 0.f, 0.f, 0.f};
  for (int pass = 0; pass < TS * TS / 32; ++pass) {
    const int p = pass * 32 + ps, py = p / TS, px = p % TS;
    const int h = h0 + py, w = w0 + px;
    f32x4 acc = bv;
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int hh = h + kh - R, ww = w + kw - R;
        if (cok && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W)
          acc += wk[kh * K + kw] * ld4<TX>(xb + (int64_t)hh * a.xhs + (int64_t)ww * a.xws);
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) tile[(4 * cg + i) * TPS + py * TS + px] = acc[i] * sigm(acc[i]);
  }
  __syncthreads();
  const int L = a.H * a.W;
  float* u0 = a.u + (int64_t)b * 2 * a.C * L;
  float* u1 = u0 + (int64_t)a.C * L;
  for (int e = t; e < CB * TS * TS; e += NT) {   // x frame: w fastest
    const int c = e / (TS * TS), py = (e / TS) % TS, px = e % TS;
    const int h = h0 + py, w = w0 + px;
    if (c0 + c < a.C && h < a.H && w < a.W) u0[(int64_t)(c0 + c) * L + h * a.W + w] = tile[c * TPS + py * TS + px];
  }
  for (int e = t; e < CB * TS * TS; e += NT) {   // x^T frame: h fastest
    const int c = e / (TS * TS), px = (e / TS) % TS, py = e % TS;
    const int h = h0 + py, w = w0 + px;
    if (c0 + c < a.C && h < a.H && w < a.W) u1[(int64_t)(c0 + c) * L + w * a.H + h] = tile[c * TPS + py * TS + px];
  }
}

// ------------------------------------------------------------------ its backward
template <typename TX, int K, int TS>
__global__ __launch_bounds__(NT) void conv_stack_bwd_kernel(const ConvArgs a) {
  constexpr int R = K / 2, TE = TS + 2 * R, GS = TE * TE + 1;   // extended tile (halo R), odd stride
  constexpr int NV = K * K + 1;                                   // dw taps + db per channel
  constexpr int NG = CB * GS > 32 * 8 * NV * 4 ? CB * GS : 32 * 8 * NV * 4;   // the reduction reuses the tile
  __shared__ float G[NG];
  const int tw = blockIdx.x % a.tiles_w, th = blockIdx.x / a.tiles_w;
  const int c0 = blockIdx.y * CB, b = blockIdx.z;
  const int h0 = th * TS, w0 = tw * TS;
  const int t = threadIdx.x, cg = t & 7, ps = t >> 3;
  const int cc = c0 + 4 * cg;
  const bool cok = cc < a.C;
  const int L = a.H * a.W;
  const float* du0 = a.du + (int64_t)b * 2 * a.C * L;
  const float* du1 = du0 + (int64_t)a.C * L;

  // 1. g = du0 + du1^T over the extended tile (0 outside the image or past C)
  for (int e = t; e < CB * TE * TE; e += NT) {
    const int c = e / (TE * TE), r = e % (TE * TE), yy = r / TE, xx = r % TE;
    const int h = h0 - R + yy, w = w0 - R + xx;
    const bool ok = c0 + c < a.C && h >= 0 && h < a.H && w >= 0 && w < a.W;
    G[c * GS + yy * TE + xx] = ok ? du0[(int64_t)(c0 + c) * L + h * a.W + w] : 0.f;
  }
  __syncthreads();
  for (int e = t; e < CB * TE * TE; e += NT) {
    const int c = e / (TE * TE), r = e % (TE * TE), xx = r / TE, yy = r % TE;
    const int h = h0 - R + yy, w = w0 - R + xx;
    if (c0 + c < a.C && h >= 0 && h < a.H && w >= 0 && w < a.W)
      G[c * GS + yy * TE + xx] += du1[(int64_t)(c0 + c) * L + w * a.H + h];
  }
  __syncthreads();

  const TX* xb = reinterpret_cast<const TX*>(a.x) + (int64_t)b * a.xbs + (cok ? cc : 0);
  f32x4 wk[K * K];
#pragma unroll
  for (int k = 0; k < K * K; ++k)
    wk[k] = cok ? f32x4{a.w[(cc + 0) * K * K + k], a.w[(cc + 1) * K * K + k], a.w[(cc + 2) * K * K + k],
                        a.w[(cc + 3) * K * K + k]}
                : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 bv = (cok && a.bias) ? *reinterpret_cast<const f32x4*>(a.bias + cc) : f32x4{0.f, 0.f, 0.f, 0.f};

  // 2. gpre = g * silu'(pre) over the extended tile (pre recomputed); dw / db from the inner pixels
  f32x4 dw[K * K], db = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < K * K; ++k) dw[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int pe = ps; pe < TE * TE; pe += NT / 8) {
    const int yy = pe / TE, xx = pe % TE;
    const int h = h0 - R + yy, w = w0 - R + xx;
    if (!cok || h < 0 || h >= a.H || w < 0 || w >= a.W) continue;   // g is 0 there
    f32x4 xt[K * K];
    f32x4 pre = bv;
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int hh = h + kh - R, ww = w + kw - R;
        xt[kh * K + kw] = (hh >= 0 && hh < a.H && ww >= 0 && ww < a.W)
                              ? ld4<TX>(xb + (int64_t)hh * a.xhs + (int64_t)ww * a.xws)
                              : f32x4{0.f, 0.f, 0.f, 0.f};
        pre += wk[kh * K + kw] * xt[kh * K + kw];
      }
    f32x4 gp;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float s = sigm(pre[i]);
      float* gr = &G[(4 * cg + i) * GS + yy * TE + xx];
      gp[i] = *gr * (s * (1.f + pre[i] * (1.f - s)));
      *gr = gp[i];
    }
    if (yy >= R && yy < R + TS && xx >= R && xx < R + TS) {
      db += gp;
#pragma unroll
      for (int k = 0; k < K * K; ++k) dw[k] += gp * xt[k];
    }
  }
  __syncthreads();

  // 3. dx = the transposed depthwise conv of gpre, at the inner pixels
  TX* dxb = reinterpret_cast<TX*>(a.dx) + (int64_t)b * L * a.C;
  for (int pe = ps; pe < TS * TS; pe += NT / 8) {
    const int py = pe / TS, px = pe % TS, h = h0 + py, w = w0 + px;
    if (!cok || h >= a.H || w >= a.W) continue;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int yy = py + 2 * R - kh, xx = px + 2 * R - kw;   // (py + R) - (kh - R)
        const f32x4 g4 = f32x4{G[(4 * cg + 0) * GS + yy * TE + xx], G[(4 * cg + 1) * GS + yy * TE + xx],
                               G[(4 * cg + 2) * GS + yy * TE + xx], G[(4 * cg + 3) * GS + yy * TE + xx]};
        acc += wk[kh * K + kw] * g4;
      }
    st4<TX>(dxb + ((int64_t)h * a.W + w) * a.C + cc, acc);
  }
  __syncthreads();

  // 4. this workgroup's dw / db: the 32 pixel slots summed in order -> workspace
  float* red = G;   // [ps][cg][NV][4]
#pragma unroll
  for (int k = 0; k < K * K; ++k) *reinterpret_cast<f32x4*>(&red[((ps * 8 + cg) * NV + k) * 4]) = dw[k];
  *reinterpret_cast<f32x4*>(&red[((ps * 8 + cg) * NV + K * K) * 4]) = db;
  __syncthreads();
  float* wsb = a.ws + (int64_t)(b * a.tiles + blockIdx.x) * a.C * NV;
  for (int v = t; v < CB * NV; v += NT) {
    const int c = v / NV, j = v % NV;
    if (c0 + c >= a.C) continue;
    float s = 0.f;
    for (int q = 0; q < 32; ++q) s += red[((q * 8 + c / 4) * NV + j) * 4 + (c & 3)];
    wsb[j < K * K ? (c0 + c) * (K * K) + j : a.C * (K * K) + c0 + c] = s;
  }
}

// ------------------------------------------------------------------ merge + LayerNorm + silu(z)
// One workgroup owns a TS x TS pixel tile of one image and ALL its channels: the merged tile
// (C x TP fp32, TP = TS * TS) sits in LDS, loaded once in the x frame (directions 0, 2) and once in the
// x^T frame (directions 1, 3, h fastest: coalesced either way).  Per-pixel statistics come from
// pixel-owner threads (pixel p, channel slice s of S = NT / TP); the channels-last outputs from
// channel-owner threads (4 consecutive channels each, looping over the tile's pixels: coalesced
// 16-B z / dy / y / dz accesses).  TS = 16 for C <= 128, 8 for C <= 512, 4 for C <= 2048 (LDS).
struct MergeArgs {
  int B, H, W, C, tiles_w, tiles;
  float eps;
  const float* out;
  const void* z;
  int64_t zbs, zhs, zws;
  const float* lw;
  const float* lb;
  void* y;
  float* mean;
  float* rstd;
  const void* dy;
  int64_t dybs, dyhs, dyws;
  float* dout;
  void* dz;
  float* ws;   // [B * tiles][2 C]: dLN weight partials, then dLN bias partials
};

inline int merge_ts(int C) { return C <= 128 ? 16 : (C <= 512 ? 8 : (C <= 2048 ? 4 : 0)); }
inline size_t merge_lds_bytes(int C, int ts) {
  const int tp = ts * ts, s = NT / tp;
  return ((size_t)C * (tp + 1) + 2 * (size_t)s * tp + 4 * (size_t)tp + 8 * (size_t)NT) * sizeof(float);
}
// channel-owner split: thread t owns channel quad t % NQ (NQ = C / 4) and walks the pixels
// pg, pg + PG, ... of the tile (pg = t / NQ, PG = NT / NQ groups when NQ < NT) -- every thread busy
// at small C, 16-B accesses of consecutive threads adjacent in the channels-last rows
struct Owner {
  int cq, pg, npg;
  __device__ Owner(int C, int t) {
    const int nq = C / 4;
    if (nq >= NT) { cq = t; pg = 0; npg = 1; }
    else { npg = NT / nq; cq = t % nq; pg = t / nq; if (pg >= npg) cq = nq; }   // cq == nq: idle
  }
};

// T[c][p] = ((y1 + y2) + y3) + y4 of all channels over the tile (0 outside the image)
template <int TS>
__device__ __forceinline__ void load_merged_all(const MergeArgs& a, int b, int h0, int w0, float* T) {
  constexpr int TP = TS * TS;
  const int t = threadIdx.x, L = a.H * a.W;
  const float* o = a.out + (int64_t)b * 4 * a.C * L;
  const int64_t blk = (int64_t)a.C * L;
  for (int e = t; e < a.C * TP; e += NT) {
    const int c = e / TP, r = e % TP, py = r / TS, px = r % TS;
    const int h = h0 + py, w = w0 + px;
    float v = 0.f;
    if (h < a.H && w < a.W) {
      const int64_t i = (int64_t)c * L + h * a.W + w;
      v = o[i] + o[2 * blk + i];   // y1 (direction 0) + y2 (direction 2, walked backwards in place)
    }
    T[c * (TP + 1) + r] = v;
  }
  __syncthreads();
  for (int e = t; e < a.C * TP; e += NT) {
    const int c = e / TP, r = e % TP, px = r / TS, py = r % TS;
    const int h = h0 + py, w = w0 + px;
    if (h < a.H && w < a.W) {
      const int64_t i = (int64_t)c * L + w * a.H + h;
      float& v = T[c * (TP + 1) + py * TS + px];
      v = (v + o[blk + i]) + o[3 * blk + i];   // + y3 (direction 1, x^T frame) + y4 (direction 3)
    }
  }
  __syncthreads();
}

template <typename TZ, typename TY, int TS>
__global__ __launch_bounds__(NT) void merge_fwd_kernel(const MergeArgs a) {
  constexpr int TP = TS * TS, S = NT / TP;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* T = sm;                              // [C][TP + 1]
  float* red = T + a.C * (TP + 1);            // [S][TP]
  float* smu = red + 2 * S * TP;              // [TP]
  float* srs = smu + TP;                      // [TP]
  const int tw = blockIdx.x % a.tiles_w, th = blockIdx.x / a.tiles_w, b = blockIdx.y;
  const int h0 = th * TS, w0 = tw * TS;
  const int t = threadIdx.x;
  load_merged_all<TS>(a, b, h0, w0, T);
  // per-pixel mean, then centred variance (two passes over LDS), S channel slices per pixel
  const int p = t % TP, sl = t / TP;
  float sum = 0.f;
  for (int c = sl; c < a.C; c += S) sum += T[c * (TP + 1) + p];
  red[sl * TP + p] = sum;
  __syncthreads();
  if (sl == 0) {
    float r = red[p];
    for (int j = 1; j < S; ++j) r += red[j * TP + p];
    smu[p] = r / (float)a.C;
  }
  __syncthreads();
  const float mu = smu[p];
  float q = 0.f;
  for (int c = sl; c < a.C; c += S) {
    const float d = T[c * (TP + 1) + p] - mu;
    q += d * d;
  }
  red[sl * TP + p] = q;
  __syncthreads();
  if (sl == 0) {
    float r = red[p];
    for (int j = 1; j < S; ++j) r += red[j * TP + p];
    const float rs = rsqrtf(r / (float)a.C + a.eps);
    srs[p] = rs;
    const int h = h0 + p / TS, w = w0 + p % TS;
    if (h < a.H && w < a.W) {
      const int64_t pix = ((int64_t)b * a.H + h) * a.W + w;
      a.mean[pix] = mu;
      a.rstd[pix] = rs;
    }
  }
  __syncthreads();
  // channel-owner threads: y = (xhat w + b) * silu(z), channels-last
  const Owner ow(a.C, t);
  for (int cq = ow.cq; 4 * cq < a.C; cq += NT) {
    const int ch = 4 * cq;
    const f32x4 lw = *reinterpret_cast<const f32x4*>(a.lw + ch);
    const f32x4 lb = a.lb ? *reinterpret_cast<const f32x4*>(a.lb + ch) : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int pp = ow.pg; pp < TP; pp += ow.npg) {
      const int h = h0 + pp / TS, w = w0 + pp % TS;
      if (h >= a.H || w >= a.W) continue;
      const f32x4 zz = ld4<TZ>(reinterpret_cast<const TZ*>(a.z) + (int64_t)b * a.zbs + (int64_t)h * a.zhs +
                               (int64_t)w * a.zws + ch);
      const float m = smu[pp], rs = srs[pp];
      f32x4 yv;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float yln = (T[(ch + i) * (TP + 1) + pp] - m) * rs * lw[i] + lb[i];
        yv[i] = yln * (zz[i] * sigm(zz[i]));
      }
      st4<TY>(reinterpret_cast<TY*>(a.y) + (((int64_t)b * a.H + h) * a.W + w) * a.C + ch, yv);
    }
  }
}

template <typename TZ, typename TY, int TS>
__global__ __launch_bounds__(NT) void merge_bwd_kernel(const MergeArgs a) {
  constexpr int TP = TS * TS, S = NT / TP;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* T = sm;                              // [C][TP + 1]: the merged tile, then d(merge)
  float* ra = T + a.C * (TP + 1);             // [S][TP]
  float* rb = ra + S * TP;                    // [S][TP]
  float* smu = rb + S * TP;                   // [TP] mean, rstd, mean(dxhat), mean(dxhat xhat)
  float* srs = smu + TP;
  float* sma = srs + TP;
  float* smb = sma + TP;
  const int tw = blockIdx.x % a.tiles_w, th = blockIdx.x / a.tiles_w, b = blockIdx.y;
  const int h0 = th * TS, w0 = tw * TS;
  const int t = threadIdx.x;
  if (t < TP) {
    const int h = h0 + t / TS, w = w0 + t % TS;
    const bool in = h < a.H && w < a.W;
    const int64_t pix = ((int64_t)b * a.H + h) * a.W + w;
    smu[t] = in ? a.mean[pix] : 0.f;
    srs[t] = in ? a.rstd[pix] : 0.f;
  }
  load_merged_all<TS>(a, b, h0, w0, T);
  auto zrow = [&](int h, int w) {
    return reinterpret_cast<const TZ*>(a.z) + (int64_t)b * a.zbs + (int64_t)h * a.zhs + (int64_t)w * a.zws;
  };
  auto dyrow = [&](int h, int w) {
    return reinterpret_cast<const TY*>(a.dy) + (int64_t)b * a.dybs + (int64_t)h * a.dyhs + (int64_t)w * a.dyws;
  };
  // pass A (pixel p, channel slice sl): sum(dxhat), sum(dxhat xhat)
  {
    const int p = t % TP, sl = t / TP;
    const int h = h0 + p / TS, w = w0 + p % TS;
    float sa = 0.f, sb = 0.f;
    if (h < a.H && w < a.W) {
      const TZ* zr = zrow(h, w);
      const TY* gr = dyrow(h, w);
      const float m = smu[p], rs = srs[p];
      for (int cq = sl; 4 * cq < a.C; cq += S) {
        const int ch = 4 * cq;
        const f32x4 zz = ld4<TZ>(zr + ch), dy = ld4<TY>(gr + ch);
        const f32x4 lw = *reinterpret_cast<const f32x4*>(a.lw + ch);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float xh = (T[(ch + i) * (TP + 1) + p] - m) * rs;
          const float dxh = dy[i] * (zz[i] * sigm(zz[i])) * lw[i];
          sa += dxh;
          sb += dxh * xh;
        }
      }
    }
    ra[sl * TP + p] = sa;
    rb[sl * TP + p] = sb;
  }
  __syncthreads();
  if (t < TP) {
    float x = ra[t], y = rb[t];
    for (int j = 1; j < S; ++j) {
      x += ra[j * TP + t];
      y += rb[j * TP + t];
    }
    sma[t] = x / (float)a.C;
    smb[t] = y / (float)a.C;
  }
  __syncthreads();
  // pass B (channel owner): dz, dLN weight / bias, d(merge) -> T (each entry rewritten by its owner only)
  float* wsb = a.ws + (int64_t)(b * a.tiles + blockIdx.x) * 2 * a.C;
  float* rg = smb + TP;   // [pixel group][4 NQ] weight then bias partials (NQ < NT)
  const Owner ow(a.C, t);
  for (int cq = ow.cq; 4 * cq < a.C; cq += NT) {
    const int ch = 4 * cq;
    const f32x4 lw = *reinterpret_cast<const f32x4*>(a.lw + ch);
    const f32x4 lb = a.lb ? *reinterpret_cast<const f32x4*>(a.lb + ch) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 dgw = f32x4{0.f, 0.f, 0.f, 0.f}, dgb = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int pp = ow.pg; pp < TP; pp += ow.npg) {
      const int h = h0 + pp / TS, w = w0 + pp % TS;
      if (h >= a.H || w >= a.W) continue;
      const f32x4 zz = ld4<TZ>(zrow(h, w) + ch), dy = ld4<TY>(dyrow(h, w) + ch);
      const float m = smu[pp], rs = srs[pp], ma = sma[pp], mb = smb[pp];
      f32x4 dzv;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float& v = T[(ch + i) * (TP + 1) + pp];
        const float xh = (v - m) * rs;
        const float s = sigm(zz[i]);
        const float dyln = dy[i] * (zz[i] * s);
        dzv[i] = dy[i] * (xh * lw[i] + lb[i]) * (s * (1.f + zz[i] * (1.f - s)));
        dgw[i] += dyln * xh;
        dgb[i] += dyln;
        v = rs * (dyln * lw[i] - ma - xh * mb);
      }
      st4<TZ>(reinterpret_cast<TZ*>(a.dz) + (((int64_t)b * a.H + h) * a.W + w) * a.C + ch, dzv);
    }
    if (ow.npg == 1) {
      *reinterpret_cast<f32x4*>(wsb + ch) = dgw;
      *reinterpret_cast<f32x4*>(wsb + a.C + ch) = dgb;
    } else {
      *reinterpret_cast<f32x4*>(rg + ow.pg * a.C + ch) = dgw;
      *reinterpret_cast<f32x4*>(rg + (ow.npg + ow.pg) * a.C + ch) = dgb;
    }
  }
  __syncthreads();
  if (ow.npg > 1) {   // the pixel groups' partials, in group order
    for (int c = t; c < 2 * a.C; c += NT) {
      const int which = c / a.C, ch = c % a.C;
      float r = 0.f;
      for (int g = 0; g < ow.npg; ++g) r += rg[(which * ow.npg + g) * a.C + ch];
      wsb[which * a.C + ch] = r;
    }
  }
  // d(merge) -> the four direction gradients, each in its own frame
  const int L = a.H * a.W;
  float* o = a.dout + (int64_t)b * 4 * a.C * L;
  const int64_t blk = (int64_t)a.C * L;
  for (int e = t; e < a.C * TP; e += NT) {   // directions 0, 2: x frame
    const int c = e / TP, r = e % TP, qy = r / TS, qx = r % TS;
    const int hh = h0 + qy, ww = w0 + qx;
    if (hh < a.H && ww < a.W) {
      const int64_t i = (int64_t)c * L + hh * a.W + ww;
      const float v = T[c * (TP + 1) + r];
      o[i] = v;
      o[2 * blk + i] = v;
    }
  }
  for (int e = t; e < a.C * TP; e += NT) {   // directions 1, 3: x^T frame
    const int c = e / TP, r = e % TP, qx = r / TS, qy = r % TS;
    const int hh = h0 + qy, ww = w0 + qx;
    if (hh < a.H && ww < a.W) {
      const int64_t i = (int64_t)c * L + ww * a.H + hh;
      const float v = T[c * (TP + 1) + qy * TS + qx];
      o[blk + i] = v;
      o[3 * blk + i] = v;
    }
  }
}

// ------------------------------------------------------------------ workgroup partials -> parameter gradients
// dst[i] = sum_{k < s} src[k * stride + i] (fixed order: slabs k = part, part + 8, ... per thread, then the
// 8 parts in order).  The partial count is large (batch x tiles) and the rows short (C x 10 floats), so
// the slabs are split over 8 threads per column (mc_sum_slabs walks all of them in one thread).
__global__ __launch_bounds__(256) void reduce_partials_kernel(int s, int n, const float* __restrict__ src, int64_t stride,
                                                              float* __restrict__ dst) {
  __shared__ float part[8][33];
  const int col = blockIdx.x * 32 + (threadIdx.x & 31), q = threadIdx.x >> 5;
  float acc = 0.f;
  if (col < n)
    for (int k = q; k < s; k += 8) acc += src[(int64_t)k * stride + col];
  part[q][threadIdx.x & 31] = acc;
  __syncthreads();
  if (q == 0 && col < n) {
    float r = part[0][threadIdx.x];
#pragma unroll
    for (int j = 1; j < 8; ++j) r += part[j][threadIdx.x];
    dst[col] = r;
  }
}

static void reduce_partials(int s, int n, const float* src, int64_t stride, float* dst, hipStream_t st) {
  hipLaunchKernelGGL(reduce_partials_kernel, dim3((unsigned)((n + 31) / 32)), dim3(256), 0, st, s, n, src, stride, dst);
}

// ------------------------------------------------------------------ host side
static int check_launch(const char* who) {
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "%s: launch failed: %s", who, hipGetErrorString(e));
  return MC_OK;
}

static int conv_validate(const mc_ss2d_conv_params* p, const char* who) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "%s: null params", who);
  MC_CHECK(p->batch >= 0 && p->height >= 0 && p->width >= 0 && p->channels >= 0, MC_ERR_SHAPE, "%s: negative shape", who);
  MC_CHECK(p->ksize == 3, MC_ERR_SHAPE, "%s: ksize %d (SS2D's depthwise conv is 3 x 3)", who, p->ksize);
  MC_CHECK(p->channels % 4 == 0 && p->x_batch_stride % 4 == 0 && p->x_row_stride % 4 == 0 && p->x_col_stride % 4 == 0,
           MC_ERR_SHAPE, "%s: channels and the channels-last strides must be multiples of 4", who);
  MC_CHECK(p->xtype == MC_DTYPE_F32 || p->xtype == MC_DTYPE_BF16 || p->xtype == MC_DTYPE_F16, MC_ERR_DTYPE,
           "%s: x must be f32 / bf16 / f16", who);
  const uintptr_t al = p->xtype == MC_DTYPE_F32 ? 15u : 7u;
  MC_CHECK(p->x && p->weight && (reinterpret_cast<uintptr_t>(p->x) & al) == 0 &&
               (!p->bias || aligned16(p->bias)),
           MC_ERR_INVALID, "%s: x / weight must be non-null, x 4-channel aligned, bias 16-B aligned", who);
  return MC_OK;
}

static void conv_args(const mc_ss2d_conv_params* p, ConvArgs& a, dim3& grid) {
  const int ts = conv_ts(p->height, p->width);
  a.B = p->batch; a.H = p->height; a.W = p->width; a.C = p->channels;
  a.tiles_w = (a.W + ts - 1) / ts;
  a.tiles = a.tiles_w * ((a.H + ts - 1) / ts);
  a.xbs = p->x_batch_stride; a.xhs = p->x_row_stride; a.xws = p->x_col_stride;
  a.x = p->x; a.w = p->weight; a.bias = p->bias;
  grid = dim3((unsigned)a.tiles, (unsigned)((a.C + CB - 1) / CB), (unsigned)a.B);
}

static int merge_validate(const mc_ss2d_merge_params* p, const char* who) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "%s: null params", who);
  MC_CHECK(p->batch >= 0 && p->height >= 0 && p->width >= 0 && p->channels > 0 && merge_ts(p->channels) > 0,
           MC_ERR_SHAPE, "%s: bad shape (channels in [4, 2048])", who);
  MC_CHECK(p->channels % 4 == 0 && p->z_batch_stride % 4 == 0 && p->z_row_stride % 4 == 0 && p->z_col_stride % 4 == 0,
           MC_ERR_SHAPE, "%s: channels and the channels-last strides of z must be multiples of 4", who);
  auto okt = [](int t) { return t == MC_DTYPE_F32 || t == MC_DTYPE_BF16 || t == MC_DTYPE_F16; };
  MC_CHECK(okt(p->ztype) && okt(p->ytype), MC_ERR_DTYPE, "%s: z / y must be f32 / bf16 / f16", who);
  MC_CHECK(p->out && p->z && p->ln_weight && p->mean && p->rstd && aligned16(p->ln_weight) &&
               (!p->ln_bias || aligned16(p->ln_bias)),
           MC_ERR_INVALID, "%s: out, z, ln_weight, mean, rstd non-null; LayerNorm parameters 16-B aligned", who);
  return MC_OK;
}

static void merge_args(const mc_ss2d_merge_params* p, MergeArgs& a, dim3& grid) {
  const int ts = merge_ts(p->channels);
  a.B = p->batch; a.H = p->height; a.W = p->width; a.C = p->channels; a.eps = p->eps;
  a.tiles_w = (a.W + ts - 1) / ts;
  a.tiles = a.tiles_w * ((a.H + ts - 1) / ts);
  a.out = p->out; a.z = p->z; a.zbs = p->z_batch_stride; a.zhs = p->z_row_stride; a.zws = p->z_col_stride;
  a.lw = p->ln_weight; a.lb = p->ln_bias; a.y = p->y; a.mean = p->mean; a.rstd = p->rstd;
  grid = dim3((unsigned)a.tiles, (unsigned)a.B);
}

template <int K, int TS>
static void conv_launch(bool bwd, int xtype, const ConvArgs& a, dim3 grid, hipStream_t s) {
  if (bwd) {
    if (xtype == MC_DTYPE_F32) hipLaunchKernelGGL((conv_stack_bwd_kernel<float, K, TS>), grid, dim3(NT), 0, s, a);
    else if (xtype == MC_DTYPE_BF16) hipLaunchKernelGGL((conv_stack_bwd_kernel<bf16_t, K, TS>), grid, dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((conv_stack_bwd_kernel<f16_t, K, TS>), grid, dim3(NT), 0, s, a);
  } else {
    if (xtype == MC_DTYPE_F32) hipLaunchKernelGGL((conv_stack_fwd_kernel<float, K, TS>), grid, dim3(NT), 0, s, a);
    else if (xtype == MC_DTYPE_BF16) hipLaunchKernelGGL((conv_stack_fwd_kernel<bf16_t, K, TS>), grid, dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((conv_stack_fwd_kernel<f16_t, K, TS>), grid, dim3(NT), 0, s, a);
  }
}

template <int K>
static int conv_fwd_t(const mc_ss2d_conv_params* p, hipStream_t s) {
  ConvArgs a{};
  dim3 grid;
  conv_args(p, a, grid);
  a.u = p->u;
  if (conv_ts(a.H, a.W) == 16) conv_launch<K, 16>(false, p->xtype, a, grid, s);
  else conv_launch<K, 8>(false, p->xtype, a, grid, s);
  return check_launch("mc_ss2d_conv_stack_fwd");
}

template <typename TZ, typename TY, int TS>
static void merge_launch_ts(bool bwd, const MergeArgs& a, dim3 grid, hipStream_t s) {
  const size_t lds = merge_lds_bytes(a.C, TS);
  if (bwd) hipLaunchKernelGGL((merge_bwd_kernel<TZ, TY, TS>), grid, dim3(NT), lds, s, a);
  else hipLaunchKernelGGL((merge_fwd_kernel<TZ, TY, TS>), grid, dim3(NT), lds, s, a);
}
template <typename TZ, typename TY>
static void merge_launch(bool bwd, const MergeArgs& a, dim3 grid, hipStream_t s) {
  const int ts = merge_ts(a.C);
  if (ts == 16) merge_launch_ts<TZ, TY, 16>(bwd, a, grid, s);
  else if (ts == 8) merge_launch_ts<TZ, TY, 8>(bwd, a, grid, s);
  else merge_launch_ts<TZ, TY, 4>(bwd, a, grid, s);
}
template <typename TZ>
static void merge_launch_y(int ytype, bool bwd, const MergeArgs& a, dim3 grid, hipStream_t s) {
  if (ytype == MC_DTYPE_F32) merge_launch<TZ, float>(bwd, a, grid, s);
  else if (ytype == MC_DTYPE_BF16) merge_launch<TZ, bf16_t>(bwd, a, grid, s);
  else merge_launch<TZ, f16_t>(bwd, a, grid, s);
}
static void merge_dispatch(const mc_ss2d_merge_params* p, bool bwd, const MergeArgs& a, dim3 grid, hipStream_t s) {
  if (p->ztype == MC_DTYPE_F32) merge_launch_y<float>(p->ytype, bwd, a, grid, s);
  else if (p->ztype == MC_DTYPE_BF16) merge_launch_y<bf16_t>(p->ytype, bwd, a, grid, s);
  else merge_launch_y<f16_t>(p->ytype, bwd, a, grid, s);
}

}  // namespace ss2d
}  // namespace mc

using namespace mc;
using namespace mc::ss2d;

extern "C" int mc_ss2d_conv_stack_fwd(const mc_ss2d_conv_params* p, void* stream) {
  int rc = conv_validate(p, "mc_ss2d_conv_stack_fwd");
  if (rc) return rc;
  MC_CHECK(p->u != nullptr, MC_ERR_INVALID, "mc_ss2d_conv_stack_fwd: u must be non-null");
  if ((int64_t)p->batch * p->height * p->width * p->channels == 0) return MC_OK;
  return conv_fwd_t<3>(p, (hipStream_t)stream);
}

extern "C" size_t mc_ss2d_conv_bwd_workspace_bytes(int32_t batch, int32_t height, int32_t width, int32_t channels,
                                                   int32_t ksize) {
  const int ts = conv_ts(height, width);
  const int64_t tiles = (int64_t)((width + ts - 1) / ts) * ((height + ts - 1) / ts);
  return (size_t)batch * tiles * channels * (ksize * ksize + 1) * sizeof(float);
}

extern "C" int mc_ss2d_conv_stack_bwd(const mc_ss2d_conv_bwd_params* p, void* stream) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_ss2d_conv_stack_bwd: null params");
  int rc = conv_validate(&p->fwd, "mc_ss2d_conv_stack_bwd");
  if (rc) return rc;
  const mc_ss2d_conv_params& f = p->fwd;
  MC_CHECK(p->du && p->dx && p->dweight, MC_ERR_INVALID, "mc_ss2d_conv_stack_bwd: du, dx, dweight must be non-null");
  const uintptr_t al = f.xtype == MC_DTYPE_F32 ? 15u : 7u;
  MC_CHECK((reinterpret_cast<uintptr_t>(p->dx) & al) == 0, MC_ERR_INVALID, "mc_ss2d_conv_stack_bwd: dx misaligned");
  const size_t need = mc_ss2d_conv_bwd_workspace_bytes(f.batch, f.height, f.width, f.channels, f.ksize);
  MC_CHECK(p->workspace && p->workspace_bytes >= need, MC_ERR_WORKSPACE,
           "mc_ss2d_conv_stack_bwd: workspace must be >= %zu bytes", need);
  hipStream_t s = (hipStream_t)stream;
  constexpr int K = 3, NV = K * K + 1;
  if ((int64_t)f.batch * f.height * f.width == 0 || f.channels == 0) {
    if (f.channels) {
      (void)hipMemsetAsync(p->dweight, 0, (size_t)f.channels * K * K * 4, s);
      if (p->dbias) (void)hipMemsetAsync(p->dbias, 0, (size_t)f.channels * 4, s);
    }
    return MC_OK;
  }
  ConvArgs a{};
  dim3 grid;
  conv_args(&f, a, grid);
  a.du = p->du; a.dx = p->dx; a.ws = reinterpret_cast<float*>(p->workspace);
  if (conv_ts(a.H, a.W) == 16) conv_launch<K, 16>(true, f.xtype, a, grid, s);
  else conv_launch<K, 8>(true, f.xtype, a, grid, s);
  rc = check_launch("mc_ss2d_conv_stack_bwd");
  if (rc) return rc;
  const int nwg = f.batch * a.tiles;
  reduce_partials(nwg, f.channels * K * K, a.ws, (int64_t)f.channels * NV, p->dweight, s);
  if (p->dbias) reduce_partials(nwg, f.channels, a.ws + (int64_t)f.channels * K * K, (int64_t)f.channels * NV, p->dbias, s);
  return check_launch("mc_ss2d_conv_stack_bwd (partials)");
}

extern "C" int mc_ss2d_merge_ln_gate_fwd(const mc_ss2d_merge_params* p, void* stream) {
  int rc = merge_validate(p, "mc_ss2d_merge_ln_gate_fwd");
  if (rc) return rc;
  MC_CHECK(p->y != nullptr, MC_ERR_INVALID, "mc_ss2d_merge_ln_gate_fwd: y must be non-null");
  if ((int64_t)p->batch * p->height * p->width == 0) return MC_OK;
  MergeArgs a{};
  dim3 grid;
  merge_args(p, a, grid);
  merge_dispatch(p, false, a, grid, (hipStream_t)stream);
  return check_launch("mc_ss2d_merge_ln_gate_fwd");
}

extern "C" size_t mc_ss2d_merge_bwd_workspace_bytes(int32_t batch, int32_t height, int32_t width, int32_t channels) {
  const int ts = merge_ts(channels) > 0 ? merge_ts(channels) : 4;
  const int64_t tiles = (int64_t)((width + ts - 1) / ts) * ((height + ts - 1) / ts);
  return (size_t)batch * tiles * 2 * channels * sizeof(float);
}

extern "C" int mc_ss2d_merge_ln_gate_bwd(const mc_ss2d_merge_bwd_params* p, void* stream) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_ss2d_merge_ln_gate_bwd: null params");
  int rc = merge_validate(&p->fwd, "mc_ss2d_merge_ln_gate_bwd");
  if (rc) return rc;
  const mc_ss2d_merge_params& f = p->fwd;
  MC_CHECK(p->dy && p->dout && p->dz && p->dln_weight, MC_ERR_INVALID,
           "mc_ss2d_merge_ln_gate_bwd: dy, dout, dz, dln_weight must be non-null");
  MC_CHECK(p->dy_batch_stride % 4 == 0 && p->dy_row_stride % 4 == 0 && p->dy_col_stride % 4 == 0, MC_ERR_SHAPE,
           "mc_ss2d_merge_ln_gate_bwd: dy strides must be multiples of 4");
  const size_t need = mc_ss2d_merge_bwd_workspace_bytes(f.batch, f.height, f.width, f.channels);
  MC_CHECK(p->workspace && p->workspace_bytes >= need, MC_ERR_WORKSPACE,
           "mc_ss2d_merge_ln_gate_bwd: workspace must be >= %zu bytes", need);
  hipStream_t s = (hipStream_t)stream;
  if ((int64_t)f.batch * f.height * f.width == 0) {
    (void)hipMemsetAsync(p->dln_weight, 0, (size_t)f.channels * 4, s);
    if (p->dln_bias) (void)hipMemsetAsync(p->dln_bias, 0, (size_t)f.channels * 4, s);
    return MC_OK;
  }
  MergeArgs a{};
  dim3 grid;
  merge_args(&f, a, grid);
  a.dy = p->dy; a.dybs = p->dy_batch_stride; a.dyhs = p->dy_row_stride; a.dyws = p->dy_col_stride;
  a.dout = p->dout; a.dz = p->dz; a.ws = reinterpret_cast<float*>(p->workspace);
  merge_dispatch(&f, true, a, grid, s);
  rc = check_launch("mc_ss2d_merge_ln_gate_bwd");
  if (rc) return rc;
  const int nwg = f.batch * a.tiles;
  reduce_partials(nwg, f.channels, a.ws, 2 * (int64_t)f.channels, p->dln_weight, s);
  if (p->dln_bias) reduce_partials(nwg, f.channels, a.ws + f.channels, 2 * (int64_t)f.channels, p->dln_bias, s);
  return check_launch("mc_ss2d_merge_ln_gate_bwd (partials)");
}

// ------------------------------------------------------------------ grouped projections (mc_ss2d_group_proj)
// Y[b][g][m][l] = A + sum_n W[g][m][n] X[b][g % mod][n][l].  Lane = position (64 consecutive l: the
// X[n][l] loads are coalesced 256-B rows); a wave owns kGpM output rows, so each X value feeds kGpM FMAs
// from registers and W[g][m][n] is wave-uniform (scalar loads; with m contiguous, w_ms == 1, one
// 64-B scalar load per n).  Long reductions (rows_in >= 64) split n over the workgroup's 4 waves,
// whose partial sums meet in LDS and are added in wave order; short ones give each wave its own row
// chunk.  Every sum runs in a fixed order: deterministic.
constexpr int kGpM = 16;     // output rows per wave
constexpr int kGpW = 4;      // waves per workgroup

template <bool kSplitN, bool kMC>
__global__ __launch_bounds__(64 * kGpW) void group_proj_kernel(const mc_ss2d_group_proj_params p) {
  __shared__ float part[kSplitN ? (kGpW - 1) * kGpM * 64 : 1];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = blockIdx.x * 64 + lane;
  const int bg = blockIdx.y;
  const int b = bg / p.groups, g = bg % p.groups;
  const int m0 = (kSplitN ? blockIdx.z : blockIdx.z * kGpW + w) * kGpM;
  if (!kSplitN && m0 >= p.rows_out) return;          // wave-uniform (no barrier in this form)
  const int n0 = kSplitN ? (int)(((int64_t)w * p.rows_in) / kGpW) : 0;
  const int n1 = kSplitN ? (int)(((int64_t)(w + 1) * p.rows_in) / kGpW) : p.rows_in;
  const bool ok = l < p.seqlen;
  const int lc = ok ? l : p.seqlen - 1;
  const float* __restrict__ X = p.x + (int64_t)b * p.x_bs + (int64_t)(g % p.x_group_mod) * p.x_gs + lc;
  const float* __restrict__ W = p.w + (int64_t)g * p.w_gs + (int64_t)m0 * (kMC ? 1 : p.w_ms);
  const int mcount = min(kGpM, p.rows_out - m0);
  float acc[kGpM];
#pragma unroll
  for (int i = 0; i < kGpM; ++i) acc[i] = 0.f;
  // a whole 16-row chunk reads 16 consecutive weights per n (one scalar load when m is contiguous); the
  // last, partial chunk re-reads its last row for the rows past M (computed, never stored)
  auto sweep = [&](auto full) __attribute__((always_inline)) {
    auto wv = [&](int i, int n) __attribute__((always_inline)) {
      const int ie = decltype(full)::value ? i : min(i, mcount - 1);
      return kMC ? W[(int64_t)n * p.w_ns + ie] : W[(int64_t)ie * p.w_ms + (int64_t)n * p.w_ns];
    };
    int n = n0;
    for (; n + 4 <= n1; n += 4) {
      float xv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) xv[q] = X[(int64_t)(n + q) * p.x_ns];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < kGpM; ++i) acc[i] = fmaf(wv(i, n + q), xv[q], acc[i]);
    }
    for (; n < n1; ++n) {
      const float xv = X[(int64_t)n * p.x_ns];
#pragma unroll
      for (int i = 0; i < kGpM; ++i) acc[i] = fmaf(wv(i, n), xv, acc[i]);
    }
  };
  if (mcount == kGpM) sweep(std::true_type());
  else sweep(std::false_type());
  if constexpr (kSplitN) {
    if (w > 0) {
#pragma unroll
      for (int i = 0; i < kGpM; ++i) part[((w - 1) * kGpM + i) * 64 + lane] = acc[i];
    }
    __syncthreads();
    if (w > 0) return;
#pragma unroll
    for (int v = 0; v < kGpW - 1; ++v)
#pragma unroll
      for (int i = 0; i < kGpM; ++i) acc[i] += part[(v * kGpM + i) * 64 + lane];
  }
  if (!ok) return;
  const float* A = p.acc ? p.acc + (int64_t)b * p.a_bs + (int64_t)g * p.a_gs + (int64_t)m0 * p.a_ms + l : nullptr;
  float* Y = p.y + (int64_t)b * p.y_bs + (int64_t)g * p.y_gs + (int64_t)m0 * p.y_ms + l;
#pragma unroll
  for (int i = 0; i < kGpM; ++i)
    if (i < mcount) Y[(int64_t)i * p.y_ms] = (A ? A[(int64_t)i * p.a_ms] : 0.f) + acc[i];
}

extern "C" int mc_ss2d_group_proj(const mc_ss2d_group_proj_params* p, void* stream) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_ss2d_group_proj: null params");
  MC_CHECK(p->batch >= 0 && p->groups >= 1 && p->rows_out >= 0 && p->rows_in >= 0 && p->seqlen >= 0 &&
               p->x_group_mod >= 1 && p->x_group_mod <= p->groups,
           MC_ERR_SHAPE, "mc_ss2d_group_proj: bad shape (B %d G %d M %d N %d L %d mod %d)", p->batch, p->groups,
           p->rows_out, p->rows_in, p->seqlen, p->x_group_mod);
  MC_CHECK(p->rows_out <= 4096 && (int64_t)p->batch * p->groups < 65536, MC_ERR_SHAPE,
           "mc_ss2d_group_proj: rows_out %d (<= 4096) or batch * groups %lld (< 65536) out of range", p->rows_out,
           (long long)p->batch * p->groups);
  MC_CHECK(p->w && p->y && (p->x || p->rows_in == 0), MC_ERR_INVALID, "mc_ss2d_group_proj: null pointer");
  if ((int64_t)p->batch * p->rows_out * p->seqlen == 0) return MC_OK;
  const bool split = p->rows_in >= 64;
  const bool mc = p->w_ms == 1;
  const dim3 grid((p->seqlen + 63) / 64, p->batch * p->groups,
                  split ? (p->rows_out + kGpM - 1) / kGpM : (p->rows_out + kGpM * kGpW - 1) / (kGpM * kGpW));
  hipStream_t s = (hipStream_t)stream;
  if (split && mc) hipLaunchKernelGGL((group_proj_kernel<true, true>), grid, dim3(64 * kGpW), 0, s, *p);
  else if (split) hipLaunchKernelGGL((group_proj_kernel<true, false>), grid, dim3(64 * kGpW), 0, s, *p);
  else if (mc) hipLaunchKernelGGL((group_proj_kernel<false, true>), grid, dim3(64 * kGpW), 0, s, *p);
  else hipLaunchKernelGGL((group_proj_kernel<false, false>), grid, dim3(64 * kGpW), 0, s, *p);
  return check_launch("mc_ss2d_group_proj");
}
