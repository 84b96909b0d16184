// patch.hip -- the image input path of the towers' patch embedding (include/mc_ops.h:
// mc_patch_embed_input), gfx950.
//
// Reference: the ISIC dataset's images go through timm / open_clip transforms (resize, crop,
// ToTensor, Normalize(mean, std): src/mamba_clip/data.py get_transform 37-108, IsicChallengeDataset
// 242-386) into a float NCHW batch, then the visual tower's patch-embed conv (k = s = P).  Here the
// last two host-side steps and the conv's input reshuffle are one device pass:
//   patches[(b * ph + i) * pw + j, (c * P + ky) * P + kx] = scale[c] * img(b, c, i*P + ky, j*P + kx) + shift[c]
// from either a float NCHW batch (scale / shift nullable: a plain im2col + cast) or the raw decoded
// uint8 NHWC images (scale = 1 / (255 std), shift = -mean / std: ToTensor + Normalize).
// One thread writes 4 consecutive patch columns (kx .. kx+3 of one (c, ky)): 4 contiguous input
// pixels, one 8-B (16-bit) / 16-B (fp32) store; consecutive threads walk the patch row in memory order.
#include "mc_common.h"
#include "../../include/mc_ops.h"

namespace mc {
namespace patch {

template <typename T> __device__ __forceinline__ f32x4 load4(const T* p);
template <> __device__ __forceinline__ f32x4 load4<float>(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
template <> __device__ __forceinline__ f32x4 load4<bf16_t>(const bf16_t* p) {
  const uint2 w = *reinterpret_cast<const uint2*>(p);
  return f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
               __uint_as_float(w.y & 0xffff0000u)};
}
template <> __device__ __forceinline__ f32x4 load4<f16_t>(const f16_t* p) {
  const uint2 w = *reinterpret_cast<const uint2*>(p);
  return f32x4{(float)__builtin_bit_cast(f16_t, (uint16_t)(w.x & 0xffffu)), (float)__builtin_bit_cast(f16_t, (uint16_t)(w.x >> 16)),
               (float)__builtin_bit_cast(f16_t, (uint16_t)(w.y & 0xffffu)), (float)__builtin_bit_cast(f16_t, (uint16_t)(w.y >> 16))};
}
template <typename T> __device__ __forceinline__ void store4(T* p, f32x4 v);
template <> __device__ __forceinline__ void store4<float>(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
template <> __device__ __forceinline__ void store4<bf16_t>(bf16_t* p, f32x4 v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(cvt_pk2<bf16_t>(v.x, v.y), cvt_pk2<bf16_t>(v.z, v.w));
}
template <> __device__ __forceinline__ void store4<f16_t>(f16_t* p, f32x4 v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(cvt_pk2<f16_t>(v.x, v.y), cvt_pk2<f16_t>(v.z, v.w));
}

struct Args {
  int batch, C, H, W, P, ph, pw;
  const void* img;
  const float* scale;
  const float* shift;
  void* out;
};

// float NCHW input: unit = (patch row, c, ky, kx / 4)
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void patch_nchw_kernel(const Args a) {
  const int q = a.P / 4;                        // 4-column groups per patch row
  const int per_row = a.C * a.P * q;            // units per patch row
  const int64_t total = (int64_t)a.batch * a.ph * a.pw * per_row;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t prow = u / per_row;
    const int r = (int)(u - prow * per_row);
    const int g = r % q, ky = (r / q) % a.P, c = r / (q * a.P);
    const int j = (int)(prow % a.pw), i = (int)((prow / a.pw) % a.ph), b = (int)(prow / ((int64_t)a.pw * a.ph));
    const TI* src = reinterpret_cast<const TI*>(a.img) + (((int64_t)b * a.C + c) * a.H + i * a.P + ky) * a.W + j * a.P + 4 * g;
    f32x4 v = load4<TI>(src);
    if (a.scale) v = v * a.scale[c] + a.shift[c];
    store4<TO>(reinterpret_cast<TO*>(a.out) + prow * (int64_t)a.C * a.P * a.P + ((int64_t)c * a.P + ky) * a.P + 4 * g, v);
  }
}

// uint8 NHWC input (decoded images): unit = (patch row, ky, kx / 4); 4 pixels x C bytes in, C stores out
template <typename TO, int C>
__global__ __launch_bounds__(256) void patch_nhwc_u8_kernel(const Args a) {
  const int q = a.P / 4;
  const int per_row = a.P * q;
  const int64_t total = (int64_t)a.batch * a.ph * a.pw * per_row;
  float sc[C], sh[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    sc[c] = a.scale ? a.scale[c] : 1.f;
    sh[c] = a.scale ? a.shift[c] : 0.f;
  }
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t prow = u / per_row;
    const int r = (int)(u - prow * per_row);
    const int g = r % q, ky = r / q;
    const int j = (int)(prow % a.pw), i = (int)((prow / a.pw) % a.ph), b = (int)(prow / ((int64_t)a.pw * a.ph));
    const uint8_t* src = reinterpret_cast<const uint8_t*>(a.img) +
                         ((((int64_t)b * a.H + i * a.P + ky) * a.W + j * a.P + 4 * g) * C);
    uint8_t px[4 * C];
#pragma unroll
    for (int k = 0; k < 4 * C; ++k) px[k] = src[k];   // 4 * C contiguous bytes (12 for RGB)
    TO* dst = reinterpret_cast<TO*>(a.out) + prow * (int64_t)C * a.P * a.P + (int64_t)ky * a.P + 4 * g;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const f32x4 v = f32x4{(float)px[c], (float)px[C + c], (float)px[2 * C + c], (float)px[3 * C + c]} * sc[c] + sh[c];
      store4<TO>(dst + (int64_t)c * a.P * a.P, v);
    }
  }
}

template <typename TI>
static void launch_nchw(int otype, const Args& a, dim3 grid, hipStream_t s) {
  if (otype == MC_DTYPE_F32) hipLaunchKernelGGL((patch_nchw_kernel<TI, float>), grid, dim3(256), 0, s, a);
  else if (otype == MC_DTYPE_BF16) hipLaunchKernelGGL((patch_nchw_kernel<TI, bf16_t>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((patch_nchw_kernel<TI, f16_t>), grid, dim3(256), 0, s, a);
}
template <int C>
static void launch_u8(int otype, const Args& a, dim3 grid, hipStream_t s) {
  if (otype == MC_DTYPE_F32) hipLaunchKernelGGL((patch_nhwc_u8_kernel<float, C>), grid, dim3(256), 0, s, a);
  else if (otype == MC_DTYPE_BF16) hipLaunchKernelGGL((patch_nhwc_u8_kernel<bf16_t, C>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((patch_nhwc_u8_kernel<f16_t, C>), grid, dim3(256), 0, s, a);
}

}  // namespace patch
}  // namespace mc

using namespace mc;

extern "C" int mc_patch_embed_input(const mc_patch_input_params* p, void* stream) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_patch_embed_input: null params");
  MC_CHECK(p->batch >= 0 && p->channels > 0 && p->patch > 0 && p->patch % 4 == 0 && p->height % p->patch == 0 &&
               p->width % p->patch == 0,
           MC_ERR_SHAPE, "mc_patch_embed_input: patch must be a multiple of 4 dividing H and W (got P %d, %dx%d)",
           p->patch, p->height, p->width);
  const bool u8 = p->in_dtype == MC_DTYPE_U8;
  MC_CHECK(u8 ? p->layout == MC_LAYOUT_NHWC : p->layout == MC_LAYOUT_NCHW, MC_ERR_DTYPE,
           "mc_patch_embed_input: uint8 input is NHWC (decoded images), float input NCHW");
  MC_CHECK(u8 || p->in_dtype == MC_DTYPE_F32 || p->in_dtype == MC_DTYPE_BF16 || p->in_dtype == MC_DTYPE_F16,
           MC_ERR_DTYPE, "mc_patch_embed_input: bad input dtype %d", p->in_dtype);
  MC_CHECK(p->out_dtype == MC_DTYPE_F32 || p->out_dtype == MC_DTYPE_BF16 || p->out_dtype == MC_DTYPE_F16,
           MC_ERR_DTYPE, "mc_patch_embed_input: bad output dtype %d", p->out_dtype);
  MC_CHECK(!u8 || p->channels == 3 || p->channels == 1, MC_ERR_SHAPE, "mc_patch_embed_input: uint8 input has 1 or 3 channels");
  if (p->batch == 0) return MC_OK;   // empty batch: nothing to read, pointers may be null
  MC_CHECK(p->img && p->out && (!p->scale) == (!p->shift), MC_ERR_INVALID,
           "mc_patch_embed_input: img / out non-null; scale and shift both given or both null");
  const int ib = p->in_dtype == MC_DTYPE_F32 ? 16 : 8;
  MC_CHECK(u8 || ((reinterpret_cast<uintptr_t>(p->img) % ib) == 0), MC_ERR_INVALID, "mc_patch_embed_input: misaligned image");
  MC_CHECK((reinterpret_cast<uintptr_t>(p->out) % (p->out_dtype == MC_DTYPE_F32 ? 16 : 8)) == 0, MC_ERR_INVALID,
           "mc_patch_embed_input: misaligned output");
  patch::Args a;
  a.batch = p->batch; a.C = p->channels; a.H = p->height; a.W = p->width; a.P = p->patch;
  a.ph = a.H / a.P; a.pw = a.W / a.P;
  a.img = p->img; a.scale = p->scale; a.shift = p->shift; a.out = p->out;
  const int64_t units = (int64_t)a.batch * a.ph * a.pw * (u8 ? 1 : a.C) * a.P * (a.P / 4);
  const dim3 grid((unsigned)std::min<int64_t>((units + 255) / 256, 65536));
  hipStream_t s = (hipStream_t)stream;
  if (u8) {
    if (a.C == 3) patch::launch_u8<3>(p->out_dtype, a, grid, s);
    else patch::launch_u8<1>(p->out_dtype, a, grid, s);
  } else if (p->in_dtype == MC_DTYPE_F32) patch::launch_nchw<float>(p->out_dtype, a, grid, s);
  else if (p->in_dtype == MC_DTYPE_BF16) patch::launch_nchw<bf16_t>(p->out_dtype, a, grid, s);
  else patch::launch_nchw<f16_t>(p->out_dtype, a, grid, s);
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_patch_embed_input: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}
