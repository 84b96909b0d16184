// scan_fwd.hip -- selective-scan forward for MI355X (gfx950, CDNA4).
//
// Computes (reference semantics: /root/reference/src/mamba_clip/model.py:83-169,
// the op behind mamba_ssm's selective_scan_fn called at model.py:539-550):
//   dt   = softplus(delta + delta_bias[d])                  (optional softplus / bias)
//   x_t  = exp(dt_t * A[d,n]) * x_{t-1} + dt_t * B[b,g,n,t] * u_t
//   y_t  = sum_n C[b,g,n,t] * x_t[n]  (+ D[d] * u_t)  (* silu(z_t))
//
// Design (DESIGN.md "scan_fwd"):
//  * One thread owns one (b, d) channel and keeps all dstate states in
//    registers, walking the sequence in chunks of kT = 32 positions.  This is
//    the work-optimal form of the recurrence (no parallel-prefix overhead);
//    B*D channels give >= 3 waves/SIMD at the benchmark shapes.
//  * A workgroup = up to 256 channels of ONE (batch, group), so B_t / C_t are
//    wave-uniform: they are staged once per chunk in LDS as fp32 [t][n] and
//    read with broadcast ds_read_b128.
//  * u / delta tiles are moved HBM -> registers with fully coalesced 16-byte
//    loads along the sequence (64-B row segments), written to LDS rows, and
//    each thread then reads back its own row (bank-conflict-free: row stride
//    = 144 B for 16-bit inputs).  The next chunk's loads are issued right after
//    the LDS write, so their latency hides under this chunk's recurrence.
//  * y (+D u) is written back over the thread's own (already consumed) LDS
//    row in fp32; a cooperative pass then applies the z gate with coalesced z
//    loads and out stores.  HBM traffic = the algorithmic bytes.
//  * exp(dt*A) = exp2(dt * A*log2e) on v_exp_f32.
#include "mc_common.h"
#include "../../include/mc_scan.h"

namespace mc {
namespace scan {

constexpr int kT = MC_SCAN_CHUNK;  // sequence positions per chunk
constexpr int kMaxRows = 256;      // channels per workgroup

// LDS row of one channel for one chunk: kT/4 blocks, block k = {u[4k..4k+3],
// delta[4k..4k+3]} (2 x 4 elements).  After the thread has consumed block k
// it writes y[4k..4k+3] (fp32, 16 B) over the block's first 16 bytes, so the
// y tile needs no extra LDS.
template <typename TI>
struct RowLayout {
  static constexpr int kHalf = 4 * (int)sizeof(TI);         // 4 elements of one array
  static constexpr int kBlock = 2 * kHalf;                   // >= 16 B (room for 4 fp32 y)
  static constexpr int kBytes = (kT / 4) * kBlock;
  static constexpr int kStride = kBytes + 16;                // pad: conflict-free row reads
};

struct FwdArgs {
  int batch, dim, seqlen, dstate, n_groups, n_chunks;
  int softplus;
  int64_t u_bs, u_ds, dt_bs, dt_ds, z_bs, z_ds, o_bs, o_ds;
  int64_t B_bs, B_gs, B_ns, C_bs, C_gs, C_ns;
  const void* u; const void* delta; const float* A; const void* B; const void* C;
  const float* D; const void* z; const float* delta_bias;
  void* out; float* chunk_states; float* last_state;
};

template <typename TI, typename TW, int kN, bool kAligned>
__global__ __launch_bounds__(kMaxRows, 2) void scan_fwd_kernel(const FwdArgs a) {
  using L = RowLayout<TI>;
  constexpr int VI = ElemTraits<TI>::kVec;      // elements per 16-B vector (inputs)
  constexpr int VW = ElemTraits<TW>::kVec;      // elements per 16-B vector (B/C)
  constexpr int kVPR = kT / VI;                 // vectors per row segment
  constexpr int kBCRow = kT / VW;               // vectors per (n) row of a B/C chunk
  constexpr int kBCVecs = kN * kBCRow;          // vectors in one B (or C) chunk tile
  constexpr int kBCPer = (2 * kBCVecs + 63) / 64;  // per thread, sized for a 64-row workgroup

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int rows = blockDim.x;
  char* rowbuf = smem;
  float* bc = reinterpret_cast<float*>(smem + rows * L::kStride);  // [kT][2*kN]: B then C

  const int tid = threadIdx.x;
  const int b = blockIdx.z;
  const int g = blockIdx.y;
  const int H = a.dim / a.n_groups;
  const int dbase = g * H + blockIdx.x * rows;
  const int nrows = min(rows, H - (int)blockIdx.x * rows);
  const int L_ = a.seqlen;
  const bool hasZ = a.z != nullptr;
  const bool softplus = a.softplus != 0;

  const TI* __restrict__ u = reinterpret_cast<const TI*>(a.u) + (int64_t)b * a.u_bs;
  const TI* __restrict__ dl = reinterpret_cast<const TI*>(a.delta) + (int64_t)b * a.dt_bs;
  const TI* __restrict__ zp = reinterpret_cast<const TI*>(a.z) + (int64_t)b * a.z_bs;
  TI* __restrict__ out = reinterpret_cast<TI*>(a.out) + (int64_t)b * a.o_bs;
  const TW* __restrict__ Bp = reinterpret_cast<const TW*>(a.B) + (int64_t)b * a.B_bs + (int64_t)g * a.B_gs;
  const TW* __restrict__ Cp = reinterpret_cast<const TW*>(a.C) + (int64_t)b * a.C_bs + (int64_t)g * a.C_gs;

  // ---- per-channel constants
  const int my_d = dbase + tid;
  const bool my_ok = tid < nrows;
  float A2[kN];
#pragma unroll
  for (int n = 0; n < kN; ++n)
    A2[n] = (my_ok && n < a.dstate) ? a.A[(int64_t)my_d * a.dstate + n] * kLog2e : 0.f;
  const float Dv = (my_ok && a.D) ? a.D[my_d] : 0.f;
  const float biasv = (my_ok && a.delta_bias) ? a.delta_bias[my_d] : 0.f;

  float x[kN];
#pragma unroll
  for (int n = 0; n < kN; ++n) x[n] = 0.f;

  // ---- cooperative tile movers.  Vector j = tid + k*rows -> (row j / kVPR,
  // col j % kVPR): kVPR consecutive lanes cover one 64-B row segment.
  // Rows past the group end are clamped onto a valid row (loaded, never stored).
  uint4 pu[kVPR], pd[kVPR], pbc[kBCPer];

  auto load_tiles = [&](int l0) {
    const bool full = kAligned && (l0 + kT <= L_);
#pragma unroll
    for (int k = 0; k < kVPR; ++k) {
      const int j = tid + k * rows;
      const int r = min(j / kVPR, nrows - 1), c = j % kVPR;
      const int col0 = l0 + c * VI;
      const TI* su = u + (int64_t)(dbase + r) * a.u_ds + col0;
      const TI* sd = dl + (int64_t)(dbase + r) * a.dt_ds + col0;
      if (full) {
        pu[k] = ld16(su);
        pd[k] = ld16(sd);
      } else {
        const int nv = max(0, min(VI, L_ - col0));
        pu[k] = ld16_masked(su, nv);
        pd[k] = ld16_masked(sd, nv);
      }
    }
#pragma unroll
    for (int k = 0; k < kBCPer; ++k) {
      const int j = tid + k * rows;
      const bool isC = j >= kBCVecs;
      const int jj = isC ? j - kBCVecs : j;
      const int n = min(jj / kBCRow, a.dstate - 1), c = jj % kBCRow;
      const int col0 = l0 + c * VW;
      const TW* src = (isC ? Cp + (int64_t)n * a.C_ns : Bp + (int64_t)n * a.B_ns) + col0;
      if (j < 2 * kBCVecs) {
        if (full) pbc[k] = ld16(src);
        else pbc[k] = ld16_masked(src, max(0, min(VW, L_ - col0)));
      }
    }
  };
  auto store_tiles_lds = [&]() {
#pragma unroll
    for (int k = 0; k < kVPR; ++k) {
      const int j = tid + k * rows;
      const int r = j / kVPR, c = j % kVPR;
      char* row = rowbuf + r * L::kStride;
      if constexpr (L::kHalf == 16) {   // fp32: one vector = one half-block
        char* blk = row + c * L::kBlock;
        st16(blk, pu[k]);
        st16(blk + L::kHalf, pd[k]);
      } else {                          // 16-bit: one vector = two half-blocks
        char* blk = row + 2 * c * L::kBlock;
        *reinterpret_cast<uint2*>(blk) = make_uint2(pu[k].x, pu[k].y);
        *reinterpret_cast<uint2*>(blk + L::kHalf) = make_uint2(pd[k].x, pd[k].y);
        *reinterpret_cast<uint2*>(blk + L::kBlock) = make_uint2(pu[k].z, pu[k].w);
        *reinterpret_cast<uint2*>(blk + L::kBlock + L::kHalf) = make_uint2(pd[k].z, pd[k].w);
      }
    }
#pragma unroll
    for (int k = 0; k < kBCPer; ++k) {
      const int j = tid + k * rows;
      if (j < 2 * kBCVecs) {
        const bool isC = j >= kBCVecs;
        const int jj = isC ? j - kBCVecs : j;
        const int n = jj / kBCRow, c = jj % kBCRow;
        float* dst = bc + (c * VW) * (2 * kN) + (isC ? kN : 0) + n;
        const bool live = n < a.dstate;   // padded states read B = C = 0
#pragma unroll
        for (int e = 0; e < VW; ++e) dst[e * 2 * kN] = live ? elem_f<TW>(pbc[k], e) : 0.f;
      }
    }
  };

  load_tiles(0);
  for (int ch = 0; ch < a.n_chunks; ++ch) {
    const int l0 = ch * kT;
    __syncthreads();  // previous chunk's gate pass is done with rowbuf / bc
    store_tiles_lds();
    __syncthreads();
    if (ch + 1 < a.n_chunks) load_tiles(l0 + kT);  // in flight during the recurrence

    // ---- the recurrence over this chunk, one channel per thread
    if (my_ok) {
      char* row = rowbuf + tid * L::kStride;
#pragma unroll 2
      for (int t4 = 0; t4 < kT; t4 += 4) {
        char* blk = row + (t4 / 4) * L::kBlock;
        uint4 bu, bd;   // elements 0..3 of each
        if constexpr (L::kHalf == 16) {
          bu = ld16(blk);
          bd = ld16(blk + L::kHalf);
        } else {
          const uint4 q = ld16(blk);
          bu = make_uint4(q.x, q.y, 0u, 0u);
          bd = make_uint4(q.z, q.w, 0u, 0u);
        }
        float yv[4];
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          const int t = t4 + tt;
          const float uv = elem_f<TI>(bu, tt);
          const float dr = elem_f<TI>(bd, tt) + biasv;
          float dt = softplus ? softplus_f(dr) : dr;
          dt = (l0 + t < L_) ? dt : 0.f;  // past the end: state frozen
          const float du = dt * uv;
          const float4* bct = reinterpret_cast<const float4*>(bc + t * 2 * kN);
          float y = 0.f;
#pragma unroll
          for (int n4 = 0; n4 < kN / 4; ++n4) {
            const float4 bq = bct[n4];
            const float4 cq = bct[kN / 4 + n4];
#define MC_STEP(i, BB, CC)                                \
            {                                             \
              const float dA = fast_exp2(dt * A2[n4 * 4 + i]); \
              x[n4 * 4 + i] = fmaf(dA, x[n4 * 4 + i], du * BB); \
              y = fmaf(CC, x[n4 * 4 + i], y);             \
            }
            MC_STEP(0, bq.x, cq.x)
            MC_STEP(1, bq.y, cq.y)
            MC_STEP(2, bq.z, cq.z)
            MC_STEP(3, bq.w, cq.w)
#undef MC_STEP
          }
          yv[tt] = fmaf(Dv, uv, y);
        }
        *reinterpret_cast<float4*>(blk) = make_float4(yv[0], yv[1], yv[2], yv[3]);
      }
      if (a.chunk_states) {
        float* cs = a.chunk_states + (((int64_t)b * a.dim + my_d) * a.n_chunks + ch) * a.dstate;
        if ((a.dstate & 3) == 0) {
#pragma unroll
          for (int n4 = 0; n4 < kN / 4; ++n4)
            if (n4 * 4 < a.dstate)
              reinterpret_cast<float4*>(cs)[n4] = make_float4(x[4 * n4], x[4 * n4 + 1], x[4 * n4 + 2], x[4 * n4 + 3]);
        } else {
#pragma unroll
          for (int n = 0; n < kN; ++n)
            if (n < a.dstate) cs[n] = x[n];
        }
      }
    }
    __syncthreads();

    // ---- gate + store: coalesced along the sequence
    const bool full = kAligned && (l0 + kT <= L_);
#pragma unroll
    for (int k = 0; k < kVPR; ++k) {
      const int j = tid + k * rows;
      const int r = j / kVPR, c = j % kVPR;
      const int col0 = l0 + c * VI;
      const char* yrow = rowbuf + r * L::kStride;
      const TI* zsrc = zp + (int64_t)(dbase + min(r, nrows - 1)) * a.z_ds + col0;
      const int nv = max(0, min(VI, L_ - col0));
      uint4 zv = make_uint4(0u, 0u, 0u, 0u);
      if (hasZ) zv = full ? ld16(zsrc) : ld16_masked(zsrc, nv);
      float o[VI];
#pragma unroll
      for (int e4 = 0; e4 < VI; e4 += 4) {
        const float4 yq = *reinterpret_cast<const float4*>(yrow + (c * (VI / 4) + e4 / 4) * L::kBlock);
        o[e4 + 0] = yq.x; o[e4 + 1] = yq.y; o[e4 + 2] = yq.z; o[e4 + 3] = yq.w;
      }
      if (hasZ) {
#pragma unroll
        for (int e = 0; e < VI; ++e) o[e] *= silu_f(elem_f<TI>(zv, e));
      }
      const uint4 ov = pack_f<TI>(o);
      TI* dst = out + (int64_t)(dbase + r) * a.o_ds + col0;
      if (r < nrows) {
        if (full) st16(dst, ov);
        else st16_masked(dst, ov, nv);
      }
    }
  }

  if (a.last_state && my_ok) {
    float* ls = a.last_state + ((int64_t)b * a.dim + my_d) * a.dstate;
#pragma unroll
    for (int n = 0; n < kN; ++n)
      if (n < a.dstate) ls[n] = x[n];
  }
}

// ------------------------------------------------------------------ host dispatch
template <typename TI, typename TW, int kN>
static int launch_fwd_n(const FwdArgs& a, bool aligned, hipStream_t s) {
  const int H = a.dim / a.n_groups;
  const int rows = H >= kMaxRows ? kMaxRows : ((H + 63) / 64) * 64;
  dim3 grid((H + rows - 1) / rows, a.n_groups, a.batch);
  const size_t lds = (size_t)rows * RowLayout<TI>::kStride + (size_t)kT * 2 * kN * sizeof(float);
  if (aligned)
    hipLaunchKernelGGL((scan_fwd_kernel<TI, TW, kN, true>), grid, dim3(rows), lds, s, a);
  else
    hipLaunchKernelGGL((scan_fwd_kernel<TI, TW, kN, false>), grid, dim3(rows), lds, s, a);
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_scan_fwd: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

template <typename TI, typename TW>
static int launch_fwd_t(const FwdArgs& a, bool aligned, hipStream_t s) {
  if (a.dstate <= 8) return launch_fwd_n<TI, TW, 8>(a, aligned, s);
  if (a.dstate <= 16) return launch_fwd_n<TI, TW, 16>(a, aligned, s);
  return launch_fwd_n<TI, TW, 32>(a, aligned, s);
}

}  // namespace scan
}  // namespace mc

// ------------------------------------------------------------------ C ABI
using namespace mc;
using namespace mc::scan;

extern "C" int32_t mc_scan_n_chunks(int32_t seqlen) { return seqlen <= 0 ? 0 : (seqlen + kT - 1) / kT; }

extern "C" size_t mc_scan_chunk_states_bytes(int32_t batch, int32_t dim, int32_t seqlen, int32_t dstate) {
  return (size_t)batch * dim * mc_scan_n_chunks(seqlen) * dstate * sizeof(float);
}

int mc_validate_common(int batch, int dim, int seqlen, int dstate, int n_groups, int itype, int wtype,
                       const char* who) {
  MC_CHECK(batch >= 0 && dim > 0 && seqlen >= 0, MC_ERR_SHAPE, "%s: bad shape batch=%d dim=%d seqlen=%d", who,
           batch, dim, seqlen);
  MC_CHECK(dstate >= 1 && dstate <= MC_SCAN_MAX_DSTATE, MC_ERR_SHAPE, "%s: dstate=%d must be in [1, %d]", who,
           dstate, MC_SCAN_MAX_DSTATE);
  MC_CHECK(n_groups >= 1 && dim % n_groups == 0, MC_ERR_SHAPE, "%s: dim=%d not divisible by n_groups=%d", who,
           dim, n_groups);
  MC_CHECK(itype >= MC_DTYPE_F32 && itype <= MC_DTYPE_F16, MC_ERR_DTYPE, "%s: bad input dtype %d", who, itype);
  MC_CHECK(wtype >= MC_DTYPE_F32 && wtype <= MC_DTYPE_F16, MC_ERR_DTYPE, "%s: bad weight dtype %d", who, wtype);
  return MC_OK;
}

static bool vec_ok(const void* p, int64_t s0, int64_t s1, int64_t s2, int elem_bytes) {
  const int64_t v = 16 / elem_bytes;
  return p == nullptr || (aligned16(p) && s0 % v == 0 && s1 % v == 0 && s2 % v == 0);
}

extern "C" int mc_scan_fwd(const mc_scan_fwd_params* p, void* stream) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_scan_fwd: null params");
  int rc = mc_validate_common(p->batch, p->dim, p->seqlen, p->dstate, p->n_groups, p->itype, p->wtype,
                              "mc_scan_fwd");
  if (rc) return rc;
  MC_CHECK(p->u && p->delta && p->A && p->B && p->C && p->out, MC_ERR_INVALID,
           "mc_scan_fwd: u, delta, A, B, C and out must be non-null");
  if (p->batch == 0 || p->seqlen == 0) {
    // nothing to scan; a zero-length sequence leaves the state at zero
    if (p->last_state)
      (void)hipMemsetAsync(p->last_state, 0, (size_t)p->batch * p->dim * p->dstate * 4, (hipStream_t)stream);
    return MC_OK;
  }
  FwdArgs a;
  a.batch = p->batch; a.dim = p->dim; a.seqlen = p->seqlen; a.dstate = p->dstate; a.n_groups = p->n_groups;
  a.n_chunks = mc_scan_n_chunks(p->seqlen);
  a.softplus = p->delta_softplus;
  a.u_bs = p->u_batch_stride; a.u_ds = p->u_dim_stride;
  a.dt_bs = p->delta_batch_stride; a.dt_ds = p->delta_dim_stride;
  a.z_bs = p->z_batch_stride; a.z_ds = p->z_dim_stride;
  a.o_bs = p->out_batch_stride; a.o_ds = p->out_dim_stride;
  a.B_bs = p->B_batch_stride; a.B_gs = p->B_group_stride; a.B_ns = p->B_dstate_stride;
  a.C_bs = p->C_batch_stride; a.C_gs = p->C_group_stride; a.C_ns = p->C_dstate_stride;
  a.u = p->u; a.delta = p->delta; a.A = p->A; a.B = p->B; a.C = p->C; a.D = p->D; a.z = p->z;
  a.delta_bias = p->delta_bias; a.out = p->out; a.chunk_states = p->chunk_states; a.last_state = p->last_state;

  const int ib = p->itype == MC_DTYPE_F32 ? 4 : 2;
  const int wb = p->wtype == MC_DTYPE_F32 ? 4 : 2;
  const bool aligned = vec_ok(p->u, p->u_batch_stride, p->u_dim_stride, 0, ib) &&
                       vec_ok(p->delta, p->delta_batch_stride, p->delta_dim_stride, 0, ib) &&
                       vec_ok(p->z, p->z_batch_stride, p->z_dim_stride, 0, ib) &&
                       vec_ok(p->out, p->out_batch_stride, p->out_dim_stride, 0, ib) &&
                       vec_ok(p->B, p->B_batch_stride, p->B_group_stride, p->B_dstate_stride, wb) &&
                       vec_ok(p->C, p->C_batch_stride, p->C_group_stride, p->C_dstate_stride, wb);
  hipStream_t s = (hipStream_t)stream;
  const int it = p->itype, wt = p->wtype;
  if (it == MC_DTYPE_F32 && wt == MC_DTYPE_F32) return launch_fwd_t<float, float>(a, aligned, s);
  if (it == MC_DTYPE_F32 && wt == MC_DTYPE_BF16) return launch_fwd_t<float, bf16_t>(a, aligned, s);
  if (it == MC_DTYPE_BF16 && wt == MC_DTYPE_BF16) return launch_fwd_t<bf16_t, bf16_t>(a, aligned, s);
  if (it == MC_DTYPE_BF16 && wt == MC_DTYPE_F32) return launch_fwd_t<bf16_t, float>(a, aligned, s);
  if (it == MC_DTYPE_F16 && wt == MC_DTYPE_F16) return launch_fwd_t<f16_t, f16_t>(a, aligned, s);
  if (it == MC_DTYPE_F16 && wt == MC_DTYPE_F32) return launch_fwd_t<f16_t, float>(a, aligned, s);
  MC_CHECK(false, MC_ERR_DTYPE, "mc_scan_fwd: unsupported dtype combination itype=%d wtype=%d", it, wt);
}
