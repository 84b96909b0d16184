// scan_bwd.hip -- selective-scan backward for MI355X (gfx950, CDNA4).
//
// Reverse-mode of the recurrence in scan_fwd.hip (reference semantics
// /root/reference/src/mamba_clip/model.py:83-169; the op behind
// selective_scan_cuda.bwd reached through mamba_ssm's SelectiveScanFn):
//   gy_t  = dout_t * silu(z_t)                  dz_t = dout_t * y_t * silu'(z_t)
//   h_t,n = C_t,n gy_t + a_{t+1,n} h_{t+1,n}     (adjoint of the state, a = exp(dt A))
//   dC_t,n = sum_d gy_t x_t,n        dB_t,n = sum_d h_t,n dt_t u_t
//   du_t  = D gy_t + sum_n h_t,n dt_t B_t,n
//   ddt_t = sum_n h_t,n (A_n a_t,n x_{t-1,n} + B_t,n u_t),  ddelta_t = ddt_t * sigmoid(delta_t + bias)
//   dA_n  = sum_{b,t} h_t,n dt_t a_t,n x_{t-1,n}    dD = sum gy u    dbias = sum ddelta
//
// Design (DESIGN.md "scan_bwd"):
//  * one wave = 64 channels of one (batch, group); tiles of kS = 16 positions
//    walked in reverse; each tile restarts from the fp32 state the training
//    forward saved at its start (chunk_states), so nothing is recomputed
//    across tiles.
//  * inside a tile the state index n is the outer (fully unrolled) loop: a
//    forward sweep keeps x_t,n and a_t,n for the 16 positions in VGPRs, the
//    reverse sweep consumes them; per-position accumulators (du, ddt, y) stay
//    in VGPRs across n.
//  * dB/dC (sums over the 64 channels of the wave) use an in-register
//    transpose-reduce: permlane32_swap / permlane16_swap / DPP row_ror:8 /
//    ds_swizzle / quad_perm halving stages turn 32 per-lane values into 32 wave sums in
//    ~2 VALU per value, then land in a per-wave fp32 slab.  A small second
//    kernel sums the slabs over waves / batches: deterministic, no atomics.
#include "scan_common.h"

namespace mc {
namespace scan {

constexpr int kTB = kS;  // positions per backward tile (== saved-state granularity)

struct BwdArgs {
  int batch, dim, seqlen, dstate, n_groups, n_states, nblk, total_blocks, softplus;
  int64_t u_bs, u_ds, dt_bs, dt_ds, z_bs, z_ds, go_bs, go_ds;
  int64_t du_bs, du_ds, ddt_bs, ddt_ds, dz_bs, dz_ds;  // output strides (seqlen stride 1)
  const void* u; const void* delta; const void* z; const void* dout;
  const float* A; const float* bct; const float* D; const float* delta_bias;
  const float* chunk_states;
  void* du; void* ddelta; void* dz;
  float* slab_bc;                    // [b*G+g][nblk][kN][2][seqlen]
  float* slab_a;                     // [b][dim][kN]
  float* slab_d;                     // [b][dim]
  float* slab_bias;                  // [b][dim]
};

__device__ __forceinline__ float dpp_f(float v, int ctrl_sel) {
  // ctrl_sel: 0 -> row_ror:8 (xor 8), 1 -> ds_swizzle xor 4, 2 -> quad_perm[2,3,0,1] (xor 2),
  // 3 -> quad_perm[1,0,3,2] (xor 1).  Every partner is lane ^ bit exactly: the
  // halving stages need partners that agree on the bits already reduced
  // (row_ror:4 is NOT xor 4 -- it can flip bit 3; tools/ubench/reduce_check.hip).
  const int iv = __float_as_int(v);
  int r;
  if (ctrl_sel == 0) r = __builtin_amdgcn_update_dpp(iv, iv, 0x128, 0xF, 0xF, false);
  else if (ctrl_sel == 1) r = __builtin_amdgcn_ds_swizzle(iv, 0x101F);  // bitmask mode: and 0x1F, xor 4
  else if (ctrl_sel == 2) r = __builtin_amdgcn_update_dpp(iv, iv, 0x4E, 0xF, 0xF, false);
  else r = __builtin_amdgcn_update_dpp(iv, iv, 0xB1, 0xF, 0xF, false);
  return __int_as_float(r);
}

// 32 per-lane values -> 32 sums over the wave's 64 lanes.  Afterwards lane l
// holds the sum of value index l >> 1 (both lanes of a pair hold it).
__device__ __forceinline__ float wave_transpose_reduce32(float (&v)[32], int lane) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {  // bit 5: lanes 0-31 keep [0,16), lanes 32-63 keep [16,32)
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j]), __float_as_uint(v[j + 16]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {   // bit 4: even 16-lane rows keep [0,8), odd rows keep [8,16)
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[j]), __float_as_uint(v[j + 8]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2;
#pragma unroll
  for (int j = 0; j < 4; ++j) {   // bit 3 via row_ror:8 (== xor 8 inside a row)
    const float keep = b3 ? v[j + 4] : v[j], send = b3 ? v[j] : v[j + 4];
    v[j] = keep + dpp_f(send, 0);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {   // bit 2 via ds_swizzle xor 4
    const float keep = b2 ? v[j + 2] : v[j], send = b2 ? v[j] : v[j + 2];
    v[j] = keep + dpp_f(send, 1);
  }
  {                               // bit 1 via quad_perm [2,3,0,1]
    const float keep = b1 ? v[1] : v[0], send = b1 ? v[0] : v[1];
    v[0] = keep + dpp_f(send, 2);
  }
  return v[0] + dpp_f(v[0], 3);  // bit 0 via quad_perm [1,0,3,2]
}

// Raw row (staging) and processed row share one LDS region per lane.
template <typename TI>
struct BwdRow {
  static constexpr int kRawArr = kTB * (int)sizeof(TI);  // bytes of one raw array segment
  static constexpr int kRawBytes = 4 * kRawArr;          // u, delta, z, dout
  static constexpr int kProcBytes = 4 * kTB * 4;         // 4 fp32 arrays of kTB
  static constexpr int kBytes = kRawBytes > kProcBytes ? kRawBytes : kProcBytes;
  static constexpr int kStride = kBytes + 16;
};

template <typename TI, int kN, bool kAligned>
__global__ __launch_bounds__(kRows, 2) void scan_bwd_kernel(const BwdArgs a) {
  using RW = BwdRow<TI>;
  constexpr int VI = ElemTraits<TI>::kVec;
  constexpr int kVPR = kTB / VI;        // 16-B vectors per raw row segment (2 for 16-bit, 4 for fp32)

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* rowbuf = smem;                                                  // [64][kStride]
  float* bcT = reinterpret_cast<float*>(smem + kRows * RW::kStride);    // [2kN][kTB]: B rows then C rows
  // per-lane, per-state scalars, [slot][n][lane] (lane-minor: conflict-free):
  // slot 0 = A*log2e, 1 = tile start state, 2 = adjoint carry, 3 = dA accumulator
  float* lst = bcT + 2 * kN * kTB;

  const int lane = threadIdx.x;
  const int lin = xcd_remap(blockIdx.x, a.total_blocks);
  const int dblk = lin % a.nblk;
  const int bg = lin / a.nblk;
  const int g = bg % a.n_groups, b = bg / a.n_groups;
  const int H = a.dim / a.n_groups;
  const int dbase = g * H + dblk * kRows;
  const int nrows = min(kRows, H - dblk * kRows);
  const int L_ = a.seqlen;
  const bool hasZ = a.z != nullptr;
  const bool softplus = a.softplus != 0;
  const int my_d = dbase + lane;
  const bool my_ok = lane < nrows;
  const int my_dc = dbase + min(lane, nrows - 1);

  const TI* __restrict__ u = reinterpret_cast<const TI*>(a.u) + (int64_t)b * a.u_bs;
  const TI* __restrict__ dl = reinterpret_cast<const TI*>(a.delta) + (int64_t)b * a.dt_bs;
  const TI* __restrict__ zp = reinterpret_cast<const TI*>(a.z) + (int64_t)b * a.z_bs;
  const TI* __restrict__ gop = reinterpret_cast<const TI*>(a.dout) + (int64_t)b * a.go_bs;

#pragma unroll
  for (int n = 0; n < kN; ++n) {
    lst[(0 * kN + n) * kRows + lane] = (n < a.dstate) ? a.A[(int64_t)my_dc * a.dstate + n] * kLog2e : 0.f;
    lst[(2 * kN + n) * kRows + lane] = 0.f;
    lst[(3 * kN + n) * kRows + lane] = 0.f;
  }
  const float Dv = a.D ? a.D[my_dc] : 0.f;
  const float biasv = a.delta_bias ? a.delta_bias[my_dc] : 0.f;
  float dDacc = 0.f, dbacc = 0.f;

  const int ntiles = (L_ + kTB - 1) / kTB;
  for (int ti = ntiles - 1; ti >= 0; --ti) {
    const int l0 = ti * kTB;
    const bool full = kAligned && (l0 + kTB <= L_);
    __syncthreads();  // previous tile's output pass is done with the rows

    // ---- stage raw u / delta / z / dout (coalesced along the sequence)
#pragma unroll
    for (int k = 0; k < kVPR; ++k) {
      const int j = lane + k * kRows;
      const int r = j / kVPR, c = j % kVPR;
      const int rr = min(r, nrows - 1);
      const int col0 = l0 + c * VI;
      const int nv = max(0, min(VI, L_ - col0));
      const int64_t ro = dbase + rr;
      const TI* s0 = u + ro * a.u_ds + col0;
      const TI* s1 = dl + ro * a.dt_ds + col0;
      const TI* s2 = zp + ro * a.z_ds + col0;
      const TI* s3 = gop + ro * a.go_ds + col0;
      const uint4 q0 = full ? ld16(s0) : ld16_masked(s0, nv);
      const uint4 q1 = full ? ld16(s1) : ld16_masked(s1, nv);
      const uint4 q2 = hasZ ? (full ? ld16(s2) : ld16_masked(s2, nv)) : make_uint4(0u, 0u, 0u, 0u);
      const uint4 q3 = full ? ld16(s3) : ld16_masked(s3, nv);
      char* row = rowbuf + r * RW::kStride + c * 16;
      st16(row, q0);
      st16(row + RW::kRawArr, q1);
      st16(row + 2 * RW::kRawArr, q2);
      st16(row + 3 * RW::kRawArr, q3);
    }
    // ---- B/C tile, transposed to [2kN][kTB] (per-n rows of positions)
    {
      const float* src = a.bct + ((int64_t)bg * L_ + l0) * (2 * kN);
      const int nval = min(kTB, L_ - l0) * (2 * kN);
      for (int v = lane; v < kTB * 2 * kN; v += kRows) {
        const int t = v / (2 * kN), jn = v % (2 * kN);
        bcT[jn * kTB + t] = v < nval ? src[v] : 0.f;
      }
    }
    __syncthreads();

    // ---- per-position scalars of my channel
    float dt[kTB], uu[kTB], gy[kTB];
    float* prow = reinterpret_cast<float*>(rowbuf + lane * RW::kStride);  // processed: gz @ [2kTB], sg @ [3kTB]
    {
      const char* row = rowbuf + lane * RW::kStride;
      uint4 ru[kVPR], rd[kVPR], rz[kVPR], rg[kVPR];
#pragma unroll
      for (int k = 0; k < kVPR; ++k) {
        ru[k] = ld16(row + k * 16);
        rd[k] = ld16(row + RW::kRawArr + k * 16);
        rz[k] = ld16(row + 2 * RW::kRawArr + k * 16);
        rg[k] = ld16(row + 3 * RW::kRawArr + k * 16);
      }
      float gz[kTB], sg[kTB];
#pragma unroll
      for (int t = 0; t < kTB; ++t) {
        const float uv = elem_f<TI>(ru[t / VI], t % VI);
        const float r = elem_f<TI>(rd[t / VI], t % VI) + biasv;
        const float go = elem_f<TI>(rg[t / VI], t % VI);
        const bool live = l0 + t < L_;
        float d = softplus ? softplus_f(r) : r;
        // d softplus/dr = sigmoid(r) (torch: grad 1 above the threshold 20)
        float s = softplus ? (r > 20.f ? 1.f : sigmoid_f(r)) : 1.f;
        d = live ? d : 0.f;
        dt[t] = d;
        sg[t] = s;
        uu[t] = uv;
        if (hasZ) {
          const float zv = elem_f<TI>(rz[t / VI], t % VI);
          const float sgz = sigmoid_f(zv);
          gy[t] = go * zv * sgz;                                   // dout * silu(z)
          gz[t] = go * sgz * (1.f + zv * (1.f - sgz));             // dout * silu'(z)
        } else {
          gy[t] = go;
          gz[t] = 0.f;
        }
      }
      // all lanes' raw reads precede these writes (one wave, program order)
#pragma unroll
      for (int t4 = 0; t4 < kTB; t4 += 4) {
        *reinterpret_cast<float4*>(prow + 2 * kTB + t4) = make_float4(gz[t4], gz[t4 + 1], gz[t4 + 2], gz[t4 + 3]);
        *reinterpret_cast<float4*>(prow + 3 * kTB + t4) = make_float4(sg[t4], sg[t4 + 1], sg[t4 + 2], sg[t4 + 3]);
      }
    }

    // ---- tile start state (saved by the forward), zero for the first tile
    {
      const float* cs = a.chunk_states + (((int64_t)b * a.dim + my_dc) * a.n_states + max(ti - 1, 0)) * a.dstate;
#pragma unroll
      for (int n = 0; n < kN; ++n) lst[(1 * kN + n) * kRows + lane] = (ti > 0 && n < a.dstate) ? cs[n] : 0.f;
    }

    float ys[kTB], du[kTB], ddt[kTB];
#pragma unroll
    for (int t = 0; t < kTB; ++t) { ys[t] = 0.f; du[t] = 0.f; ddt[t] = 0.f; }

#pragma unroll 1
    for (int n = 0; n < kN; ++n) {
      const float A2n = lst[(0 * kN + n) * kRows + lane];
      const float x0n = lst[(1 * kN + n) * kRows + lane];
      float Bn[kTB], Cn[kTB];
#pragma unroll
      for (int t4 = 0; t4 < kTB; t4 += 4) {
        const float4 bq = *reinterpret_cast<const float4*>(bcT + n * kTB + t4);
        const float4 cq = *reinterpret_cast<const float4*>(bcT + (kN + n) * kTB + t4);
        Bn[t4] = bq.x; Bn[t4 + 1] = bq.y; Bn[t4 + 2] = bq.z; Bn[t4 + 3] = bq.w;
        Cn[t4] = cq.x; Cn[t4 + 1] = cq.y; Cn[t4 + 2] = cq.z; Cn[t4 + 3] = cq.w;
      }
      const float An = A2n * kLn2;
      // forward sweep: states and decays of this tile
      float xs[kTB], as[kTB];
      float x = x0n;
#pragma unroll
      for (int t = 0; t < kTB; ++t) {
        const float aa = fast_exp2(dt[t] * A2n);
        x = fmaf(aa, x, dt[t] * uu[t] * Bn[t]);
        xs[t] = x;
        as[t] = aa;
        ys[t] = fmaf(Cn[t], x, ys[t]);
      }
      // reverse sweep
      float h = lst[(2 * kN + n) * kRows + lane];
      float red[32];
      float dAn = 0.f;
#pragma unroll
      for (int t = kTB - 1; t >= 0; --t) {
        h = fmaf(Cn[t], gy[t], h);
        const float xp = t > 0 ? xs[t - 1] : x0n;
        const float hdt = h * dt[t];
        red[t] = hdt * uu[t];              // dB_t,n contribution
        red[kTB + t] = gy[t] * xs[t];      // dC_t,n contribution
        du[t] = fmaf(hdt, Bn[t], du[t]);
        const float hax = h * as[t] * xp;
        ddt[t] = fmaf(An, hax, fmaf(h * Bn[t], uu[t], ddt[t]));
        dAn = fmaf(hax, dt[t], dAn);
        h *= as[t];
      }
      lst[(2 * kN + n) * kRows + lane] = h;
      lst[(3 * kN + n) * kRows + lane] += my_ok ? dAn : 0.f;
      // channel sums of dB / dC for (n, 16 positions): lanes past the group end contribute 0
      if (!my_ok) {
#pragma unroll
        for (int i = 0; i < 32; ++i) red[i] = 0.f;
      }
      const float tot = wave_transpose_reduce32(red, lane);
      if ((lane & 1) == 0 && n < a.dstate) {
        const int k = lane >> 1;
        const int which = k >> 4, t = k & 15;
        if (l0 + t < L_)
          a.slab_bc[((((int64_t)bg * a.nblk + dblk) * kN + n) * 2 + which) * L_ + l0 + t] = tot;
      }
    }

    // ---- per-position outputs of my channel -> rows (fp32), then coalesced stores
    {
      float gz[kTB], sg[kTB];
#pragma unroll
      for (int t4 = 0; t4 < kTB; t4 += 4) {
        const float4 a4 = *reinterpret_cast<const float4*>(prow + 2 * kTB + t4);
        const float4 b4 = *reinterpret_cast<const float4*>(prow + 3 * kTB + t4);
        gz[t4] = a4.x; gz[t4 + 1] = a4.y; gz[t4 + 2] = a4.z; gz[t4 + 3] = a4.w;
        sg[t4] = b4.x; sg[t4 + 1] = b4.y; sg[t4 + 2] = b4.z; sg[t4 + 3] = b4.w;
      }
      float o_du[kTB], o_dd[kTB], o_dz[kTB];
#pragma unroll
      for (int t = 0; t < kTB; ++t) {
        const bool live = l0 + t < L_;
        const float y = fmaf(Dv, uu[t], ys[t]);
        o_dz[t] = gz[t] * y;
        o_du[t] = fmaf(Dv, gy[t], du[t]);
        const float dr = ddt[t] * sg[t];
        o_dd[t] = dr;
        if (live && my_ok) {
          dDacc = fmaf(gy[t], uu[t], dDacc);
          dbacc += dr;
        }
      }
#pragma unroll
      for (int t4 = 0; t4 < kTB; t4 += 4) {
        *reinterpret_cast<float4*>(prow + t4) = make_float4(o_du[t4], o_du[t4 + 1], o_du[t4 + 2], o_du[t4 + 3]);
        *reinterpret_cast<float4*>(prow + kTB + t4) = make_float4(o_dd[t4], o_dd[t4 + 1], o_dd[t4 + 2], o_dd[t4 + 3]);
        *reinterpret_cast<float4*>(prow + 2 * kTB + t4) = make_float4(o_dz[t4], o_dz[t4 + 1], o_dz[t4 + 2], o_dz[t4 + 3]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kVPR; ++k) {
      const int j = lane + k * kRows;
      const int r = j / kVPR, c = j % kVPR;
      if (r >= nrows) continue;
      const int col0 = l0 + c * VI;
      const int nv = max(0, min(VI, L_ - col0));
      const float* src = reinterpret_cast<const float*>(rowbuf + r * RW::kStride);
      const int64_t dd = dbase + r;
#pragma unroll
      for (int which = 0; which < 3; ++which) {
        if (which == 2 && !hasZ) continue;
        float v[VI];
#pragma unroll
        for (int e = 0; e < VI; ++e) v[e] = src[which * kTB + c * VI + e];
        const int64_t off = which == 0   ? (int64_t)b * a.du_bs + dd * a.du_ds
                            : which == 1 ? (int64_t)b * a.ddt_bs + dd * a.ddt_ds
                                         : (int64_t)b * a.dz_bs + dd * a.dz_ds;
        TI* dst = reinterpret_cast<TI*>(which == 0 ? a.du : (which == 1 ? a.ddelta : a.dz)) + off + col0;
        const uint4 q = pack_f<TI>(v);
        if (full) st16(dst, q);
        else st16_masked(dst, q, nv);
      }
    }
  }

  if (my_ok) {
#pragma unroll
    for (int n = 0; n < kN; ++n) a.slab_a[((int64_t)b * a.dim + my_d) * kN + n] = lst[(3 * kN + n) * kRows + lane];
    a.slab_d[(int64_t)b * a.dim + my_d] = dDacc;
    a.slab_bias[(int64_t)b * a.dim + my_d] = dbacc;
  }
}

// dB / dC: sum the per-wave slabs; dA / dD / dbias: sum the per-batch slabs.
template <typename TW, int kN>
__global__ __launch_bounds__(256) void scan_bwd_reduce_bc(const float* __restrict__ slab, int batch, int G, int nblk,
                                                           int dstate, int L, TW* __restrict__ dB, TW* __restrict__ dC) {
  const int64_t total = (int64_t)batch * G * dstate * 2 * L;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(i % L);
    int64_t r = i / L;
    const int which = (int)(r % 2);
    r /= 2;
    const int n = (int)(r % dstate);
    const int64_t bgi = r / dstate;
    float s = 0.f;
    for (int k = 0; k < nblk; ++k) s += slab[(((bgi * nblk + k) * kN + n) * 2 + which) * L + l];
    TW* dst = which ? dC : dB;
    dst[(bgi * dstate + n) * L + l] = from_f<TW>(s);
  }
}

// Column sums over the batch: out[c] = sum_b in[b][c] (row stride ld).  A
// block = 32 columns x 8 batch lanes; the 8 partials meet in LDS in a fixed
// order (deterministic).  Used for dA (cols = (d, n)), dD and dbias (cols = d).
__global__ __launch_bounds__(256) void scan_bwd_colsum(const float* __restrict__ in, int batch, int cols, int64_t ld,
                                                       int out_cols, int col_div, int col_mod, float* __restrict__ out) {
  __shared__ float part[8][33];
  const int cx = threadIdx.x & 31, q = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cx;
  float s = 0.f;
  if (c < cols)
    for (int bb = q; bb < batch; bb += 8) s += in[(int64_t)bb * ld + c];
  part[q][cx] = s;
  __syncthreads();
  if (q == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += part[k][cx];
    // column c of the slab -> output index (drop padded states: c = d*col_div + n, keep n < col_mod)
    const int d = c / col_div, n = c % col_div;
    if (n < col_mod) out[(int64_t)d * col_mod + n] = t;
  }
  (void)out_cols;
}

struct BwdWs {
  size_t bct, slab_bc, slab_a, slab_d, slab_bias, total;
};
static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
static BwdWs bwd_ws_layout(int batch, int dim, int seqlen, int dstate, int G) {
  const int np = padded_dstate(dstate);
  const int nblk = (dim / G + kRows - 1) / kRows;
  BwdWs w;
  size_t o = 0;
  w.bct = o; o += align256(bct_bytes(batch, seqlen, dstate, G));
  w.slab_bc = o; o += align256((size_t)batch * G * nblk * np * 2 * seqlen * 4);
  w.slab_a = o; o += align256((size_t)batch * dim * np * 4);
  w.slab_d = o; o += align256((size_t)batch * dim * 4);
  w.slab_bias = o; o += align256((size_t)batch * dim * 4);
  w.total = o;
  return w;
}

template <typename TI, int kN>
static int launch_bwd_n(const BwdArgs& a, bool aligned, hipStream_t s) {
  const size_t lds = (size_t)kRows * BwdRow<TI>::kStride + (size_t)2 * kN * kTB * 4 + (size_t)4 * kN * kRows * 4;
  if (aligned)
    hipLaunchKernelGGL((scan_bwd_kernel<TI, kN, true>), dim3(a.total_blocks), dim3(kRows), lds, s, a);
  else
    hipLaunchKernelGGL((scan_bwd_kernel<TI, kN, false>), dim3(a.total_blocks), dim3(kRows), lds, s, a);
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_scan_bwd: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

template <typename TI>
static int launch_bwd_t(const BwdArgs& a, bool aligned, hipStream_t s) {
  const int np = padded_dstate(a.dstate);
  if (np == 8) return launch_bwd_n<TI, 8>(a, aligned, s);
  if (np == 16) return launch_bwd_n<TI, 16>(a, aligned, s);
  return launch_bwd_n<TI, 32>(a, aligned, s);
}

template <typename TW, int kN>
static void launch_reduce(const BwdArgs& a, void* dB, void* dC, float* dA, float* dD, float* dbias, hipStream_t s) {
  const int64_t total = (int64_t)a.batch * a.n_groups * a.dstate * 2 * a.seqlen;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL((scan_bwd_reduce_bc<TW, kN>), dim3(grid), dim3(256), 0, s, a.slab_bc, a.batch, a.n_groups,
                     a.nblk, a.dstate, a.seqlen, reinterpret_cast<TW*>(dB), reinterpret_cast<TW*>(dC));
  const int ca = a.dim * kN;
  hipLaunchKernelGGL(scan_bwd_colsum, dim3((ca + 31) / 32), dim3(256), 0, s, a.slab_a, a.batch, ca, (int64_t)ca,
                     a.dim * a.dstate, kN, a.dstate, dA);
  if (dD)
    hipLaunchKernelGGL(scan_bwd_colsum, dim3((a.dim + 31) / 32), dim3(256), 0, s, a.slab_d, a.batch, a.dim,
                       (int64_t)a.dim, a.dim, 1, 1, dD);
  if (dbias)
    hipLaunchKernelGGL(scan_bwd_colsum, dim3((a.dim + 31) / 32), dim3(256), 0, s, a.slab_bias, a.batch, a.dim,
                       (int64_t)a.dim, a.dim, 1, 1, dbias);
}

template <typename TW>
static void launch_reduce_t(const BwdArgs& a, void* dB, void* dC, float* dA, float* dD, float* dbias, hipStream_t s) {
  const int np = padded_dstate(a.dstate);
  if (np == 8) launch_reduce<TW, 8>(a, dB, dC, dA, dD, dbias, s);
  else if (np == 16) launch_reduce<TW, 16>(a, dB, dC, dA, dD, dbias, s);
  else launch_reduce<TW, 32>(a, dB, dC, dA, dD, dbias, s);
}

}  // namespace scan
}  // namespace mc

using namespace mc;
using namespace mc::scan;

extern "C" size_t mc_scan_bwd_workspace_bytes(int32_t batch, int32_t dim, int32_t seqlen, int32_t dstate,
                                              int32_t n_groups) {
  if (batch <= 0 || dim <= 0 || seqlen <= 0 || dstate <= 0 || n_groups <= 0 || dim % n_groups) return 0;
  return bwd_ws_layout(batch, dim, seqlen, dstate, n_groups).total;
}

extern "C" int mc_scan_bwd(const mc_scan_bwd_params* p, void* stream) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_scan_bwd: null params");
  int rc = validate_common(p->batch, p->dim, p->seqlen, p->dstate, p->n_groups, p->itype, p->wtype, "mc_scan_bwd");
  if (rc) return rc;
  MC_CHECK(p->A && p->dA, MC_ERR_INVALID, "mc_scan_bwd: A and dA must be non-null");
  MC_CHECK(!p->D || p->dD, MC_ERR_INVALID, "mc_scan_bwd: dD required when D is given");
  MC_CHECK(!p->delta_bias || p->ddelta_bias, MC_ERR_INVALID, "mc_scan_bwd: ddelta_bias required with delta_bias");
  hipStream_t s = (hipStream_t)stream;
  const int np = padded_dstate(p->dstate);
  if (p->batch == 0 || p->seqlen == 0) {
    // no positions: parameter gradients are zero, per-position gradients are empty
    (void)hipMemsetAsync(p->dA, 0, (size_t)p->dim * p->dstate * 4, s);
    if (p->dD) (void)hipMemsetAsync(p->dD, 0, (size_t)p->dim * 4, s);
    if (p->ddelta_bias) (void)hipMemsetAsync(p->ddelta_bias, 0, (size_t)p->dim * 4, s);
    return MC_OK;
  }
  MC_CHECK(p->u && p->delta && p->B && p->C && p->dout && p->du && p->ddelta && p->dB && p->dC, MC_ERR_INVALID,
           "mc_scan_bwd: u, delta, B, C, dout and du, ddelta, dB, dC must be non-null");
  MC_CHECK(!p->z || p->dz, MC_ERR_INVALID, "mc_scan_bwd: dz required when z is given");
  MC_CHECK(p->chunk_states, MC_ERR_INVALID, "mc_scan_bwd: chunk_states (from the training forward) required");
  const BwdWs w = bwd_ws_layout(p->batch, p->dim, p->seqlen, p->dstate, p->n_groups);
  MC_CHECK(p->workspace && p->workspace_bytes >= w.total && (reinterpret_cast<uintptr_t>(p->workspace) & 255) == 0,
           MC_ERR_WORKSPACE, "mc_scan_bwd: workspace must be >= %zu bytes and 256-B aligned (got %zu)", w.total,
           p->workspace_bytes);
  char* ws = reinterpret_cast<char*>(p->workspace);
  hipError_t e = relayout_bc(p->wtype, p->B, p->C, p->B_batch_stride, p->B_group_stride, p->B_dstate_stride,
                             p->C_batch_stride, p->C_group_stride, p->C_dstate_stride, p->batch, p->n_groups,
                             p->seqlen, p->dstate, reinterpret_cast<float*>(ws + w.bct), s);
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_scan_bwd: B/C relayout launch failed: %s", hipGetErrorString(e));

  BwdArgs a;
  a.batch = p->batch; a.dim = p->dim; a.seqlen = p->seqlen; a.dstate = p->dstate; a.n_groups = p->n_groups;
  a.n_states = mc_scan_n_chunks(p->seqlen);
  const int H = p->dim / p->n_groups;
  a.nblk = (H + kRows - 1) / kRows;
  a.total_blocks = p->batch * p->n_groups * a.nblk;
  a.softplus = p->delta_softplus;
  a.u_bs = p->u_batch_stride; a.u_ds = p->u_dim_stride;
  a.dt_bs = p->delta_batch_stride; a.dt_ds = p->delta_dim_stride;
  a.z_bs = p->z_batch_stride; a.z_ds = p->z_dim_stride;
  a.go_bs = p->dout_batch_stride; a.go_ds = p->dout_dim_stride;
  a.u = p->u; a.delta = p->delta; a.z = p->z; a.dout = p->dout;
  a.A = p->A; a.bct = reinterpret_cast<const float*>(ws + w.bct); a.D = p->D; a.delta_bias = p->delta_bias;
  a.chunk_states = p->chunk_states;
  a.du = p->du; a.ddelta = p->ddelta; a.dz = p->dz;
  a.du_bs = p->du_batch_stride; a.du_ds = p->du_dim_stride;
  a.ddt_bs = p->ddelta_batch_stride; a.ddt_ds = p->ddelta_dim_stride;
  a.dz_bs = p->dz_batch_stride; a.dz_ds = p->dz_dim_stride;
  a.slab_bc = reinterpret_cast<float*>(ws + w.slab_bc);
  a.slab_a = reinterpret_cast<float*>(ws + w.slab_a);
  a.slab_d = reinterpret_cast<float*>(ws + w.slab_d);
  a.slab_bias = reinterpret_cast<float*>(ws + w.slab_bias);
  (void)np;

  const int ib = p->itype == MC_DTYPE_F32 ? 4 : 2;
  // outputs are contiguous: the vector path also needs 16-B aligned rows there
  const bool aligned = vec_ok(p->u, p->u_batch_stride, p->u_dim_stride, 0, ib) &&
                       vec_ok(p->delta, p->delta_batch_stride, p->delta_dim_stride, 0, ib) &&
                       vec_ok(p->z, p->z_batch_stride, p->z_dim_stride, 0, ib) &&
                       vec_ok(p->dout, p->dout_batch_stride, p->dout_dim_stride, 0, ib) &&
                       vec_ok(p->du, p->du_batch_stride, p->du_dim_stride, 0, ib) &&
                       vec_ok(p->ddelta, p->ddelta_batch_stride, p->ddelta_dim_stride, 0, ib) &&
                       vec_ok(p->dz, p->dz_batch_stride, p->dz_dim_stride, 0, ib);
  if (p->itype == MC_DTYPE_F32) rc = launch_bwd_t<float>(a, aligned, s);
  else if (p->itype == MC_DTYPE_BF16) rc = launch_bwd_t<bf16_t>(a, aligned, s);
  else rc = launch_bwd_t<f16_t>(a, aligned, s);
  if (rc) return rc;
  if (p->wtype == MC_DTYPE_F32) launch_reduce_t<float>(a, p->dB, p->dC, p->dA, p->dD, p->ddelta_bias, s);
  else if (p->wtype == MC_DTYPE_BF16) launch_reduce_t<bf16_t>(a, p->dB, p->dC, p->dA, p->dD, p->ddelta_bias, s);
  else launch_reduce_t<f16_t>(a, p->dB, p->dC, p->dA, p->dD, p->ddelta_bias, s);
  e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_scan_bwd: reduce launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}
