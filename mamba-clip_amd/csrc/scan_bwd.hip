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
//  * each lane reads / writes its own row's positions as 16-B vectors (no
//    LDS staging of the rows).  LDS holds the B/C tile and the per-lane,
//    per-state scalars (A, tile-start state, mid-tile state, adjoint carry;
//    18 KB per wave at dstate 16) so the n-loop never waits on global memory.
//  * the n-loop runs on 8-position sub-tiles (register budget); the state at
//    the middle of a 16-position tile is recomputed from the saved tile-start
//    state by a short forward pre-pass.
//  * inside a tile the state index n is the outer loop: a forward sweep keeps
//    x_t,n and a_t,n for the 16 positions in VGPRs, the reverse sweep consumes
//    them; per-position accumulators stay in VGPRs across n:
//      S_t = sum_n h B,  Q_t = sum_n h A a x_{t-1},  y_t = sum_n C x
//    so du = dt S + D gy and ddt = Q + u S need no per-n work.
//  * dB/dC (sums over the 64 channels of the wave) use an in-register
//    transpose-reduce: permlane32_swap / permlane16_swap / DPP row_ror:8 /
//    ds_swizzle / quad_perm halving stages turn 16 per-lane values into 16
//    wave sums in ~2 VALU per value, then land in a per-wave fp32 slab.  A
//    small second kernel sums the slabs over waves / batches: deterministic,
//    no atomics.
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
  float* slab_a;                     // [b][kN][dim] (dA partials, one owner per element)
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

// NV per-lane values -> NV sums over the wave's 64 lanes (NV in {8, 16, 32}).
// Halving stages over lane bits 5, 4, 3, ... pair value j with j + NV/2^k;
// the remaining low lane bits are summed in full.  Afterwards lane l holds
// the sum of value index l / (64 / NV).
template <int NV>
__device__ __forceinline__ float wave_transpose_reduce(float (&v)[NV], int lane) {
  static_assert(NV == 8 || NV == 16 || NV == 32, "NV in {8, 16, 32}");
#pragma unroll
  for (int j = 0; j < NV / 2; ++j) {   // lane bit 5
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j]), __float_as_uint(v[j + NV / 2]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int j = 0; j < NV / 4; ++j) {   // lane bit 4
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[j]), __float_as_uint(v[j + NV / 4]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2;
#pragma unroll
  for (int j = 0; j < NV / 8; ++j) {   // lane bit 3 via row_ror:8 (== xor 8 inside a row)
    const float keep = b3 ? v[j + NV / 8] : v[j], send = b3 ? v[j] : v[j + NV / 8];
    v[j] = keep + dpp_f(send, 0);
  }
  if constexpr (NV >= 16) {
#pragma unroll
    for (int j = 0; j < NV / 16; ++j) {   // lane bit 2 via ds_swizzle xor 4
      const float keep = b2 ? v[j + NV / 16] : v[j], send = b2 ? v[j] : v[j + NV / 16];
      v[j] = keep + dpp_f(send, 1);
    }
  } else {
    v[0] += dpp_f(v[0], 1);
  }
  if constexpr (NV >= 32) {             // lane bit 1 via quad_perm [2,3,0,1]
    const float keep = b1 ? v[1] : v[0], send = b1 ? v[0] : v[1];
    v[0] = keep + dpp_f(send, 2);
  } else {
    v[0] += dpp_f(v[0], 2);
  }
  return v[0] + dpp_f(v[0], 3);         // lane bit 0 via quad_perm [1,0,3,2]
}

constexpr int kSub = kTB / 2;            // positions per sub-tile of the n-loop (8)

// Own-row vector I/O: a lane reads / writes kSub consecutive positions of its
// own (b, d) row as 16-B vectors (no LDS staging: a wave revisits its rows
// tile after tile, so L2 sees whole lines).
template <typename TI>
__device__ __forceinline__ void load_row_sub(const TI* __restrict__ p, int l0, int L, bool full,
                                             uint4 (&q)[kSub / ElemTraits<TI>::kVec]) {
  constexpr int VI = ElemTraits<TI>::kVec;
#pragma unroll
  for (int k = 0; k < kSub / VI; ++k) {
    const int col0 = l0 + k * VI;
    if (full) q[k] = ld16(p + col0);
    else q[k] = ld16_masked(p + col0, max(0, min(VI, L - col0)));
  }
}

template <typename TI>
__device__ __forceinline__ void store_row_sub(TI* __restrict__ p, int l0, int L, bool full, const float (&v)[kSub]) {
  constexpr int VI = ElemTraits<TI>::kVec;
#pragma unroll
  for (int k = 0; k < kSub / VI; ++k) {
    float w[VI];
#pragma unroll
    for (int e = 0; e < VI; ++e) w[e] = v[k * VI + e];
    const int col0 = l0 + k * VI;
    if (full) st16(p + col0, pack_f<TI>(w));
    else st16_masked(p + col0, pack_f<TI>(w), max(0, min(VI, L - col0)));
  }
}

template <typename TI, int kN, bool kAligned>
__global__ __launch_bounds__(kRows, 2) void scan_bwd_kernel(const BwdArgs a) {
  constexpr int VI = ElemTraits<TI>::kVec;
  constexpr int kVPS = kSub / VI;   // 16-B vectors per sub-tile of one row (1 for 16-bit, 2 for fp32)

  extern __shared__ __attribute__((aligned(16))) float smem_f[];
  float* bcT = smem_f;                   // [2kN][kTB]: B rows then C rows of this tile
  float* carry = bcT + 2 * kN * kTB;     // [kN][kRows]: adjoint carried into the previous positions
  float* xmid = carry + kN * kRows;      // [kN][kRows]: state after the tile's first sub-tile
  float* x0s = xmid + kN * kRows;        // [kN][kRows]: saved state at the tile start
  float* a2s = x0s + kN * kRows;         // [kN][kRows]: A * log2(e)

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
  const int my_dc = dbase + min(lane, nrows - 1);   // lanes past the group end mirror a valid row (never stored)

  const TI* __restrict__ urow = reinterpret_cast<const TI*>(a.u) + (int64_t)b * a.u_bs + (int64_t)my_dc * a.u_ds;
  const TI* __restrict__ drow = reinterpret_cast<const TI*>(a.delta) + (int64_t)b * a.dt_bs + (int64_t)my_dc * a.dt_ds;
  const TI* __restrict__ zrow = reinterpret_cast<const TI*>(a.z) + (int64_t)b * a.z_bs + (int64_t)my_dc * a.z_ds;
  const TI* __restrict__ grow = reinterpret_cast<const TI*>(a.dout) + (int64_t)b * a.go_bs + (int64_t)my_dc * a.go_ds;
  TI* __restrict__ durow = reinterpret_cast<TI*>(a.du) + (int64_t)b * a.du_bs + (int64_t)my_dc * a.du_ds;
  TI* __restrict__ ddrow = reinterpret_cast<TI*>(a.ddelta) + (int64_t)b * a.ddt_bs + (int64_t)my_dc * a.ddt_ds;
  TI* __restrict__ dzrow = reinterpret_cast<TI*>(a.dz) + (int64_t)b * a.dz_bs + (int64_t)my_dc * a.dz_ds;
  const float* __restrict__ Arow = a.A + (int64_t)my_dc * a.dstate;
  const float* __restrict__ csrow = a.chunk_states + ((int64_t)b * a.dim + my_dc) * a.n_states * a.dstate;

  // per-lane, per-state scalars live in LDS ([n][lane]: conflict-free) so the
  // n-loop never waits on global memory
#pragma unroll
  for (int n = 0; n < kN; ++n) {
    carry[n * kRows + lane] = 0.f;
    a2s[n * kRows + lane] = n < a.dstate ? Arow[n] * kLog2e : 0.f;
  }
  // dA_n accumulators: a register ring rotated once per n step (the n-loop is
  // not unrolled), so dAr[0] always belongs to the current n
  float dAr[kN];
#pragma unroll
  for (int n = 0; n < kN; ++n) dAr[n] = 0.f;
  const float Dv = a.D ? a.D[my_dc] : 0.f;
  const float biasv = a.delta_bias ? a.delta_bias[my_dc] : 0.f;
  float dDacc = 0.f, dbacc = 0.f;

  // raw vectors of one sub-tile -> per-position scalars
  auto prep = [&](const uint4 (&rd)[kVPS], const uint4 (&ru)[kVPS], const uint4 (&rz)[kVPS],
                  const uint4 (&rg)[kVPS], int p0, int t, float& dtv, float& sgv, float& uv, float& gyv, float& gzv) {
    uv = elem_f<TI>(ru[t / VI], t % VI);
    const float r = elem_f<TI>(rd[t / VI], t % VI) + biasv;
    const float go = elem_f<TI>(rg[t / VI], t % VI);
    const bool live = p0 + t < L_;
    const float d = softplus ? softplus_f(r) : r;
    // d softplus/dr = sigmoid(r) (torch: gradient 1 above the threshold 20)
    sgv = softplus ? (r > 20.f ? 1.f : sigmoid_f(r)) : 1.f;
    dtv = live ? d : 0.f;
    if (hasZ) {
      const float zv = elem_f<TI>(rz[t / VI], t % VI);
      const float sgz = sigmoid_f(zv);
      gyv = go * zv * sgz;                              // dout * silu(z)
      gzv = go * sgz * (1.f + zv * (1.f - sgz));        // dout * silu'(z)
    } else {
      gyv = go;
      gzv = 0.f;
    }
  };
  auto load_raw = [&](int p0, bool full, uint4 (&ru)[kVPS], uint4 (&rd)[kVPS], uint4 (&rz)[kVPS],
                      uint4 (&rg)[kVPS]) {
    load_row_sub<TI>(urow, p0, L_, full, ru);
    load_row_sub<TI>(drow, p0, L_, full, rd);
    if (hasZ) {
      load_row_sub<TI>(zrow, p0, L_, full, rz);
    } else {
#pragma unroll
      for (int k = 0; k < kVPS; ++k) rz[k] = make_uint4(0u, 0u, 0u, 0u);
    }
    load_row_sub<TI>(grow, p0, L_, full, rg);
  };

  const int ntiles = (L_ + kTB - 1) / kTB;
  for (int ti = ntiles - 1; ti >= 0; --ti) {
    const int l0 = ti * kTB;
    const bool has_hi = l0 + kSub < L_;            // second sub-tile has live positions
    __syncthreads();  // previous tile is done with bcT / xmid / x0s
    // saved tile-start state -> LDS (zero for the first tile)
#pragma unroll
    for (int n = 0; n < kN; ++n) x0s[n * kRows + lane] = (ti > 0 && n < a.dstate) ? csrow[(ti - 1) * a.dstate + n] : 0.f;
    {   // B/C tile, transposed to [2kN][kTB] (per-n rows of positions)
      const float* src = a.bct + ((int64_t)bg * L_ + l0) * (2 * kN);
      const int nval = min(kTB, L_ - l0) * (2 * kN);
      for (int v = lane; v < kTB * 2 * kN; v += kRows) {
        const int t = v / (2 * kN), jn = v % (2 * kN);
        bcT[jn * kTB + t] = v < nval ? src[v] : 0.f;
      }
    }
    __syncthreads();

    // ---- state after the first sub-tile (restart point of the second), from the saved tile-start state
    if (has_hi) {
      float dt[kSub], dtu[kSub];
      {
        uint4 ru[kVPS], rd[kVPS], rz[kVPS], rg[kVPS];
        load_raw(l0, kAligned, ru, rd, rz, rg);   // l0 + kSub < L: the first sub-tile is full
#pragma unroll
        for (int t = 0; t < kSub; ++t) {
          float sgv, uv, gyv, gzv;
          prep(rd, ru, rz, rg, l0, t, dt[t], sgv, uv, gyv, gzv);
          dtu[t] = dt[t] * uv;
        }
      }
#pragma unroll 1
      for (int n = 0; n < kN; ++n) {
        const float A2n = a2s[n * kRows + lane];
        float x = x0s[n * kRows + lane];
        const float* Bt = bcT + n * kTB;
#pragma unroll
        for (int t = 0; t < kSub; ++t) x = fmaf(fast_exp2(dt[t] * A2n), x, dtu[t] * Bt[t]);
        xmid[n * kRows + lane] = x;
      }
    }

    // ---- the two sub-tiles, last first
#pragma unroll 1
    for (int sub = has_hi ? 1 : 0; sub >= 0; --sub) {
      const int p0 = l0 + sub * kSub;
      const bool full = kAligned && (p0 + kSub <= L_);
      float dt[kSub], dtu[kSub], gy[kSub];
      {
        uint4 ru[kVPS], rd[kVPS], rz[kVPS], rg[kVPS];
        load_raw(p0, full, ru, rd, rz, rg);
#pragma unroll
        for (int t = 0; t < kSub; ++t) {
          float sgv, uv, gzv;
          prep(rd, ru, rz, rg, p0, t, dt[t], sgv, uv, gy[t], gzv);
          dtu[t] = dt[t] * uv;
        }
      }
      // S_t = sum_n h B ;  Q_t = sum_n h A a x_{t-1} ;  ys_t = sum_n C x
      float ys[kSub], S[kSub], Q[kSub];
#pragma unroll
      for (int t = 0; t < kSub; ++t) { ys[t] = 0.f; S[t] = 0.f; Q[t] = 0.f; }

#pragma unroll 1
      for (int n = 0; n < kN; ++n) {
        const bool nok = n < a.dstate;
        const float A2n = a2s[n * kRows + lane];
        const float An = A2n * kLn2;
        const float x0n = (sub ? xmid : x0s)[n * kRows + lane];
        const float* Bt = bcT + n * kTB + sub * kSub;
        const float* Ct = bcT + (kN + n) * kTB + sub * kSub;
        // forward sweep: states and decays of this sub-tile
        float xs[kSub], as[kSub];
        float x = x0n;
#pragma unroll
        for (int t = 0; t < kSub; ++t) {
          const float aa = fast_exp2(dt[t] * A2n);
          x = fmaf(aa, x, dtu[t] * Bt[t]);
          xs[t] = x;
          as[t] = aa;
          ys[t] = fmaf(Ct[t], x, ys[t]);
        }
        float red[kSub];
        // dC_t,n = sum over the wave's channels of gy_t x_t,n
#pragma unroll
        for (int t = 0; t < kSub; ++t) red[t] = my_ok ? gy[t] * xs[t] : 0.f;
        {
          const float tot = wave_transpose_reduce<kSub>(red, lane);
          const int t = lane / (64 / kSub);
          if ((lane & (64 / kSub - 1)) == 0 && nok && p0 + t < L_)
            a.slab_bc[((((int64_t)bg * a.nblk + dblk) * kN + n) * 2 + 1) * L_ + p0 + t] = tot;
        }
        // reverse sweep
        float h = carry[n * kRows + lane];
        float dAn = 0.f;
#pragma unroll
        for (int t = kSub - 1; t >= 0; --t) {
          h = fmaf(Ct[t], gy[t], h);
          const float xp = t > 0 ? xs[t - 1] : x0n;
          S[t] = fmaf(h, Bt[t], S[t]);
          red[t] = my_ok ? h * dtu[t] : 0.f;              // dB_t,n contribution
          const float ha = h * as[t];
          const float hax = ha * xp;
          Q[t] = fmaf(hax, An, Q[t]);
          dAn = fmaf(hax, dt[t], dAn);
          h = ha;
        }
        carry[n * kRows + lane] = h;
        {
          const float head = dAr[0] + dAn;
#pragma unroll
          for (int k = 0; k < kN - 1; ++k) dAr[k] = dAr[k + 1];
          dAr[kN - 1] = head;
        }
        {
          const float tot = wave_transpose_reduce<kSub>(red, lane);
          const int t = lane / (64 / kSub);
          if ((lane & (64 / kSub - 1)) == 0 && nok && p0 + t < L_)
            a.slab_bc[((((int64_t)bg * a.nblk + dblk) * kN + n) * 2 + 0) * L_ + p0 + t] = tot;
        }
      }

      // ---- per-position outputs of my channel (raw vectors re-read: L1/L2 hits)
      {
        uint4 ru[kVPS], rd[kVPS], rz[kVPS], rg[kVPS];
        load_raw(p0, full, ru, rd, rz, rg);
        float o_du[kSub], o_dd[kSub], o_dz[kSub];
#pragma unroll
        for (int t = 0; t < kSub; ++t) {
          float dtv, sgv, uv, gyv, gzv;
          prep(rd, ru, rz, rg, p0, t, dtv, sgv, uv, gyv, gzv);
          const float y = fmaf(Dv, uv, ys[t]);
          o_dz[t] = gzv * y;
          o_du[t] = fmaf(Dv, gyv, dtv * S[t]);
          const float dr = fmaf(uv, S[t], Q[t]) * sgv;
          o_dd[t] = dr;
          if (p0 + t < L_ && my_ok) {
            dDacc = fmaf(gyv, uv, dDacc);
            dbacc += dr;
          }
        }
        if (my_ok) {
          store_row_sub<TI>(durow, p0, L_, full, o_du);
          store_row_sub<TI>(ddrow, p0, L_, full, o_dd);
          if (hasZ) store_row_sub<TI>(dzrow, p0, L_, full, o_dz);
        }
      }
    }
  }

  if (my_ok) {
    // slab_a is [b][n][d]: coalesced along d
#pragma unroll
    for (int n = 0; n < kN; ++n) a.slab_a[((int64_t)b * kN + n) * a.dim + my_d] = dAr[n];
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

// dA[d][n] = sum_b slab[b][n][d] (slab row stride ld): columns c = n * dim + d
// (coalesced along d), output transposed to (dim, dstate).  Fixed-order sums.
__global__ __launch_bounds__(256) void scan_bwd_colsum_nd(const float* __restrict__ in, int batch, int dim,
                                                          int dstate, int64_t ld, float* __restrict__ out) {
  __shared__ float part[8][33];
  const int cx = threadIdx.x & 31, q = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cx;
  const int cols = dim * dstate;
  float s = 0.f;
  if (c < cols)
    for (int bb = q; bb < batch; bb += 8) s += in[(int64_t)bb * ld + c];
  part[q][cx] = s;
  __syncthreads();
  if (q == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += part[k][cx];
    const int n = c / dim, d = c % dim;
    out[(int64_t)d * dstate + n] = t;
  }
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
  const size_t lds = (size_t)2 * kN * kTB * 4 + (size_t)4 * kN * kRows * 4;   // bcT + carry, xmid, x0s, a2s
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
  // slab_a is [b][n][d]: column c = n * dim + d -> dA[d][n] (transposed on output)
  const int ca = a.dim * a.dstate;
  hipLaunchKernelGGL(scan_bwd_colsum_nd, dim3((ca + 31) / 32), dim3(256), 0, s, a.slab_a, a.batch, a.dim, a.dstate,
                     (int64_t)a.dim * kN, dA);
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
