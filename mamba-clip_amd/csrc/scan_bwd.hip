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
//  * one wave = 64 channels of one (batch, group); tiles of kTB = kS = 8
//    positions walked in reverse; each tile restarts from the fp32 state the
//    training forward saved at its start (chunk_states), so nothing is
//    recomputed across tiles and no mid-tile pre-pass is needed.
//  * state pairs (n, n+1) in packed fp32; the pair loop is fully unrolled, so
//    A, the adjoint carry and the dA accumulators of every pair stay in VGPRs.
//    Per pair and tile: a forward sweep (x, a kept in VGPRs), the reverse
//    adjoint sweep; per-position accumulators carried across pairs:
//      S_t = sum_n h B,  Q_t = sum_n h A a x_{t-1},  y_t = sum_n C x
//    so du = dt S + D gy and ddt = (Q + u S) sigmoid need no per-n work.
//  * each lane reads / writes its own row's positions as 16-B vectors; the
//    next tile's rows, B/C quads and saved state are prefetched into
//    registers under the current tile.  The tile's B/C block sits in LDS as
//    [pair][position]{B_n, B_n+1, C_n, C_n+1}: one broadcast ds_read_b128.
//  * dB/dC (sums over the 64 channels of the wave) use an in-register
//    transpose-reduce: permlane32_swap / permlane16_swap / DPP row_ror:8 /
//    ds_swizzle / quad_perm halving stages turn 16 per-lane values into 16
//    wave sums in ~2.5 VALU per value, then land in a per-wave fp32 slab.  A
//    small second kernel sums the slabs over waves / batches: deterministic,
//    no atomics.
#include <cstdlib>
#include <type_traits>

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
  float* slab_bc;                    // [b*G+g][nblk][seqlen][2][kN]  (dB partials, then dC partials)
  float* slab_a;                     // [b][kN][dim] (dA partials, one owner per element)
  float* slab_d;                     // [b][dim]
  float* slab_bias;                  // [b][dim]
  const void* y; int64_t y_bs, y_ds;  // forward's pre-gate output (required with z)
};

__device__ __forceinline__ float dpp_f(float v, int ctrl_sel) {
  // ctrl_sel: 0 -> row_ror:8 (xor 8), 1 -> xor 4 (row_shl/shr:4 by bank), 2 -> quad_perm[2,3,0,1] (xor 2),
  // 3 -> quad_perm[1,0,3,2] (xor 1).  Every partner is lane ^ bit exactly: the
  // halving stages need partners that agree on the bits already reduced
  // (row_ror:4 is NOT xor 4 -- it can flip bit 3; tools/ubench/reduce_check.hip).
  const int iv = __float_as_int(v);
  int r;
  if (ctrl_sel == 0) r = __builtin_amdgcn_update_dpp(iv, iv, 0x128, 0xF, 0xF, false);
  else if (ctrl_sel == 1) {
    // xor 4 inside each 16-lane row, on the VALU (no LDS, so no lgkmcnt wait):
    // banks 0/2 (lanes 0-3, 8-11) take lane + 4 (row_shl:4), banks 1/3 take lane - 4 (row_shr:4)
    const int lo = __builtin_amdgcn_update_dpp(iv, iv, 0x104, 0xF, 0x5, false);
    r = __builtin_amdgcn_update_dpp(lo, iv, 0x114, 0xF, 0xA, false);
  }
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

// Own-row vector I/O: a lane reads / writes the kTB consecutive positions of
// its own (b, d) row as 16-B vectors (no LDS staging of the rows: a wave
// revisits its rows tile after tile, so L2 sees whole lines).  Addresses are a
// wave-uniform base (SGPRs) + a 32-bit per-lane element offset, so each row
// costs one VGPR instead of a 64-bit pointer pair (the host checks the range).
template <typename TI>
__device__ __forceinline__ void load_row_tile(const TI* __restrict__ base, uint32_t off, int l0, int L, bool full,
                                              uint4 (&q)[kTB / ElemTraits<TI>::kVec]) {
  constexpr int VI = ElemTraits<TI>::kVec;
#pragma unroll
  for (int k = 0; k < kTB / VI; ++k) {
    const int col0 = l0 + k * VI;
    const TI* p = base + (uint32_t)(off + col0);
    if (full) q[k] = ld16(p);
    else q[k] = ld16_masked(p, max(0, min(VI, L - col0)));
  }
}

template <typename TI>
__device__ __forceinline__ void store_row_tile(TI* __restrict__ base, uint32_t off, int l0, int L, bool full,
                                               const float (&v)[kTB]) {
  constexpr int VI = ElemTraits<TI>::kVec;
#pragma unroll
  for (int k = 0; k < kTB / VI; ++k) {
    float w[VI];
#pragma unroll
    for (int e = 0; e < VI; ++e) w[e] = v[k * VI + e];
    const int col0 = l0 + k * VI;
    TI* p = base + (uint32_t)(off + col0);
    if (full) st16(p, pack_f<TI>(w));
    else st16_masked(p, pack_f<TI>(w), max(0, min(VI, L - col0)));
  }
}

// One wave = 64 channels of one (batch, group); tiles of kTB = 8 positions in
// reverse; state PAIRS (n, n+1) are the unit of work, in packed fp32
// (v_pk_mul_f32 / v_pk_fma_f32), fully unrolled over the kN / 2 pairs so the
// per-pair lane constants (A, the adjoint carry, the dA accumulator) live in
// VGPRs.  Per pair and tile: a forward sweep from the saved tile-start state
// (decays and states kept in VGPRs), the dC contributions reduced across the
// wave, then the reverse adjoint sweep and the dB reduction.  The tile's B/C
// block is staged in LDS as [pair][position]{B_n, B_n+1, C_n, C_n+1} so one
// broadcast ds_read_b128 serves a (pair, position).  The next tile's rows,
// B/C block and saved state are prefetched into registers under this tile.
template <typename TI, int kN, bool kAligned, int kGrp>
__global__ __launch_bounds__(kRows, kGrp >= 4 ? 1 : 2) void scan_bwd_kernel(const BwdArgs a) {
  constexpr int VI = ElemTraits<TI>::kVec;
  constexpr int kVT = kTB / VI;            // 16-B vectors per row tile (1 for 16-bit, 2 for fp32)
  constexpr int kP = kN / 2;               // state pairs
  constexpr int kBCQ = kP * kTB;           // (pair, position) quads of one tile
  constexpr int kBCPer = (kBCQ + kRows - 1) / kRows;

  extern __shared__ __attribute__((aligned(16))) float smem_f[];
  f32x4* bcq = reinterpret_cast<f32x4*>(smem_f);   // [kP][kTB] B/C quads of the tile
  // per-lane, per-pair scalars that persist across pairs / tiles live in LDS
  // ([pair][lane] f32x2: conflict-free ds_read_b64), read and written once per
  // pair and tile -- keeps the fully unrolled pair loop within 256 VGPRs
  f32x2* carry_s = reinterpret_cast<f32x2*>(bcq + kBCQ);   // adjoint carried into the previous tile
  f32x2* dA_s = carry_s + kP * kRows;                      // dA accumulators
  f32x2* x0_s = dA_s + kP * kRows;                         // saved state at the tile start
  f32x2* a2_s = x0_s + kP * kRows;                         // A * log2(e)
  float* dbc_s = reinterpret_cast<float*>(a2_s + kP * kRows);   // [kTB][2][kN] this tile's dB / dC sums

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
  const bool my_ok = lane < nrows;
  const int my_d = dbase + lane;
  const int my_dc = dbase + min(lane, nrows - 1);   // lanes past the group end mirror a valid row (never stored)

  // Row-block addressing.  kAligned: buffer resources (base + byte range of
  // this wave's rows in SGPRs) and ONE 32-bit VGPR offset per access, rebuilt
  // from an opaque lane id where used instead of being held across the pair
  // loop; reads past a row block return 0, so ragged tails load branch-free
  // and are masked where used.  !kAligned (odd strides): plain pointers.
  const int64_t rows_u = (int64_t)b * a.u_bs + (int64_t)dbase * a.u_ds;
  const int64_t rows_d = (int64_t)b * a.dt_bs + (int64_t)dbase * a.dt_ds;
  const int64_t rows_z = hasZ ? (int64_t)b * a.z_bs + (int64_t)dbase * a.z_ds : rows_u;
  const int64_t rows_g = (int64_t)b * a.go_bs + (int64_t)dbase * a.go_ds;
  const TI* __restrict__ ub = reinterpret_cast<const TI*>(a.u) + rows_u;
  const TI* __restrict__ db = reinterpret_cast<const TI*>(a.delta) + rows_d;
  const TI* __restrict__ zb = hasZ ? reinterpret_cast<const TI*>(a.z) + rows_z : ub;
  const TI* __restrict__ gb = reinterpret_cast<const TI*>(a.dout) + rows_g;
  TI* __restrict__ dub = reinterpret_cast<TI*>(a.du) + (int64_t)b * a.du_bs + (int64_t)dbase * a.du_ds;
  TI* __restrict__ ddb = reinterpret_cast<TI*>(a.ddelta) + (int64_t)b * a.ddt_bs + (int64_t)dbase * a.ddt_ds;
  TI* __restrict__ dzb = reinterpret_cast<TI*>(a.dz) + (int64_t)b * a.dz_bs + (int64_t)dbase * a.dz_ds;
  const int64_t zds64 = hasZ ? a.z_ds : a.u_ds;
  const TI* __restrict__ yb = hasZ ? reinterpret_cast<const TI*>(a.y) + (int64_t)b * a.y_bs + (int64_t)dbase * a.y_ds : ub;
  const int64_t yds64 = hasZ ? a.y_ds : a.u_ds;
  const float* __restrict__ csb = a.chunk_states + ((int64_t)b * a.dim + dbase) * a.n_states * a.dstate;
  const uint32_t cs_ds = (uint32_t)(a.n_states * a.dstate);
  const float* __restrict__ bcsrc = a.bct + (int64_t)bg * L_ * (2 * kN);
  auto row_of_lane = [&]() -> uint32_t { return (uint32_t)min(opaque_lane_id(), nrows - 1); };
  auto span = [&](int64_t ds) -> uint32_t { return (uint32_t)(((int64_t)(nrows - 1) * ds + L_) * (int64_t)sizeof(TI)); };
  const __amdgpu_buffer_rsrc_t rs_u = make_rsrc(ub, span(a.u_ds)), rs_d = make_rsrc(db, span(a.dt_ds));
  const __amdgpu_buffer_rsrc_t rs_z = make_rsrc(zb, span(zds64)), rs_g = make_rsrc(gb, span(a.go_ds));
  const __amdgpu_buffer_rsrc_t rs_y = make_rsrc(yb, span(yds64));
  const __amdgpu_buffer_rsrc_t rs_du = make_rsrc(dub, span(a.du_ds)), rs_dd = make_rsrc(ddb, span(a.ddt_ds));
  const __amdgpu_buffer_rsrc_t rs_dz = make_rsrc(hasZ ? (const void*)dzb : (const void*)dub, span(hasZ ? a.dz_ds : a.du_ds));
  const __amdgpu_buffer_rsrc_t rs_cs = make_rsrc(csb, (uint32_t)nrows * cs_ds * 4u);
  const __amdgpu_buffer_rsrc_t rs_bc = make_rsrc(bcsrc, (uint32_t)L_ * (2 * kN) * 4u);
  const __amdgpu_buffer_rsrc_t rs_slab =
      make_rsrc(a.slab_bc + ((int64_t)bg * a.nblk + dblk) * L_ * (2 * kN), (uint32_t)L_ * (2 * kN) * 4u);
  // one row tile of a tensor: [l0, l0 + kTB) of this lane's row
  auto tile_in = [&](const __amdgpu_buffer_rsrc_t& rs, const TI* base, int64_t ds, int l0, bool full,
                     uint4 (&q)[kVT]) {
    const uint32_t rl = row_of_lane();
    if constexpr (kAligned) {
#pragma unroll
      for (int k = 0; k < kVT; ++k)
        q[k] = buf_ld16(rs, (rl * (uint32_t)ds + (uint32_t)(l0 + k * VI)) * (uint32_t)sizeof(TI));
    } else {
      load_row_tile<TI>(base + (int64_t)rl * ds, 0, l0, L_, full, q);
    }
  };
  auto pack_tile = [&](const float (&v)[kTB], uint4 (&q)[kVT]) {
#pragma unroll
    for (int k = 0; k < kVT; ++k) {
      float w[VI];
#pragma unroll
      for (int e = 0; e < VI; ++e) w[e] = v[k * VI + e];
      q[k] = pack_f<TI>(w);
    }
  };
  // kAligned only: store a packed row tile (positions past L masked off)
  auto tile_out_q = [&](const __amdgpu_buffer_rsrc_t& rs, int64_t ds, uint32_t rl, int l0, bool full,
                        const uint4 (&q)[kVT]) {
#pragma unroll
    for (int k = 0; k < kVT; ++k) {
      const uint32_t off = (rl * (uint32_t)ds + (uint32_t)(l0 + k * VI)) * (uint32_t)sizeof(TI);
      if (full) buf_st16(rs, off, q[k]);
      else buf_st16_masked<TI>(rs, off, q[k], max(0, min(VI, L_ - (l0 + k * VI))));
    }
  };
  auto tile_out = [&](const __amdgpu_buffer_rsrc_t& rs, TI* base, int64_t ds, uint32_t rl, int l0, bool full,
                      const float (&v)[kTB]) {
    if constexpr (kAligned) {
      uint4 q[kVT];
      pack_tile(v, q);
      tile_out_q(rs, ds, rl, l0, full, q);
    } else {
      store_row_tile<TI>(base + (int64_t)rl * ds, 0, l0, L_, full, v);
    }
  };

  // exact-width state rows (dstate == kN, the common case): A and the saved
  // states move as 16-B vectors, issued back to back with one wait
  const bool vecN = a.dstate == kN;
  if (vecN) {
    const f32x4* A4 = reinterpret_cast<const f32x4*>(a.A + (int64_t)my_dc * kN);
    f32x4 av[kN / 4];
#pragma unroll
    for (int q = 0; q < kN / 4; ++q) av[q] = A4[q] * kLog2e;
#pragma unroll
    for (int q = 0; q < kN / 4; ++q) {
      a2_s[(2 * q) * kRows + lane] = av[q].lo;
      a2_s[(2 * q + 1) * kRows + lane] = av[q].hi;
    }
  } else {
#pragma unroll
    for (int p = 0; p < kP; ++p) {
      const int n0 = 2 * p;
      f32x2 av;
      av.x = n0 < a.dstate ? a.A[(int64_t)my_dc * a.dstate + n0] * kLog2e : 0.f;
      av.y = n0 + 1 < a.dstate ? a.A[(int64_t)my_dc * a.dstate + n0 + 1] * kLog2e : 0.f;
      a2_s[p * kRows + lane] = av;
    }
  }
#pragma unroll
  for (int p = 0; p < kP; ++p) {
    carry_s[p * kRows + lane] = f32x2{0.f, 0.f};
    dA_s[p * kRows + lane] = f32x2{0.f, 0.f};
  }
  const float Dv = a.D ? a.D[my_dc] : 0.f;
  const float biasv = a.delta_bias ? a.delta_bias[my_dc] : 0.f;
  float dDacc = 0.f, dbacc = 0.f;

  // ---- prefetch registers: one tile's rows, B/C quads and saved start
  // state.  Tiles are walked last to first, so only the first tile visited can
  // be ragged: every prefetch inside the loop is a full tile and (kAligned)
  // compiles to unconditional 16-B loads -- no control flow around the loads,
  // so nothing forces a vmcnt wait before the loads are consumed a tile later.
  uint4 ru[kVT], rd[kVT], rz[kVT], rg[kVT];
  // 16-bit inputs: rows are fetched for a GROUP of kG tiles at a time (the
  // loads go out back to back, so each 128-B line a lane touches is fetched
  // once per 8 kG positions instead of once per 8); the later tiles of the
  // group wait in su.. (kG = 4 runs at one wave per SIMD for the registers)
  constexpr int kG = (kAligned && sizeof(TI) == 2) ? kGrp : 1;
  constexpr int kS = kG > 1 ? kG - 1 : 1;
  uint4 su[kS][kVT], sd[kS][kVT], sz[kS][kVT], sg[kS][kVT];
  f32x4 pbc[kBCPer];
  f32x4 px0[kN / 4];
  auto load_rows = [&](int ti, bool full, uint4 (&qu)[kVT], uint4 (&qd)[kVT], uint4 (&qz)[kVT], uint4 (&qg)[kVT]) {
    const int l0 = ti * kTB;
    tile_in(rs_u, ub, a.u_ds, l0, full, qu);
    tile_in(rs_d, db, a.dt_ds, l0, full, qd);
    tile_in(rs_z, zb, zds64, l0, full, qz);     // (no z: a harmless re-read of u, no branch)
    tile_in(rs_g, gb, a.go_ds, l0, full, qg);
  };
  auto prefetch_bc = [&](int ti) {
    const int l0 = ti * kTB;
#pragma unroll
    for (int k = 0; k < kBCPer; ++k) {       // quad q = lane + 64 k -> (pair q / kTB, position q % kTB)
      const int q = lane + k * kRows;
      const int pp = min(q / kTB, kP - 1), t = q % kTB;
      // positions past L read as 0 (buffer range); quads q >= kBCQ are never stored
      const uint32_t off = (uint32_t)(((l0 + t) * (2 * kN) + 2 * pp) * 4);
      const uint2 bb = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs_bc, off, 0, 0));
      const uint2 cc = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs_bc, off + kN * 4, 0, 0));
      pbc[k] = f32x4{__uint_as_float(bb.x), __uint_as_float(bb.y), __uint_as_float(cc.x), __uint_as_float(cc.y)};
    }
  };
  // saved state at the start of tile ti (zero for ti == 0): the row's first
  // kN floats as kN/4 16-B loads (dword-aligned for any dstate; entries past
  // dstate are masked where consumed).  Unconditional: tile 0 gets an offset
  // past the buffer range, which reads 0.  Neither a select on the loaded data
  // nor a branch around the loads may appear here -- either makes the compiler
  // wait for them (and for every older load and store) on the spot.
  auto prefetch_x0 = [&](int ti) {
    const uint32_t off = ti > 0 ? (row_of_lane() * cs_ds + (uint32_t)((ti - 1) * a.dstate)) * 4u : 0x80000000u;
#pragma unroll
    for (int q = 0; q < kN / 4; ++q) px0[q] = __builtin_bit_cast(f32x4, buf_ld16(rs_cs, off + 16 * q));
  };

#ifdef MC_BWD_STAMPS
  uint64_t st_pro = 0, st_pair = 0, st_out = 0;
#endif
  const int ntiles = (L_ + kTB - 1) / kTB;
  // mode -1: one tile at a time; m >= 0: the m-th tile (from the top) of a group
  auto tile_body = [&](const int ti, auto mode_c) {
    constexpr int kMode = decltype(mode_c)::value;
#ifdef MC_BWD_STAMPS
    const uint64_t s0 = __builtin_amdgcn_s_memtime();
#endif
    const int l0 = ti * kTB;
    const bool full = kAligned && (l0 + kTB <= L_);
    wave_lds_sync();                             // previous tile is done with the B/C quads
#pragma unroll
    for (int k = 0; k < kBCPer; ++k) {
      const int q = lane + k * kRows;
      if ((k + 1) * kRows <= kBCQ || q < kBCQ) bcq[q] = pbc[k];
    }
    // this tile's per-position scalars (from the prefetched raw rows)
    float dt[kTB], dtu[kTB], gy[kTB];
#pragma unroll
    for (int t = 0; t < kTB; ++t) {
      // positions past L (ragged first tile) hold whatever the 16-B loads
      // returned: zero them before they meet the recurrence
      const bool tv = full || l0 + t < L_;
      const float uv = tv ? elem_f<TI>(ru[t / VI], t % VI) : 0.f;
      const float r = elem_f<TI>(rd[t / VI], t % VI) + biasv;
      const float go = tv ? elem_f<TI>(rg[t / VI], t % VI) : 0.f;
      float d = softplus ? softplus_f(r) : r;
      d = tv ? d : 0.f;
      dt[t] = d;
      // lanes mirroring a row past the group end: dtu = gy = 0 zeroes their
      // dB / dC contributions here, once per tile, instead of a select per
      // value in every pair's reductions (their own outputs are never stored)
      dtu[t] = my_ok ? d * uv : 0.f;
      if (hasZ) {
        const float zv = tv ? elem_f<TI>(rz[t / VI], t % VI) : 0.f;
        gy[t] = my_ok ? go * zv * sigmoid_f(zv) : 0.f;   // dout * silu(z)
      } else {
        gy[t] = my_ok ? go : 0.f;
      }
    }
    // saved state at the tile start -> LDS
#pragma unroll
    for (int q = 0; q < kN / 4; ++q) {
      const f32x4 v = px0[q];
      x0_s[(2 * q) * kRows + lane] = f32x2{4 * q < a.dstate ? v.x : 0.f, 4 * q + 1 < a.dstate ? v.y : 0.f};
      x0_s[(2 * q + 1) * kRows + lane] = f32x2{4 * q + 2 < a.dstate ? v.z : 0.f, 4 * q + 3 < a.dstate ? v.w : 0.f};
    }
    wave_lds_sync();                             // B/C quads staged
    // next tile's loads fly under this tile's math.  kAligned: unconditional
    // (tile -1 addresses land outside the buffers or in unused row bytes)
    if constexpr (kMode < 0) {
      if (kAligned || ti > 0) load_rows(ti - 1, kAligned, ru, rd, rz, rg);
    } else if constexpr (kMode < kG - 1) {     // next tile of the group is already here
#pragma unroll
      for (int k = 0; k < kVT; ++k) {
        ru[k] = su[kMode][k]; rd[k] = sd[kMode][k]; rz[k] = sz[kMode][k]; rg[k] = sg[kMode][k];
      }
    } else {                                   // last tile of the group: fetch the next group
      load_rows(ti - 1, true, ru, rd, rz, rg);   // (tiles below 0 land outside the buffers
#pragma unroll                                 //  or in unused row bytes)
      for (int j = 0; j < kG - 1; ++j) load_rows(ti - 2 - j, true, su[j], sd[j], sz[j], sg[j]);
    }
    prefetch_bc(ti - 1);
    prefetch_x0(ti - 1);
    // the forward's pre-gate y of this tile (dz only), consumed after the pair loop
    uint4 cy[kVT];
    tile_in(rs_y, yb, yds64, l0, full, cy);

    f32x2 S2[kTB], Q2[kTB];
#pragma unroll
    for (int t = 0; t < kTB; ++t) { S2[t] = f32x2{0.f, 0.f}; Q2[t] = f32x2{0.f, 0.f}; }

#ifdef MC_BWD_STAMPS
    const uint64_t s1 = __builtin_amdgcn_s_memtime();
    st_pro += s1 - s0;
#endif
#pragma unroll 1
    for (int p = 0; p < kP; ++p) {
      const f32x2 A2p = a2_s[p * kRows + lane];
      f32x4 bc[kTB];
#pragma unroll
      for (int t = 0; t < kTB; ++t) bc[t] = bcq[p * kTB + t];
      // forward sweep: states and decays of this pair over the tile
      f32x2 xs[kTB], as[kTB];
      const f32x2 x0p = x0_s[p * kRows + lane];
      f32x2 x = x0p;
#pragma unroll
      for (int t = 0; t < kTB; ++t) {
        const f32x2 arg = A2p * dt[t];
#ifdef MC_DIAG_NOEXP
        const f32x2 aa = arg;
#else
        const f32x2 aa = {fast_exp2(arg.x), fast_exp2(arg.y)};
#endif
        x = aa * x + bc[t].lo * dtu[t];
        xs[t] = x;
        as[t] = aa;
      }
      // dC_t,n = sum over the wave's channels of gy_t x_t,n
      {
        float red[2 * kTB];
#pragma unroll
        for (int t = 0; t < kTB; ++t) {
          const f32x2 v = xs[t] * gy[t];
          red[2 * t] = v.x;
          red[2 * t + 1] = v.y;
        }
#ifdef MC_DIAG_NORED
        float tot = 0.f;
#pragma unroll
        for (int i = 0; i < 2 * kTB; ++i) tot += red[i];
#else
        const float tot = wave_transpose_reduce<2 * kTB>(red, lane);
#endif
        const int j = lane / (64 / (2 * kTB));
        const int t = j / 2, n = 2 * p + (j & 1);
        if ((lane & (64 / (2 * kTB) - 1)) == 0)
          dbc_s[(t * 2 + 1) * kN + n] = tot;
      }
      // reverse sweep: adjoint of the state.  The B/C quads are read from LDS
      // again (the compiler barrier stops them being kept live across the dC
      // reduction: 32 VGPRs at the kernel's pressure peak)
      asm volatile("" ::: "memory");
#pragma unroll
      for (int t = 0; t < kTB; ++t) bc[t] = bcq[p * kTB + t];
      f32x2 h = carry_s[p * kRows + lane];
      f32x2 dAp = dA_s[p * kRows + lane];
      float red[2 * kTB];
#pragma unroll
      for (int t = kTB - 1; t >= 0; --t) {
        h = bc[t].hi * gy[t] + h;                  // + C_t gy_t
        S2[t] = h * bc[t].lo + S2[t];
        const f32x2 vb = h * dtu[t];
        red[2 * t] = vb.x;
        red[2 * t + 1] = vb.y;
        const f32x2 ha = h * as[t];
        const f32x2 hax = ha * (t > 0 ? xs[t - 1] : x0p);
        Q2[t] = hax * A2p + Q2[t];
        dAp = hax * dt[t] + dAp;
        h = ha;
      }
      carry_s[p * kRows + lane] = h;
      dA_s[p * kRows + lane] = dAp;
      {
#ifdef MC_DIAG_NORED
        float tot = 0.f;
#pragma unroll
        for (int i = 0; i < 2 * kTB; ++i) tot += red[i];
#else
        const float tot = wave_transpose_reduce<2 * kTB>(red, lane);
#endif
        const int j = lane / (64 / (2 * kTB));
        const int t = j / 2, n = 2 * p + (j & 1);
        if ((lane & (64 / (2 * kTB) - 1)) == 0)
          dbc_s[(t * 2 + 0) * kN + n] = tot;
      }
    }

#ifdef MC_BWD_STAMPS
    const uint64_t s2 = __builtin_amdgcn_s_memtime();
    st_pair += s2 - s1;
#endif
    // ---- the tile's dB / dC sums: one coalesced 16-B store per lane into
    // this wave's slab block (positions past L fall outside the buffer range
    // and are dropped)
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < (kTB * 2 * kN) / (4 * kRows) + ((kTB * 2 * kN) % (4 * kRows) ? 1 : 0); ++k) {
      const int f = 4 * (lane + k * kRows);
      if (f < kTB * 2 * kN) {
        const uint4 v = *reinterpret_cast<const uint4*>(dbc_s + f);
        buf_st16(rs_slab, (uint32_t)((l0 * 2 * kN + f) * 4), v);
      }
    }
    // ---- per-position outputs of my channel (this tile's rows re-read: L2
    // hits; keeping them in registers through the pair loop would spill)
    uint4 cu[kVT], cd[kVT], cz[kVT], cg[kVT];
    tile_in(rs_u, ub, a.u_ds, l0, full, cu);
    tile_in(rs_d, db, a.dt_ds, l0, full, cd);
    tile_in(rs_z, zb, zds64, l0, full, cz);
    tile_in(rs_g, gb, a.go_ds, l0, full, cg);
    float o_du[kTB], o_dd[kTB], o_dz[kTB];
#pragma unroll
    for (int t = 0; t < kTB; ++t) {
      const float uv = elem_f<TI>(cu[t / VI], t % VI);
      const float r = elem_f<TI>(cd[t / VI], t % VI) + biasv;
      const float go = elem_f<TI>(cg[t / VI], t % VI);
      const float S = S2[t].x + S2[t].y;
      const float Q = (Q2[t].x + Q2[t].y) * kLn2;   // A2 carries log2(e)
      const float sg = softplus ? (r > 20.f ? 1.f : sigmoid_f(r)) : 1.f;
      float gyv = go;
      float gz = 0.f;
      if (hasZ) {
        const float zv = elem_f<TI>(cz[t / VI], t % VI);
        const float sgz = sigmoid_f(zv);
        gyv = go * zv * sgz;
        gz = go * sgz * (1.f + zv * (1.f - sgz));
      }
      o_dz[t] = gz * elem_f<TI>(cy[t / VI], t % VI);   // y + D u, as the forward produced it
      o_du[t] = fmaf(Dv, gyv, dt[t] * S);
      const float dr = fmaf(uv, S, Q) * sg;
      o_dd[t] = dr;
      if (l0 + t < L_ && my_ok) {
        dDacc = fmaf(gyv, uv, dDacc);
        dbacc += dr;
      }
    }
    if (my_ok) {
      const uint32_t rl = row_of_lane();
      tile_out(rs_du, dub, a.du_ds, rl, l0, full, o_du);
      tile_out(rs_dd, ddb, a.ddt_ds, rl, l0, full, o_dd);
      if (hasZ) tile_out(rs_dz, dzb, a.dz_ds, rl, l0, full, o_dz);
    }
#ifdef MC_BWD_STAMPS
    st_out += __builtin_amdgcn_s_memtime() - s2;
#endif
  };

  // drain once before the loop: the loop header then merges "nothing pending"
  // from the entry edge, so consuming a prefetch never waits for the previous
  // tile's stores (vmcnt counts stores too on gfx9)
  if constexpr (kG > 1) {
    const int ngroups = (ntiles + kG - 1) / kG;   // a partial group adds tiles past L (fully masked)
    const int top = kG * ngroups - 1;
    load_rows(top, true, ru, rd, rz, rg);
#pragma unroll
    for (int j = 0; j < kG - 1; ++j) load_rows(top - 1 - j, true, su[j], sd[j], sz[j], sg[j]);
    prefetch_bc(top);
    prefetch_x0(top);
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    for (int k = ngroups - 1; k >= 0; --k) {
      const int t0 = kG * k + kG - 1;
      tile_body(t0, std::integral_constant<int, 0>());
      if constexpr (kG >= 2) tile_body(t0 - 1, std::integral_constant<int, 1>());
      if constexpr (kG >= 3) tile_body(t0 - 2, std::integral_constant<int, 2>());
      if constexpr (kG >= 4) tile_body(t0 - 3, std::integral_constant<int, 3>());
    }
  } else {
    load_rows(ntiles - 1, kAligned && ntiles * kTB <= L_, ru, rd, rz, rg);
    prefetch_bc(ntiles - 1);
    prefetch_x0(ntiles - 1);
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    for (int ti = ntiles - 1; ti >= 0; --ti) tile_body(ti, std::integral_constant<int, -1>());
  }
#ifdef MC_BWD_STAMPS
  // diagnostic build: per-wave segment cycles -> slab_d (outputs are invalid in this build)
  if (lane == 0) {
    uint64_t* dbg = reinterpret_cast<uint64_t*>(a.slab_d) + (int64_t)blockIdx.x * 4;
    dbg[0] = st_pro; dbg[1] = st_pair; dbg[2] = st_out; dbg[3] = ntiles;
  }
  return;
#endif

  if (my_ok) {
    // slab_a is [b][n][d]: coalesced along d
#pragma unroll
    for (int p = 0; p < kP; ++p) {
      const f32x2 v = dA_s[p * kRows + lane];
      a.slab_a[((int64_t)b * kN + 2 * p) * a.dim + my_d] = v.x;
      a.slab_a[((int64_t)b * kN + 2 * p + 1) * a.dim + my_d] = v.y;
    }
    a.slab_d[(int64_t)b * a.dim + my_d] = dDacc;
    a.slab_bias[(int64_t)b * a.dim + my_d] = dbacc;
  }
}

// dB / dC: sum the per-wave slabs; dA / dD / dbias: sum the per-batch slabs.
template <typename TW, int kN>
__global__ __launch_bounds__(256) void scan_bwd_reduce_bc(const float* __restrict__ slab, int batch, int G, int nblk,
                                                           int dstate, int L, TW* __restrict__ dB, TW* __restrict__ dC) {
  // thread -> (b*G+g, l, which, n), n fastest: the slab reads are coalesced
  const int64_t total = (int64_t)batch * G * L * 2 * kN;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i % kN);
    int64_t r = i / kN;
    const int which = (int)(r % 2);
    r /= 2;
    const int l = (int)(r % L);
    const int64_t bgi = r / L;
    if (n >= dstate) continue;
    float s = 0.f;
    for (int k = 0; k < nblk; ++k) s += slab[((bgi * nblk + k) * L + l) * (2 * kN) + which * kN + n];
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
  // B/C quads + carry, dA, x0, A + the tile's dB / dC sums
  const size_t lds = (size_t)(kN / 2) * kTB * 16 + (size_t)4 * (kN / 2) * kRows * 8 + (size_t)kTB * 2 * kN * 4;
  // 16-bit rows in groups of 2 tiles.  Groups of 4 (one wave per SIMD for the
  // registers) measured slower: C2 780 vs 724 us contiguous, 810 vs 817 us
  // with the mixer's channel-major views (tools/ab_scan_bwd.sh)
  if (aligned && sizeof(TI) == 2) {
    hipLaunchKernelGGL((scan_bwd_kernel<TI, kN, true, 2>), dim3(a.total_blocks), dim3(kRows), lds, s, a);
  } else if (aligned) {
    hipLaunchKernelGGL((scan_bwd_kernel<TI, kN, true, 1>), dim3(a.total_blocks), dim3(kRows), lds, s, a);
  } else {
    hipLaunchKernelGGL((scan_bwd_kernel<TI, kN, false, 1>), dim3(a.total_blocks), dim3(kRows), lds, s, a);
  }
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
  const int64_t total = (int64_t)a.batch * a.n_groups * kN * 2 * a.seqlen;
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
  MC_CHECK(!p->z || (p->dz && p->out_y), MC_ERR_INVALID,
           "mc_scan_bwd: dz and out_y (the forward's pre-gate output) required when z is given");
  MC_CHECK((int64_t)kRows * mc_scan_n_chunks(p->seqlen) * padded_dstate(p->dstate) * 4 < ((int64_t)1 << 31),
           MC_ERR_INVALID, "mc_scan_bwd: seqlen %d too long for 32-bit chunk-state offsets", p->seqlen);
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
  a.y = p->z ? p->out_y : nullptr; a.y_bs = p->out_y_batch_stride; a.y_ds = p->out_y_dim_stride;
  a.slab_bc = reinterpret_cast<float*>(ws + w.slab_bc);
  a.slab_a = reinterpret_cast<float*>(ws + w.slab_a);
  a.slab_d = reinterpret_cast<float*>(ws + w.slab_d);
  a.slab_bias = reinterpret_cast<float*>(ws + w.slab_bias);
  (void)np;

  const int ib = p->itype == MC_DTYPE_F32 ? 4 : 2;
  // outputs are contiguous: the vector path also needs 16-B aligned rows there
  bool aligned = vec_ok(p->u, p->u_batch_stride, p->u_dim_stride, 0, ib) &&
                       vec_ok(p->delta, p->delta_batch_stride, p->delta_dim_stride, 0, ib) &&
                       vec_ok(p->z, p->z_batch_stride, p->z_dim_stride, 0, ib) &&
                       vec_ok(p->dout, p->dout_batch_stride, p->dout_dim_stride, 0, ib) &&
                       vec_ok(p->du, p->du_batch_stride, p->du_dim_stride, 0, ib) &&
                       vec_ok(p->ddelta, p->ddelta_batch_stride, p->ddelta_dim_stride, 0, ib) &&
                       vec_ok(p->dz, p->dz_batch_stride, p->dz_dim_stride, 0, ib) &&
                       vec_ok(a.y, a.y_bs, a.y_ds, 0, ib);
  // the vector path addresses a wave's 64 rows with 32-bit byte offsets
  auto span_ok = [&](const void* t, int64_t ds) {
    return !t || ((int64_t)(kRows - 1) * (ds < 0 ? -ds : ds) + p->seqlen) * ib < ((int64_t)1 << 31);
  };
  const bool spans = span_ok(p->u, p->u_dim_stride) && span_ok(p->delta, p->delta_dim_stride) &&
                     span_ok(p->z, p->z_dim_stride) && span_ok(p->dout, p->dout_dim_stride) &&
                     span_ok(p->du, p->du_dim_stride) && span_ok(p->ddelta, p->ddelta_dim_stride) &&
                     span_ok(p->dz, p->dz_dim_stride) && span_ok(a.y, a.y_ds);
  aligned = aligned && spans;
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
