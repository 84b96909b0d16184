// scan_fwd_pair.hip -- selective-scan forward with state-split lane pairs (every 16-bit, N = 16 call:
// the C2 and C4 text towers).
//
// Same op as scan_fwd.hip (reference semantics /root/reference/src/mamba_clip/model.py:83-169):
//   dt_t = softplus(delta_t + delta_bias[d]);  x_t[n] = exp(dt_t A[d,n]) x_{t-1}[n] + dt_t B_t[n] u_t
//   y_t  = sum_n C_t[n] x_t[n] + D[d] u_t;     out_t = y_t * silu(z_t)
//
// Why a second long-sequence kernel: at C4 (B 64, D 3072) the one-channel-per-lane
// kernel has 3072 one-wave workgroups = 3 per SIMD with 2 resident, so every SIMD
// runs a 2 + 1 round and the last third of the grid issues from a lone wave.  Here
// a wave owns 32 channels and lane (2c + h) keeps states [8h, 8h + 8) of channel c:
//  * 6144 waves at C4 = 6 per SIMD, half the per-lane state registers -> 3 resident,
//    two full rounds, no lone-wave tail;
//  * the per-position scalars are computed ONCE per (channel, position) in the
//    cooperative staging pass, vectorised along the sequence: dt = softplus(delta +
//    bias) and du = dt u go to LDS as fp32 pairs, so the pair never repeats them;
//  * the two lanes of a channel read the same (dt, du) (one broadcast address per
//    pair) and their own half of B_t / C_t (two broadcast addresses per wave);
//  * each lane writes its partial y_t over the (dt, du) bytes it consumed; the gate
//    pass (same vector mapping as the staging, so it still holds u for D u) adds the
//    two partials, applies silu(z) and stores 16-B vectors along the sequence;
//  * B / C straight from their 16-bit rows (x_dbl slices): one 16-B vector per lane and
//    array per chunk (state row lane & 15, positions 8 (lane >> 4) + [0, 8)), converted
//    into the chunk's fp32 [position][B 16 | C 16] LDS block -- no fp32 pre-pass.
// Requirements (host-checked): dstate == 16, 16-B aligned 16-bit rows (B / C too, in the
// activation dtype), seqlen % 8 == 0, row spans < 2 GiB (32-bit buffer offsets), no
// grouped directions.
#include <type_traits>

#include "scan_common.h"

namespace mc {
namespace scan {

constexpr int kPCh = 32;   // channels per wave
constexpr int kPN = 16;    // dstate
constexpr int kPH = 8;     // states per lane
constexpr int kPG = 4;     // positions per recurrence group (32 B of {dt, du} per row)
// State pairs per lane whose decays use the packed-FMA exp2 polynomial instead of v_exp_f32 (A/B
// lever, VERDICT r03: balance the transcendental and the packed pipes).  Measured: one pair of four
// 3.20 ms, two 3.79 ms against 2.56-2.86 ms (profiles/r04/scan_fwd_exp_poly_ab.txt) -- v_exp_f32 does
// not co-issue with the packed FMAs, and the polynomial costs 15 issue slots per two values: 0.
#ifndef MC_FWD_POLY_PAIRS
#define MC_FWD_POLY_PAIRS 0
#endif
// Output rows stored non-temporally (nt cache policy): L2 keeps the u / delta / z lines whose second
// 64-B half the next chunk reads.  Interleaved C4 A/B 2.81-2.84 vs 2.83-2.86 ms; PMC writes 1.58 GB
// (= the output) instead of 1.85 GB, reads 4.35 vs 4.56 GB raw (profiles/r04/scan_fwd_nt_store_ab.txt)
#ifndef MC_FWD_NT_STORE
#define MC_FWD_NT_STORE 1
#endif

template <typename TI>
struct PairLayout {
  static constexpr int VI = ElemTraits<TI>::kVec;  // elements per 16-B vector
  static constexpr int kVPR = kT / VI;             // vectors per row and chunk
  static constexpr int kNV = kPCh * kVPR / 64;     // vectors per lane and array
  static constexpr int kStride = kT * 8 + 16;      // row: per 2 positions {dt, dt, du, du} fp32 + pad (rows on distinct banks)
  static constexpr int kRowBytes = kPCh * kStride;
  static constexpr int kBCBytes = kT * 2 * kPN * 4;
};

template <typename TI, bool kSP, int kMinW, bool kPD, bool kFine>
__global__ __launch_bounds__(64, kMinW) void scan_fwd_pair_kernel(const FwdArgs a) {
  using PL = PairLayout<TI>;
  constexpr int VI = PL::VI, kVPR = PL::kVPR, kNV = PL::kNV;
  static_assert(kT == 32 && kPN == 16 && VI == 8, "one 16-B B / C vector per lane and chunk");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* rowbuf = smem;
  float* bcl = reinterpret_cast<float*>(smem + PL::kRowBytes);   // [kT][B 16 | C 16]

  const int lane = threadIdx.x;
  const int ch = lane >> 1, h = lane & 1;
  const int lin = xcd_remap(blockIdx.x, a.total_blocks);
  const int dblk = lin % a.nblk;
  const int bg = lin / a.nblk;
  const int g = bg % a.n_groups, b = bg / a.n_groups;
  const int H = a.dim / a.n_groups;
  const int dbase = g * H + dblk * kPCh;
  const int nrows = min(kPCh, H - dblk * kPCh);
  const int L_ = a.seqlen;
  const bool hasZ = a.z != nullptr;

  auto rows_rsrc = [&](const void* base, int64_t bs, int64_t ds) {
    return make_rsrc(reinterpret_cast<const TI*>(base) + (int64_t)b * bs + (int64_t)dbase * ds,
                     (uint32_t)(((int64_t)(nrows - 1) * ds + L_) * (int64_t)sizeof(TI)));
  };
  const __amdgpu_buffer_rsrc_t rs_u = rows_rsrc(a.u, a.u_bs, a.u_ds);
  const __amdgpu_buffer_rsrc_t rs_d = rows_rsrc(kPD ? (a.delta_out ? a.delta_out : a.u) : a.delta,
                                                kPD && !a.delta_out ? a.u_bs : a.dt_bs, kPD && !a.delta_out ? a.u_ds : a.dt_ds);
  const __amdgpu_buffer_rsrc_t rs_z = rows_rsrc(hasZ ? a.z : a.u, hasZ ? a.z_bs : a.u_bs, hasZ ? a.z_ds : a.u_ds);
  const __amdgpu_buffer_rsrc_t rs_o = rows_rsrc(a.out, a.o_bs, a.o_ds);
  const __amdgpu_buffer_rsrc_t rs_y =
      rows_rsrc(a.out_y ? a.out_y : a.u, a.out_y ? a.y_bs : a.u_bs, a.out_y ? a.y_ds : a.u_ds);
  // B / C rows of this (batch, group): lane j reads state row j & 15, positions [8 (j >> 4), +8) of a
  // chunk (past the end: the next row's or zero bytes -- finite, and met only by dt = du = 0 positions)
  const __amdgpu_buffer_rsrc_t rs_B = make_rsrc(reinterpret_cast<const TI*>(a.B) + (int64_t)b * a.B_bs + (int64_t)g * a.B_gs,
                                                (uint32_t)((15 * a.B_ns + L_) * (int64_t)sizeof(TI)));
  const __amdgpu_buffer_rsrc_t rs_C = make_rsrc(reinterpret_cast<const TI*>(a.C) + (int64_t)b * a.C_bs + (int64_t)g * a.C_gs,
                                                (uint32_t)((15 * a.C_ns + L_) * (int64_t)sizeof(TI)));
  const int bcn = lane & 15, bcq = lane >> 4;
  const uint32_t bo_B = (uint32_t)((bcn * a.B_ns + 8 * bcq) * (int64_t)sizeof(TI));
  const uint32_t bo_C = (uint32_t)((bcn * a.C_ns + 8 * bcq) * (int64_t)sizeof(TI));

  // ---- projected delta: token-major dpx rows of this batch (rank values per token, 8-B pieces), the
  // wave's 32 rows of dpw; tokens past L read 0 (their delta is masked in the staging anyway)
  const __amdgpu_buffer_rsrc_t rs_px =
      make_rsrc(kPD ? reinterpret_cast<const TI*>(a.dpx) + (int64_t)b * a.dpx_bs : reinterpret_cast<const TI*>(a.u),
                kPD ? (uint32_t)(((int64_t)(L_ - 1) * a.dpx_ts + a.rank) * (int64_t)sizeof(TI)) : 0u);
  const __amdgpu_buffer_rsrc_t rs_pw =
      make_rsrc(kPD ? reinterpret_cast<const TI*>(a.dpw) + (int64_t)dbase * a.dpw_ds : reinterpret_cast<const TI*>(a.u),
                kPD ? (uint32_t)(((int64_t)(nrows - 1) * a.dpw_ds + a.rank) * (int64_t)sizeof(TI)) : 0u);

  // ---- recurrence lane constants: channel ch, states [8h, 8h + 8)
  const bool my_ok = ch < nrows;
  const int my_dc = dbase + min(ch, nrows - 1);
  f32x2 A2[kPH / 2];
#pragma unroll
  for (int p = 0; p < kPH / 2; ++p) {
    const float* ap = a.A + (int64_t)my_dc * kPN + kPH * h + 2 * p;
    A2[p] = my_ok ? f32x2{ap[0] * kLog2e, ap[1] * kLog2e} : f32x2{0.f, 0.f};
  }
  // ---- staging / gate lane constants: vector j = lane + 64 k -> row j / kVPR, block j % kVPR
  float biasv[kNV], Dv[kNV];
#pragma unroll
  for (int k = 0; k < kNV; ++k) {
    const int r = min((lane + 64 * k) / kVPR, nrows - 1);
    biasv[k] = a.delta_bias ? a.delta_bias[dbase + r] : 0.f;
    Dv[k] = a.D ? a.D[dbase + r] : 0.f;
  }
  auto voff = [&](int k, int64_t ds, int l0) {   // byte offset of this lane's vector k at chunk l0
    const int j = lane + 64 * k;
    const int r = min(j / kVPR, nrows - 1);
    return (uint32_t)(r * ds + l0 + (j % kVPR) * VI) * (uint32_t)sizeof(TI);
  };

  f32x2 x[kPH / 2];
#pragma unroll
  for (int p = 0; p < kPH / 2; ++p) x[p] = f32x2{0.f, 0.f};

  uint4 pu[kNV], pd[kNV];
  uint4 pB, pC;
  auto load_next = [&](int l0) {   // past the end: offsets fall outside the buffer ranges and read 0
#pragma unroll
    for (int k = 0; k < kNV; ++k) {
      pu[k] = buf_ld16(rs_u, voff(k, a.u_ds, l0));
      if constexpr (!kPD) pd[k] = buf_ld16(rs_d, voff(k, a.dt_ds, l0));
    }
    pB = buf_ld16(rs_B, bo_B + (uint32_t)l0 * (uint32_t)sizeof(TI));
    pC = buf_ld16(rs_C, bo_C + (uint32_t)l0 * (uint32_t)sizeof(TI));
  };

  load_next(0);
  for (int c0 = 0; c0 < a.n_chunks; ++c0) {
    const int l0 = c0 * kT;
    // ---- staging: dt = softplus(delta + bias), du = dt u as fp32 pairs; B/C chunk.  In a
    // chunk that runs past the end (L % kT != 0; L % VI == 0, so whole vectors) the vectors
    // at positions >= L stage dt = du = 0: the state stays frozen, the saved state is the one
    // after L - 1.  A uniform branch picks the masked copy, full chunks carry no selects.
    if constexpr (kPD) {
      // delta tile (32 positions x 32 channels) = dpx[l0 .., :] . dpw[rows, :]^T on 16x16x16 MFMAs:
      // lane (i = lane & 15, q = lane >> 4) feeds position / channel i and ranks [16 ks + 4q, +4), and
      // gets delta at positions 16 pb + 4q + [0, 4) of channel 16 cb + i.  Rounded to the activation
      // dtype (what the unfused dt_proj GEMM stores), then parked in the dt slots of the row buffer
      // for the staging below.
      using MM = Mfma16<TI>;
      const int i16 = lane & 15, q4 = 4 * (lane >> 4);
      f32x4 dacc[2][2];
#pragma unroll
      for (int pb = 0; pb < 2; ++pb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) dacc[pb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const uint32_t xo0 = (uint32_t)((l0 + i16) * a.dpx_ts + q4) * (uint32_t)sizeof(TI);
      const uint32_t xo1 = (uint32_t)((l0 + 16 + i16) * a.dpx_ts + q4) * (uint32_t)sizeof(TI);
      const uint32_t wo0 = (uint32_t)(min(i16, nrows - 1) * a.dpw_ds + q4) * (uint32_t)sizeof(TI);
      const uint32_t wo1 = (uint32_t)(min(16 + i16, nrows - 1) * a.dpw_ds + q4) * (uint32_t)sizeof(TI);
#pragma unroll 2
      for (int r0 = 0; r0 < a.rank; r0 += 16) {
        const uint32_t ro = (uint32_t)r0 * (uint32_t)sizeof(TI);
        const auto x0 = __builtin_bit_cast(typename MM::v4, __builtin_amdgcn_raw_buffer_load_b64(rs_px, xo0 + ro, 0, 0));
        const auto x1 = __builtin_bit_cast(typename MM::v4, __builtin_amdgcn_raw_buffer_load_b64(rs_px, xo1 + ro, 0, 0));
        const auto w0 = __builtin_bit_cast(typename MM::v4, __builtin_amdgcn_raw_buffer_load_b64(rs_pw, wo0 + ro, 0, 0));
        const auto w1 = __builtin_bit_cast(typename MM::v4, __builtin_amdgcn_raw_buffer_load_b64(rs_pw, wo1 + ro, 0, 0));
        dacc[0][0] = MM::mma(x0, w0, dacc[0][0]);
        dacc[0][1] = MM::mma(x0, w1, dacc[0][1]);
        dacc[1][0] = MM::mma(x1, w0, dacc[1][0]);
        dacc[1][1] = MM::mma(x1, w1, dacc[1][1]);
      }
#pragma unroll
      for (int pb = 0; pb < 2; ++pb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          float d[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) d[e] = to_f(from_f<TI>(dacc[pb][cb][e]));
          char* rp = rowbuf + (16 * cb + i16) * PL::kStride + (16 * pb + q4) * 8;
          reinterpret_cast<float2*>(rp)[0] = make_float2(d[0], d[1]);
          reinterpret_cast<float2*>(rp + 16)[0] = make_float2(d[2], d[3]);
        }
      wave_lds_sync();
    }
    uint4 ucur[kNV];
    auto stage = [&](auto masked) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < kNV; ++k) {
        const int j = lane + 64 * k;
        char* dst = rowbuf + (j / kVPR) * PL::kStride + (j % kVPR) * VI * 8;
        ucur[k] = pu[k];
        const bool vok = !decltype(masked)::value || l0 + (j % kVPR) * VI < L_;
        float dv[VI];
#pragma unroll
        for (int q = 0; q < VI / 2; ++q) {
          if constexpr (kPD) {
            const float2 d2 = reinterpret_cast<const float2*>(dst)[2 * q];
            dv[2 * q] = d2.x;
            dv[2 * q + 1] = d2.y;
          } else {
            dv[2 * q] = elem_f<TI>(pd[k], 2 * q);
            dv[2 * q + 1] = elem_f<TI>(pd[k], 2 * q + 1);
          }
        }
        if (kPD && a.delta_out) {   // the formed delta for the backward (rows / positions past the end dropped)
          const uint32_t ob = ((j / kVPR) < nrows && l0 + (j % kVPR) * VI < L_) ? 0u : 0x80000000u;
          buf_st16(rs_d, voff(k, a.dt_ds, l0) | ob, pack_f<TI>(dv));
        }
#pragma unroll
        for (int q = 0; q < VI / 2; ++q) {   // two positions per packed op
          const f32x2 dr = f32x2{dv[2 * q], dv[2 * q + 1]} + biasv[k];
          f32x2 dt = kSP ? softplus2_log1p(dr) : dr;
          f32x2 du = dt * f32x2{elem_f<TI>(pu[k], 2 * q), elem_f<TI>(pu[k], 2 * q + 1)};
          if constexpr (decltype(masked)::value) {   // u past L may be anything (stride padding): mask du too
            dt = vok ? dt : f32x2{0.f, 0.f};
            du = vok ? du : f32x2{0.f, 0.f};
          }
          reinterpret_cast<float4*>(dst)[q] = make_float4(dt.x, dt.y, du.x, du.y);
        }
      }
    };
    if (l0 + kT <= L_) stage(std::false_type());
    else stage(std::true_type());
    {   // B / C chunk -> [position][B 16 | C 16] fp32 (lanes j, j + 16 share a bank: 2-way, free on ds_write_b32)
      float* dst = bcl + (8 * bcq) * (2 * kPN) + bcn;
#pragma unroll
      for (int e = 0; e < VI; ++e) {
        dst[e * (2 * kPN)] = elem_f<TI>(pB, e);
        dst[e * (2 * kPN) + kPN] = elem_f<TI>(pC, e);
      }
    }
    wave_lds_sync();
    load_next(l0 + kT);
    uint4 cz[kNV];
    if (hasZ) {
#pragma unroll
      for (int k = 0; k < kNV; ++k) cz[k] = buf_ld16(rs_z, voff(k, a.z_ds, l0));
    }

    // ---- recurrence: 8 states of one channel per lane, groups of kPG positions.  The
    // next position's B/C halves and the next group's {dt, du} are read one step
    // ahead (software pipeline), so the LDS latency sits under the current step.
    {
      const char* row = rowbuf + ch * PL::kStride;
      const f32x4* bcp = reinterpret_cast<const f32x4*>(bcl + kPH * h);   // position stride 2kN floats = 8 f32x4
      f32x4 nb0 = bcp[0], nb1 = bcp[1], nc0 = bcp[kPN / 4], nc1 = bcp[kPN / 4 + 1];
      f32x4 nq0 = *reinterpret_cast<const f32x4*>(row), nq1 = *reinterpret_cast<const f32x4*>(row + 16);
      // two groups (8 positions = the fine saved-state interval) per iteration; the fine-state store
      // is a compile-time branch after the pair (a runtime test inside the pipelined loop cost ~50 %)
#pragma unroll 1
      for (int t8 = 0; t8 < kT; t8 += 2 * kPG) {
#pragma unroll
      for (int gi = 0; gi < 2; ++gi) {
        const int t0 = t8 + gi * kPG;
        const f32x4 q0 = nq0, q1 = nq1;
        {
          const int tn = (t0 + kPG) & (kT - 1);   // (last group: wraps to an unused re-read)
          nq0 = *reinterpret_cast<const f32x4*>(row + tn * 8);
          nq1 = *reinterpret_cast<const f32x4*>(row + tn * 8 + 16);
        }
        float yv[kPG];
#pragma unroll
        for (int e = 0; e < kPG; ++e) {
          const f32x4 b0 = nb0, b1 = nb1, c0v = nc0, c1v = nc1;
          {
            const f32x4* np = bcp + ((t0 + e + 1) & (kT - 1)) * (2 * kPN / 4);
            nb0 = np[0]; nb1 = np[1]; nc0 = np[kPN / 4]; nc1 = np[kPN / 4 + 1];
          }
          __builtin_amdgcn_sched_barrier(0);   // keep the reads a step ahead (the scheduler sinks them to their use)
          f32x2 dA[kPH / 2];
          // dt / du of position e: the low half of their register pairs (odd e: moved there once,
          // scan_common.h hi_to_lo), broadcast by the packed ops
          const f32x2 dtp = (e & 1) ? hi_to_lo(e < 2 ? q0.xy : q1.xy) : (e < 2 ? q0.xy : q1.xy);
          const f32x2 dup = (e & 1) ? hi_to_lo(e < 2 ? q0.zw : q1.zw) : (e < 2 ? q0.zw : q1.zw);
#pragma unroll
          for (int p = 0; p < kPH / 2; ++p) {
            const f32x2 arg = pk_mul_bcast<0>(A2[p], dtp);
            if (p < MC_FWD_POLY_PAIRS) dA[p] = exp2_poly2(arg);   // A/B lever (default 0: all v_exp_f32)
            else dA[p] = f32x2{fast_exp2(arg.x), fast_exp2(arg.y)};
          }
          x[0] = pk_fma_bcast<0>(b0.lo, dup, dA[0] * x[0]);
          x[1] = pk_fma_bcast<0>(b0.hi, dup, dA[1] * x[1]);
          x[2] = pk_fma_bcast<0>(b1.lo, dup, dA[2] * x[2]);
          x[3] = pk_fma_bcast<0>(b1.hi, dup, dA[3] * x[3]);
          f32x2 y2 = c0v.lo * x[0];
          y2 = c0v.hi * x[1] + y2;
          y2 = c1v.lo * x[2] + y2;
          y2 = c1v.hi * x[3] + y2;
          yv[e] = y2.x + y2.y;
        }
        // partial y over the {dt, du} bytes both lanes of the pair have consumed
        *reinterpret_cast<float4*>(const_cast<char*>(row) + t0 * 8 + 16 * h) = make_float4(yv[0], yv[1], yv[2], yv[3]);
      }
        if constexpr (kFine) {
          if (l0 + t8 + 2 * kPG <= L_ && my_ok) {
            // fine interval: the state after position l0 + t8 + 7 (L % 8 == 0: the last one is L - 1),
            // position-major [b][n_states][dim][16]: the wave's 32 rows of one position are 2 KB contiguous
            float4* cs = reinterpret_cast<float4*>(
                a.chunk_states + (((int64_t)b * a.n_states + (l0 + t8) / kFineS) * a.dim + dbase + ch) * kPN + kPH * h);
            cs[0] = make_float4(x[0].x, x[0].y, x[1].x, x[1].y);
            cs[1] = make_float4(x[2].x, x[2].y, x[3].x, x[3].y);
          }
        }
      }
    }
    if (!kFine && a.chunk_states && my_ok && c0 < a.n_states) {   // state after l0 + kT - 1 (kS == kT)
      float4* cs = reinterpret_cast<float4*>(a.chunk_states +
                                             (((int64_t)b * a.dim + dbase + ch) * a.n_states + c0) * kPN + kPH * h);
      cs[0] = make_float4(x[0].x, x[0].y, x[1].x, x[1].y);
      cs[1] = make_float4(x[2].x, x[2].y, x[3].x, x[3].y);
    }
    wave_lds_sync();

    // ---- gate + store: y = y_h0 + y_h1 + D u, out = y silu(z), coalesced 16-B vectors
#pragma unroll
    for (int k = 0; k < kNV; ++k) {
      const int j = opaque_lane_id() + 64 * k;
      const int r = j / kVPR;
      const char* src = rowbuf + r * PL::kStride + (j % kVPR) * VI * 8;
      float o[VI];
#pragma unroll
      for (int gi = 0; gi < VI / kPG; ++gi) {
        const f32x4 ya = reinterpret_cast<const f32x4*>(src)[2 * gi];
        const f32x4 yb = reinterpret_cast<const f32x4*>(src)[2 * gi + 1];
#pragma unroll
        for (int i = 0; i < kPG; i += 2) {
          const int e = gi * kPG + i;
          const f32x2 uu = f32x2{elem_f<TI>(ucur[k], e), elem_f<TI>(ucur[k], e + 1)};
          const f32x2 y = Dv[k] * uu + (f32x2{ya[i], ya[i + 1]} + f32x2{yb[i], yb[i + 1]});
          o[e] = y.x;
          o[e + 1] = y.y;
        }
      }
      // rows past the group end and vectors past L: out of range, dropped
      const uint32_t ob = (r < nrows && l0 + (j % kVPR) * VI < L_) ? 0u : 0x80000000u;
      if (hasZ) {
        if (a.out_y) buf_st16(rs_y, voff(k, a.y_ds, l0) | ob, pack_f<TI>(o));
#pragma unroll
        for (int e = 0; e < VI; e += 2) {
          const f32x2 g = silu2(f32x2{elem_f<TI>(cz[k], e), elem_f<TI>(cz[k], e + 1)}) * f32x2{o[e], o[e + 1]};
          o[e] = g.x;
          o[e + 1] = g.y;
        }
      }
      if constexpr (MC_FWD_NT_STORE) buf_st16_nt(rs_o, voff(k, a.o_ds, l0) | ob, pack_f<TI>(o));
      else buf_st16(rs_o, voff(k, a.o_ds, l0) | ob, pack_f<TI>(o));
    }
    wave_lds_sync();   // next chunk's staging overwrites the rows
  }

  if (a.last_state && my_ok) {
    float4* ls = reinterpret_cast<float4*>(a.last_state + ((int64_t)b * a.dim + dbase + ch) * kPN + kPH * h);
    ls[0] = make_float4(x[0].x, x[0].y, x[1].x, x[1].y);
    ls[1] = make_float4(x[2].x, x[2].y, x[3].x, x[3].y);
  }
}

// Eligibility of the pair kernel for a (validated) forward call.
bool fwd_pair_ok(const FwdArgs& a, bool aligned, int itype_bytes, int itype, int wtype) {
  auto fits = [&](int64_t ds) {
    return ((int64_t)(kPCh - 1) * (ds < 0 ? -ds : ds) + a.seqlen) * itype_bytes < ((int64_t)1 << 31);
  };
  auto bc = [&](const void* t, int64_t bs, int64_t gs, int64_t ns) {   // 16-bit rows, 16-B aligned, 32-bit spans
    return aligned16(t) && bs % 8 == 0 && gs % 8 == 0 && ns % 8 == 0 && ns >= 0 && (15 * ns + a.seqlen) * 2 < ((int64_t)1 << 31);
  };
  return itype_bytes == 2 && wtype == itype && aligned && a.dstate == kPN && a.seqlen % 8 == 0 && kS == kT &&
         a.rev_groups == 0 && a.u_groups == 0 && fits(a.u_ds) && fits(a.dt_ds) && fits(a.o_ds) &&
         (!a.z || fits(a.z_ds)) && (!a.out_y || fits(a.y_ds)) && bc(a.B, a.B_bs, a.B_gs, a.B_ns) &&
         bc(a.C, a.C_bs, a.C_gs, a.C_ns);
}

template <typename TI, int kMinW>
static int launch_pair_t(const FwdArgs& a0, hipStream_t s) {
  FwdArgs a = a0;
  const int H = a.dim / a.n_groups;
  a.nblk = (H + kPCh - 1) / kPCh;
  a.total_blocks = a.batch * a.n_groups * a.nblk;
  const size_t lds = (size_t)PairLayout<TI>::kRowBytes + PairLayout<TI>::kBCBytes;
  const dim3 grid(a.total_blocks), block(64);
  if (a.chunk_states && a.state_interval == kFineS) {   // training forward saving fine states
    if (a.dpw) {
      if (a.softplus) hipLaunchKernelGGL((scan_fwd_pair_kernel<TI, true, kMinW, true, true>), grid, block, lds, s, a);
      else hipLaunchKernelGGL((scan_fwd_pair_kernel<TI, false, kMinW, true, true>), grid, block, lds, s, a);
    } else {
      if (a.softplus) hipLaunchKernelGGL((scan_fwd_pair_kernel<TI, true, kMinW, false, true>), grid, block, lds, s, a);
      else hipLaunchKernelGGL((scan_fwd_pair_kernel<TI, false, kMinW, false, true>), grid, block, lds, s, a);
    }
  } else if (a.dpw) {
    if (a.softplus) hipLaunchKernelGGL((scan_fwd_pair_kernel<TI, true, kMinW, true, false>), grid, block, lds, s, a);
    else hipLaunchKernelGGL((scan_fwd_pair_kernel<TI, false, kMinW, true, false>), grid, block, lds, s, a);
  } else {
    if (a.softplus) hipLaunchKernelGGL((scan_fwd_pair_kernel<TI, true, kMinW, false, false>), grid, block, lds, s, a);
    else hipLaunchKernelGGL((scan_fwd_pair_kernel<TI, false, kMinW, false, false>), grid, block, lds, s, a);
  }
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_scan_fwd: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

// 16-bit rows only (fp32 rows double the staging registers and spill at 3 waves / SIMD).
// Measured alternatives (interleaved on one box, C4 ms; built under tools/ for A/B runs):
// median softplus 2.82, the same at 4 waves/SIMD (spills) 3.59, log1p softplus 2.80,
// + op_sel broadcasts of dt / du in inline asm (this kernel) 2.78; one-channel kernel 3.26.
int launch_fwd_pair(const FwdArgs& a, int itype, hipStream_t s) {
  if (itype == MC_DTYPE_BF16) return launch_pair_t<bf16_t, 3>(a, s);
  return launch_pair_t<f16_t, 3>(a, s);
}

}  // namespace scan
}  // namespace mc
