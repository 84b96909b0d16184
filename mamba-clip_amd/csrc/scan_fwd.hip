// scan_fwd.hip -- selective-scan forward for MI355X (gfx950, CDNA4).
//
// Computes (reference semantics: /root/reference/src/mamba_clip/model.py:83-169,
// the op behind mamba_ssm's selective_scan_fn called at model.py:539-550):
//   dt   = softplus(delta + delta_bias[d])                  (optional softplus / bias)
//   x_t  = exp(dt_t * A[d,n]) * x_{t-1} + dt_t * B[b,g,n,t] * u_t
//   y_t  = sum_n C[b,g,n,t] * x_t[n]  (+ D[d] * u_t)  (* silu(z_t))
//
// Design (DESIGN.md "scan_fwd"):
//  * One lane owns one (b, d) channel and keeps its dstate states in VGPRs,
//    walking the sequence in chunks of kT = 32 positions: the work-optimal
//    form of the recurrence (no parallel-prefix overhead).  B*D channels give
//    thousands of waves at the benchmark shapes.
//  * A workgroup is ONE wave = 64 channels of one (batch, group): no
//    inter-wave barriers, fine-grained grid (no tail), XCD-aware ordering so
//    the waves of one batch share an XCD's L2.
//  * B_t / C_t are wave-uniform: a pre-pass re-lays them out as fp32
//    [b][g][l][2N]; each chunk's slice is staged in LDS and read with
//    broadcast ds_read_b128 (one address for all lanes).
//  * u / delta tiles move HBM -> registers (next chunk, prefetched under the
//    current chunk's recurrence) -> LDS with fully coalesced 16-B loads along
//    the sequence; each lane then reads back its own row (conflict-free).
//    y (+D u) is written back over the consumed row in fp32, and a
//    cooperative pass applies the z gate with coalesced z loads / out stores.
//  * exp(dt*A) = exp2(dt * A*log2e) on v_exp_f32.
#include <cstdlib>

#include "scan_common.h"


namespace mc {
namespace scan {

// FwdArgs: scan_common.h
bool fwd_pair_ok(const FwdArgs& a, bool aligned, int itype_bytes, int itype, int wtype);   // scan_fwd_pair.hip
int launch_fwd_pair(const FwdArgs& a, int itype, hipStream_t s);


// Variants (template knobs, chosen on the host):
//   kG     steps per group of the recurrence loop: the B/C values of a group
//          are read from LDS together (kG * 2 * kN VGPRs live)
//   kPBC   prefetch the next chunk's B/C into registers (else: load at staging)
//   kPU    prefetch the next chunk's u / delta into registers (else: load at staging)
//   kMinW  waves per SIMD the register budget is sized for
// At C4 (B=64, D=3072: 3072 one-wave workgroups on 1024 SIMDs) the kernel is
// VALU + v_exp issue bound (~33 SIMD cycles per wave per (t, n) step, measured
// the same at 1 and 2 waves per SIMD), not HBM bound.
// kAligned: 0 = element-wise rows, 1 = 16-B aligned rows, 2 = aligned and every chunk
// full (seqlen % kT == 0: no masked-load code at all, which keeps the register
// budget of the 3-waves-per-SIMD build free of spills)
// kSP: softplus on delta (a template flag: a runtime one is a uniform branch per position
// that splits the recurrence into small basic blocks)
template <typename TI, int kN, int kAligned, int kG, bool kPBC, bool kPU, int kMinW, bool kSP>
__global__ __launch_bounds__(kRows, kMinW) void scan_fwd_kernel(const FwdArgs a) {
  using RL = RowLayout<TI>;
  constexpr int VI = RL::VI;                    // elements per 16-B vector
  constexpr int kVPR = kT / VI;                 // vectors per row segment per array

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* rowbuf = smem;
  float* bcl = reinterpret_cast<float*>(smem + kRows * RL::kStride);   // [kT][2kN] (mode 1)

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

  const TI* __restrict__ u = reinterpret_cast<const TI*>(a.u) + (int64_t)b * a.u_bs;
  // grouped directions: reversed groups walk mirrored positions; u_groups > 0 shares u blocks
  // (vector modes: the host guarantees seqlen % VI == 0, so a mirrored 16-B block is aligned)
  const bool rev = (a.rev_groups >> g) & 1;
  const int urow0 = a.u_groups ? (g % a.u_groups) * H + dblk * kRows : dbase;
  const TI* __restrict__ dl = reinterpret_cast<const TI*>(a.delta) + (int64_t)b * a.dt_bs;
  const TI* __restrict__ zp = reinterpret_cast<const TI*>(a.z) + (int64_t)b * a.z_bs;
  TI* __restrict__ out = reinterpret_cast<TI*>(a.out) + (int64_t)b * a.o_bs;
  // (whole-chunk mode) this wave's rows of u / delta / z / out as buffer ranges: 32-bit offsets
  auto rows_rsrc = [&](const void* base, int64_t ds, int row0 = -1) {
    return make_rsrc(reinterpret_cast<const TI*>(base) + (int64_t)(row0 < 0 ? dbase : row0) * ds,
                     (uint32_t)(((int64_t)(nrows - 1) * ds + L_) * (int64_t)sizeof(TI)));
  };
  const __amdgpu_buffer_rsrc_t rs_out = rows_rsrc(out, a.o_ds);
  const __amdgpu_buffer_rsrc_t rs_u = rows_rsrc(u, a.u_ds, urow0), rs_d = rows_rsrc(dl, a.dt_ds);
  const __amdgpu_buffer_rsrc_t rs_z = rows_rsrc(hasZ ? (const void*)zp : (const void*)u, hasZ ? a.z_ds : a.u_ds);
  const __amdgpu_buffer_rsrc_t rs_y =
      rows_rsrc(a.out_y ? (const void*)(reinterpret_cast<const TI*>(a.out_y) + (int64_t)b * a.y_bs) : (const void*)u,
                a.out_y ? a.y_ds : a.u_ds);

  // ---- per-channel constants
  const int my_d = dbase + lane;
  const bool my_ok = lane < nrows;
  // states are processed in pairs with packed fp32 math (v_pk_mul_f32 / v_pk_fma_f32)
  // unconditional loads (clamped row / state index), masked afterwards: no load behind a branch
  f32x2 A2[kN / 2];
  const int my_dc = dbase + min(lane, nrows - 1);
  {
    float av[kN];
#pragma unroll
    for (int n = 0; n < kN; ++n) av[n] = a.A[(int64_t)my_dc * a.dstate + min(n, a.dstate - 1)];
#pragma unroll
    for (int n = 0; n < kN; ++n) {
      const float v = (my_ok && n < a.dstate) ? av[n] * kLog2e : 0.f;
      if (n & 1) A2[n / 2].y = v; else A2[n / 2].x = v;
    }
  }
  const float Dv = (my_ok && a.D) ? a.D[my_dc] : 0.f;
  const float biasv = (my_ok && a.delta_bias) ? a.delta_bias[my_dc] : 0.f;

  f32x2 x[kN / 2];
#pragma unroll
  for (int n = 0; n < kN / 2; ++n) x[n] = f32x2{0.f, 0.f};

  // ---- register prefetch of the next chunk (issued before this chunk's
  // recurrence, consumed after it): u / delta vectors + the B/C chunk.
  constexpr int kBCVec = kT * 2 * kN / 4;                 // float4s in one B/C chunk
  constexpr int kBCPer = (kBCVec + kRows - 1) / kRows;
  uint4 pu[kVPR], pd[kVPR];
  float4 pbc[kPBC ? kBCPer : 1];
  // (whole-chunk mode) this (batch, group)'s B/C rows as a buffer range: chunks past
  // the end read 0, so the prefetch needs no branch (a branch around loads makes the
  // compiler drain the stores issued after them before the loads may be consumed)
  const __amdgpu_buffer_rsrc_t rs_bc = make_rsrc(a.bct + (int64_t)bg * L_ * (2 * kN), (uint32_t)L_ * (2 * kN) * 4u);
  auto load_bc = [&](int l0, float4 (&dst)[kBCPer]) {
    if constexpr (kAligned == 2) {
#pragma unroll
      for (int k = 0; k < kBCPer; ++k) {
        const int v = lane + k * kRows;
        const uint32_t off = v < kBCVec ? (uint32_t)(l0 * (2 * kN) + 4 * v) * 4u : 0x80000000u;
        dst[k] = __builtin_bit_cast(float4, buf_ld16(rs_bc, off));
      }
      return;
    }
    const float4* src = reinterpret_cast<const float4*>(a.bct + ((int64_t)bg * L_ + l0) * (2 * kN));
    const int nvec = min(kT, L_ - l0) * (2 * kN) / 4;
#pragma unroll
    for (int k = 0; k < kBCPer; ++k) {
      const int v = lane + k * kRows;
      dst[k] = v < nvec ? src[v] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto load_regs = [&](int l0) {
    const bool full = kAligned == 2 || (kAligned == 1 && l0 + kT <= L_);
#pragma unroll
    for (int k = 0; k < kVPR; ++k) {
      const int j = lane + k * kRows;
      const int r = j / kVPR, c = j % kVPR;
      const int rr = min(r, nrows - 1);   // rows past the group end: load a valid row, never stored
      const int col0 = l0 + c * VI;
      if constexpr (kAligned == 2) {   // 32-bit offsets into the wave's row block (no 64-bit pointers)
        // reversed group: ascending mirrored block (mc_common.h ld16_rev; past the end it goes
        // negative -> wraps out of range for row 0, reads an unused neighbour otherwise: never consumed)
        const int cm = rev ? L_ - l0 - kT + c * VI : col0;
        // (element order is reversed at staging: touching the values here would wait for the loads)
        pu[k] = buf_ld16(rs_u, (uint32_t)(rr * a.u_ds + cm) * (uint32_t)sizeof(TI));
        pd[k] = buf_ld16(rs_d, (uint32_t)(rr * a.dt_ds + cm) * (uint32_t)sizeof(TI));
        continue;
      }
      if (rev) {
        const int nv = max(0, min(VI, L_ - (l0 + (kVPR - 1 - c) * VI)));   // steps < L of block kVPR-1-c
        const int cm = L_ - l0 - kT + c * VI;
        pu[k] = ld16_top(u + (int64_t)(urow0 + rr) * a.u_ds, cm, nv);   // flipped at staging
        pd[k] = ld16_top(dl + (int64_t)(dbase + rr) * a.dt_ds, cm, nv);
        continue;
      }
      const TI* su = u + (int64_t)(urow0 + rr) * a.u_ds + col0;
      const TI* sd = dl + (int64_t)(dbase + rr) * a.dt_ds + col0;
      if (full) {
        pu[k] = ld16(su);
        pd[k] = ld16(sd);
      } else {
        const int nv = max(0, min(VI, L_ - col0));
        pu[k] = ld16_masked(su, nv);
        pd[k] = ld16_masked(sd, nv);
      }
    }
    if constexpr (kPBC) load_bc(l0, pbc);
  };

  if constexpr (kPU) load_regs(0);
  for (int ch = 0; ch < a.n_chunks; ++ch) {
    const int l0 = ch * kT;
    const bool full = kAligned == 2 || (kAligned == 1 && l0 + kT <= L_);
    if constexpr (!kPU) load_regs(l0);   // other resident waves cover the latency

    // ---- stage u / delta (vector j = lane + k*64 -> row j / kVPR, col j % kVPR) and B/C
#pragma unroll
    for (int k = 0; k < kVPR; ++k) {
      const int j = lane + k * kRows;
      const int r = j / kVPR, c = j % kVPR;
      char* blk = rowbuf + r * RL::kStride + (rev ? kVPR - 1 - c : c) * RL::kBlock;   // reversed: mirrored block
      st16(blk, rev ? reverse_elems<TI>(pu[k]) : pu[k]);        // mirrored blocks arrive in memory order
      st16(blk + 16, rev ? reverse_elems<TI>(pd[k]) : pd[k]);
    }
    {
      float4 cur[kBCPer];
      if constexpr (kPBC) {
#pragma unroll
        for (int k = 0; k < kBCPer; ++k) cur[k] = pbc[k];
      } else {
        load_bc(l0, cur);   // L2-resident (shared by the waves of this batch); latency once per chunk
      }
#pragma unroll
      for (int k = 0; k < kBCPer; ++k) {
        const int v = lane + k * kRows;
        if (v < kBCVec) reinterpret_cast<float4*>(bcl)[v] = cur[k];
      }
    }
    wave_lds_sync();
    if constexpr (kPU) {
      if constexpr (kAligned == 2) load_regs(l0 + kT);   // past the end: out-of-range offsets read 0
      else if (ch + 1 < a.n_chunks) load_regs(l0 + kT);
    }
    // this chunk's z vectors (gate pass mapping), loaded now so that they arrive
    // under the recurrence instead of stalling the gate pass
    uint4 cz[kVPR];
    if (hasZ) {
      const int ln = kAligned == 2 ? opaque_lane_id() : lane;   // rebuilt here, not held live
#pragma unroll
      for (int k = 0; k < kVPR; ++k) {
        const int j = ln + k * kRows;
        const int r = j / kVPR, c = j % kVPR;
        const int col0 = l0 + c * VI;
        if constexpr (kAligned == 2) {
          cz[k] = buf_ld16(rs_z, (uint32_t)(min(r, nrows - 1) * a.z_ds + col0) * (uint32_t)sizeof(TI));
        } else {
          const TI* zs = zp + (int64_t)(dbase + min(r, nrows - 1)) * a.z_ds + col0;
          cz[k] = full ? ld16(zs) : ld16_masked(zs, max(0, min(VI, L_ - col0)));
        }
      }
    }

    // ---- the recurrence over this chunk, one channel per lane.  Steps go
    // in groups of kG: read the group's u / delta (kG elements each), run
    // kG steps, write the kG fp32 y values back over exactly those bytes.
    {
      char* row = rowbuf + lane * RL::kStride;
#pragma unroll 1
      for (int t0 = 0; t0 < kT; t0 += kG) {
        char* pu = row + (t0 / VI) * RL::kBlock + (t0 % VI) * (int)sizeof(TI);
        char* pd = pu + 16;
        float uu[kG], dd[kG];
        {
          constexpr int kB = kG * (int)sizeof(TI);   // bytes of one array in this group
          uint4 qa, qb;
          if constexpr (kB == 16) { qa = ld16(pu); qb = ld16(pd); }
          else if constexpr (kB == 8) {
            const uint2 a2 = *reinterpret_cast<const uint2*>(pu), b2 = *reinterpret_cast<const uint2*>(pd);
            qa = make_uint4(a2.x, a2.y, 0u, 0u); qb = make_uint4(b2.x, b2.y, 0u, 0u);
          } else if constexpr (kB == 4) {
            qa = make_uint4(*reinterpret_cast<const uint32_t*>(pu), 0u, 0u, 0u);
            qb = make_uint4(*reinterpret_cast<const uint32_t*>(pd), 0u, 0u, 0u);
          } else {
            static_assert(kB >= 4, "group must cover >= 4 bytes per array");
          }
#pragma unroll
          for (int e = 0; e < kG; ++e) { uu[e] = elem_f<TI>(qa, e); dd[e] = elem_f<TI>(qb, e); }
        }
        float yv[kG];
#pragma unroll
        for (int e = 0; e < kG; ++e) {
          const int t = l0 + t0 + e;
          const float uv = uu[e];
          const float dr = dd[e] + biasv;
          float dt = kSP ? softplus_f(dr) : dr;
          if constexpr (kAligned != 2) dt = (t < L_) ? dt : 0.f;  // past the end: state frozen
          const float du = dt * uv;
          // every decay of this position first: each exp's result is consumed a
          // few pairs later, so no wait states sit between an exp and its use
          f32x2 dA[kN / 2];
#pragma unroll
          for (int p = 0; p < kN / 2; ++p) {
            const f32x2 arg = A2[p] * dt;                                   // v_pk_mul_f32
            dA[p] = f32x2{fast_exp2(arg.x), fast_exp2(arg.y)};
          }
          f32x2 y2 = {0.f, 0.f};
          {
            const f32x4* bc4 = reinterpret_cast<const f32x4*>(bcl + (t0 + e) * (2 * kN));
#pragma unroll
            for (int n4 = 0; n4 < kN / 4; ++n4) {
              const f32x4 bq = bc4[n4], cq = bc4[kN / 4 + n4];
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const int p = 2 * n4 + h;
                const f32x2 bb = h ? bq.hi : bq.lo, cc = h ? cq.hi : cq.lo;
                x[p] = dA[p] * x[p] + bb * du;                              // v_pk_mul + v_pk_fma
                y2 = cc * x[p] + y2;                                        // v_pk_fma
              }
            }
          }
          yv[e] = fmaf(Dv, uv, y2.x + y2.y);
        }
        // y[0..kG/2) -> the u bytes, y[kG/2..kG) -> the delta bytes of this group
        if (a.chunk_states && my_ok && ((t0 + kG) % kS) == 0) {
          const int sc = (l0 + t0 + kG) / kS - 1;   // saved-state index: state after position sc*kS + kS - 1
          if (sc < a.n_states) {
            float* cs = a.chunk_states + (((int64_t)b * a.dim + my_d) * a.n_states + sc) * a.dstate;
            if ((a.dstate & 3) == 0) {
#pragma unroll
              for (int n4 = 0; n4 < kN / 4; ++n4)
                if (n4 * 4 < a.dstate)
                  reinterpret_cast<float4*>(cs)[n4] =
                      make_float4(x[2 * n4].x, x[2 * n4].y, x[2 * n4 + 1].x, x[2 * n4 + 1].y);
            } else {
#pragma unroll
              for (int n = 0; n < kN; ++n)
                if (n < a.dstate) cs[n] = (n & 1) ? x[n / 2].y : x[n / 2].x;
            }
          }
        }
        if constexpr (kG == 4) {
          *reinterpret_cast<float2*>(pu) = make_float2(yv[0], yv[1]);
          *reinterpret_cast<float2*>(pd) = make_float2(yv[2], yv[3]);
        } else {
          static_assert(kG == 2, "kG in {2, 4}");
          *reinterpret_cast<float*>(pu) = yv[0];
          *reinterpret_cast<float*>(pd) = yv[1];
        }
      }
    }
    wave_lds_sync();

    // ---- gate + store, coalesced along the sequence (same vector mapping)
    const int lg = kAligned == 2 ? opaque_lane_id() : lane;   // offsets rebuilt, not held live
#pragma unroll
    for (int k = 0; k < kVPR; ++k) {
      const int j = lg + k * kRows;
      const int r = j / kVPR, c = j % kVPR;
      const int cl = rev ? kVPR - 1 - c : c;          // LDS block of this lane's vector
      const int col0 = l0 + c * VI;
      const int cm = L_ - l0 - kT + c * VI;            // (reversed) ascending mirrored position
      const int nv = max(0, min(VI, L_ - (l0 + cl * VI)));
      float o[VI];
      // y of step s (within the chunk) lives in group s / kG: first half of the
      // group's y values at the u bytes, second half at the delta bytes.
#pragma unroll
      for (int e = 0; e < VI; ++e) {
        const int st = cl * VI + e;
        const int g0 = st - st % kG;
        const int ie = st % kG;
        const char* pu = rowbuf + r * RL::kStride + (g0 / VI) * RL::kBlock + (g0 % VI) * (int)sizeof(TI);
        o[e] = reinterpret_cast<const float*>(ie < kG / 2 ? pu : pu + 16)[ie % (kG / 2)];
      }
      if (hasZ) {
        if (a.out_y && r < nrows) {
          if constexpr (kAligned == 2) {
            buf_st16(rs_y, (uint32_t)(r * a.y_ds + col0) * (uint32_t)sizeof(TI), pack_f<TI>(o));
          } else {
            TI* ydst = reinterpret_cast<TI*>(a.out_y) + (int64_t)b * a.y_bs + (int64_t)(dbase + r) * a.y_ds + col0;
            const uint4 yq = pack_f<TI>(o);
            if (full) st16(ydst, yq);
            else st16_masked(ydst, yq, nv);
          }
        }
#pragma unroll
        for (int e = 0; e < VI; ++e) o[e] *= silu_f(elem_f<TI>(cz[k], e));
      }
      if constexpr (kAligned == 2) {
        // whole chunks: every lane stores (rows past the group end fall outside the
        // buffer range and are dropped), so the store count is static and the next
        // chunk's prefetch wait does not have to drain these stores
        const uint32_t off = r < nrows ? (uint32_t)(r * a.o_ds + (rev ? cm : col0)) * (uint32_t)sizeof(TI) : 0x80000000u;
        const uint4 ov = pack_f<TI>(o);
        buf_st16(rs_out, off, rev ? reverse_elems<TI>(ov) : ov);
      } else if (r < nrows) {
        const uint4 ov = pack_f<TI>(o);
        if (rev) {
          st16_rev(out + (int64_t)(dbase + r) * a.o_ds, cm, ov, nv);
        } else {
          TI* dst = out + (int64_t)(dbase + r) * a.o_ds + col0;
          if (full) st16(dst, ov);
          else st16_masked(dst, ov, nv);
        }
      }
    }
    wave_lds_sync();  // next chunk's staging overwrites the rows
  }

  if (a.last_state && my_ok) {
    float* ls = a.last_state + ((int64_t)b * a.dim + my_d) * a.dstate;
#pragma unroll
    for (int n = 0; n < kN; ++n)
      if (n < a.dstate) ls[n] = (n & 1) ? x[n / 2].y : x[n / 2].x;
  }
}

typedef __attribute__((address_space(4))) const f32x4 cf32x4;   // constant address space: scalar loads

// Row layout of the 16-position chunk variants: per row {u vector, delta vector} blocks + 16-B pad.
template <typename TI>
struct RowLayoutP {
  static constexpr int kTP = 16;
  static constexpr int VI = ElemTraits<TI>::kVec;
  static constexpr int kBlock = 32;                 // {u vector, delta vector}
  static constexpr int kBlocks = kTP / VI;
  static constexpr int kStride = kBlocks * kBlock + 16;
};

// ------------------------------------------------------------------ multi-channel-per-lane variant
// kR channels per lane (a wave owns 64*kR channels of one (batch, group)):
// the kR recurrences are independent, so they interleave in one instruction
// stream and hide each other's latencies (ILP instead of resident waves), and
// each position's B/C row -- loaded once per wave into SGPRs -- serves kR
// times the work.  At C4 (B=64, D=3072) kR = 3 gives 1024 waves: exactly one
// per SIMD, no tail round.  u / delta / z of the next chunk are prefetched
// into registers during the current chunk (z too: the gate pass never waits
// on HBM).
template <typename TI, int kN, int kR, bool kAligned, bool kSP>
__global__ __launch_bounds__(kRows, kR == 1 ? 3 : 1) void scan_fwd_mc_kernel(const FwdArgs a) {
  using RL = RowLayoutP<TI>;
  constexpr int kTP = RL::kTP;
  constexpr int VI = RL::VI;
  constexpr int kVPR = kTP / VI;                  // vectors per row per array
  constexpr int kQ = kN / 4;
  constexpr int kW = kRows * kR;                  // channels per wave
  constexpr int kVL = kR * kVPR;                  // staged vectors per lane per array
  static_assert(kS % kTP == 0, "saved states fall on chunk ends");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* rowbuf = smem;                            // [kW][RL::kStride]

  const int lane = threadIdx.x;
  const int lin = xcd_remap(blockIdx.x, a.total_blocks);
  const int dblk = lin % a.nblk;
  const int bg = lin / a.nblk;
  const int g = bg % a.n_groups, b = bg / a.n_groups;
  const int H = a.dim / a.n_groups;
  const int dbase = g * H + dblk * kW;
  const int nrows = min(kW, H - dblk * kW);
  const int L_ = a.seqlen;
  const bool hasZ = a.z != nullptr;
  const int n_chunks = (L_ + kTP - 1) / kTP;

  const TI* __restrict__ u = reinterpret_cast<const TI*>(a.u) + (int64_t)b * a.u_bs;
  const TI* __restrict__ dl = reinterpret_cast<const TI*>(a.delta) + (int64_t)b * a.dt_bs;
  const TI* __restrict__ zp = reinterpret_cast<const TI*>(a.z) + (int64_t)b * a.z_bs;
  TI* __restrict__ out = reinterpret_cast<TI*>(a.out) + (int64_t)b * a.o_bs;
  const cf32x4* bcs = (const cf32x4*)(a.bct + (int64_t)bg * L_ * (2 * kN));

  // channel r of this lane: row lane + 64 r of the wave's block
  f32x2 A2[kR][kN / 2], x[kR][kN / 2];
  float Dv[kR], biasv[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int row = lane + kRows * r;
    const bool ok = row < nrows;
    const int d = dbase + min(row, nrows - 1);
#pragma unroll
    for (int n = 0; n < kN; ++n) {
      const float v = (ok && n < a.dstate) ? a.A[(int64_t)d * a.dstate + n] * kLog2e : 0.f;
      if (n & 1) A2[r][n / 2].y = v; else A2[r][n / 2].x = v;
    }
    Dv[r] = (ok && a.D) ? a.D[d] : 0.f;
    biasv[r] = (ok && a.delta_bias) ? a.delta_bias[d] : 0.f;
#pragma unroll
    for (int p = 0; p < kN / 2; ++p) x[r][p] = f32x2{0.f, 0.f};
  }

  // staged vector k of this lane: j = lane + 64 k -> row j / kVPR, column block j % kVPR
  uint4 pu[kVL], pd[kVL], pz[kVL];
  auto load_regs = [&](int l0) {
    const bool full = kAligned && (l0 + kTP <= L_);
#pragma unroll
    for (int k = 0; k < kVL; ++k) {
      const int j = lane + k * kRows;
      const int r = j / kVPR, c = j % kVPR;
      const int rr = min(r, nrows - 1);
      const int col0 = l0 + c * VI;
      const TI* su = u + (int64_t)(dbase + rr) * a.u_ds + col0;
      const TI* sd = dl + (int64_t)(dbase + rr) * a.dt_ds + col0;
      const TI* sz = zp + (int64_t)(dbase + rr) * a.z_ds + col0;
      if (full) {
        pu[k] = ld16(su);
        pd[k] = ld16(sd);
        if (hasZ) pz[k] = ld16(sz);
      } else {
        const int nv = max(0, min(VI, L_ - col0));
        pu[k] = ld16_masked(su, nv);
        pd[k] = ld16_masked(sd, nv);
        if (hasZ) pz[k] = ld16_masked(sz, nv);
      }
    }
  };
  auto load_bc = [&](int t, f32x4 (&dst)[2 * kQ]) {
    const cf32x4* src = bcs + (int64_t)min(t, L_ - 1) * (2 * kQ);
#pragma unroll
    for (int k = 0; k < 2 * kQ; ++k) dst[k] = src[k];
  };

  f32x4 bcA[2 * kQ], bcB[2 * kQ];
  load_bc(0, bcA);
  load_regs(0);
  for (int ch = 0; ch < n_chunks; ++ch) {
    const int l0 = ch * kTP;
    const bool full = kAligned && (l0 + kTP <= L_);
#pragma unroll
    for (int k = 0; k < kVL; ++k) {
      const int j = lane + k * kRows;
      const int r = j / kVPR, c = j % kVPR;
      char* blk = rowbuf + r * RL::kStride + c * RL::kBlock;
      st16(blk, pu[k]);
      st16(blk + 16, pd[k]);
    }
    uint4 cz[kVL];
#pragma unroll
    for (int k = 0; k < kVL; ++k) cz[k] = pz[k];
    wave_lds_sync();
    uint4 ru[kR][kVPR], rd[kR][kVPR];
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const char* rowp = rowbuf + (lane + kRows * r) * RL::kStride;
#pragma unroll
      for (int k = 0; k < kVPR; ++k) {
        ru[r][k] = ld16(rowp + k * RL::kBlock);
        rd[r][k] = ld16(rowp + k * RL::kBlock + 16);
      }
    }
    if (ch + 1 < n_chunks) load_regs(l0 + kTP);

    auto step = [&](int tt, const f32x4 (&cur)[2 * kQ], f32x4 (&nxt)[2 * kQ]) {
      const int t = l0 + tt;
      __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0): cur (issued a position ago) is back
      __builtin_amdgcn_sched_barrier(0);
      load_bc(t + 1, nxt);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const float uv = elem_f<TI>(ru[r][tt / VI], tt % VI);
        const float dr = elem_f<TI>(rd[r][tt / VI], tt % VI) + biasv[r];
        float dt = kSP ? softplus_f(dr) : dr;   // template flag: no per-position branch
        dt = (t < L_) ? dt : 0.f;
        const float du = dt * uv;
        f32x2 ya = {0.f, 0.f}, yb = {0.f, 0.f};
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
          const f32x4 bq = cur[q], cq = cur[kQ + q];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int p = 2 * q + h;
            const f32x2 bb = h ? bq.hi : bq.lo, cc = h ? cq.hi : cq.lo;
            const f32x2 arg = A2[r][p] * dt;
            const f32x2 dA = {fast_exp2(arg.x), fast_exp2(arg.y)};
            x[r][p] = dA * x[r][p] + bb * du;
            if (h) yb = cc * x[r][p] + yb;
            else ya = cc * x[r][p] + ya;
          }
        }
        const f32x2 ys = ya + yb;
        reinterpret_cast<float*>(rowbuf + (lane + kRows * r) * RL::kStride)[tt] = fmaf(Dv[r], uv, ys.x + ys.y);
      }
    };
#pragma unroll
    for (int tt = 0; tt < kTP; tt += 2) {
      step(tt, bcA, bcB);
      step(tt + 1, bcB, bcA);
    }
    // saved state after every kS positions and after the last chunk (positions
    // past L froze the state, so that one is the state after position L-1)
    if (a.chunk_states && (((l0 + kTP) % kS) == 0 || ch == n_chunks - 1)) {
      const int sc = (l0 + kTP + kS - 1) / kS - 1;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const int row = lane + kRows * r;
        if (row < nrows && sc < a.n_states) {
          float* cs = a.chunk_states + (((int64_t)b * a.dim + dbase + row) * a.n_states + sc) * a.dstate;
          if ((a.dstate & 3) == 0) {
#pragma unroll
            for (int n4 = 0; n4 < kN / 4; ++n4)
              if (n4 * 4 < a.dstate)
                reinterpret_cast<float4*>(cs)[n4] =
                    make_float4(x[r][2 * n4].x, x[r][2 * n4].y, x[r][2 * n4 + 1].x, x[r][2 * n4 + 1].y);
          } else {
#pragma unroll
            for (int n = 0; n < kN; ++n)
              if (n < a.dstate) cs[n] = (n & 1) ? x[r][n / 2].y : x[r][n / 2].x;
          }
        }
      }
    }
    wave_lds_sync();

    // ---- gate + store, coalesced along the sequence (z prefetched a chunk ago)
#pragma unroll
    for (int k = 0; k < kVL; ++k) {
      const int j = lane + k * kRows;
      const int r = j / kVPR, c = j % kVPR;
      const int col0 = l0 + c * VI;
      const int nv = max(0, min(VI, L_ - col0));
      float o[VI];
      const float4* yv = reinterpret_cast<const float4*>(rowbuf + r * RL::kStride + c * VI * 4);
#pragma unroll
      for (int e4 = 0; e4 < VI / 4; ++e4) {
        const float4 q = yv[e4];
        o[4 * e4] = q.x; o[4 * e4 + 1] = q.y; o[4 * e4 + 2] = q.z; o[4 * e4 + 3] = q.w;
      }
      if (hasZ) {
        if (a.out_y && r < nrows) {
          TI* ydst = reinterpret_cast<TI*>(a.out_y) + (int64_t)b * a.y_bs + (int64_t)(dbase + r) * a.y_ds + col0;
          const uint4 yq = pack_f<TI>(o);
          if (full) st16(ydst, yq);
          else st16_masked(ydst, yq, nv);
        }
#pragma unroll
        for (int e = 0; e < VI; ++e) o[e] *= silu_f(elem_f<TI>(cz[k], e));
      }
      if (r < nrows) {
        TI* dst = out + (int64_t)(dbase + r) * a.o_ds + col0;
        const uint4 ov = pack_f<TI>(o);
        if (full) st16(dst, ov);
        else st16_masked(dst, ov, nv);
      }
    }
    wave_lds_sync();
  }

#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int row = lane + kRows * r;
    if (a.last_state && row < nrows) {
      float* ls = a.last_state + ((int64_t)b * a.dim + dbase + row) * a.dstate;
#pragma unroll
      for (int n = 0; n < kN; ++n)
        if (n < a.dstate) ls[n] = (n & 1) ? x[r][n / 2].y : x[r][n / 2].x;
    }
  }
}

template <typename TI, int kN, int kR>
static int launch_fwd_mc(const FwdArgs& a0, bool aligned, hipStream_t s) {
  FwdArgs a = a0;
  const int H = a.dim / a.n_groups;
  a.nblk = (H + kRows * kR - 1) / (kRows * kR);
  a.total_blocks = a.batch * a.n_groups * a.nblk;
  const size_t lds = (size_t)kRows * kR * RowLayoutP<TI>::kStride;
  if (aligned && a.softplus)
    hipLaunchKernelGGL((scan_fwd_mc_kernel<TI, kN, kR, true, true>), dim3(a.total_blocks), dim3(kRows), lds, s, a);
  else if (aligned)
    hipLaunchKernelGGL((scan_fwd_mc_kernel<TI, kN, kR, true, false>), dim3(a.total_blocks), dim3(kRows), lds, s, a);
  else if (a.softplus)
    hipLaunchKernelGGL((scan_fwd_mc_kernel<TI, kN, kR, false, true>), dim3(a.total_blocks), dim3(kRows), lds, s, a);
  else
    hipLaunchKernelGGL((scan_fwd_mc_kernel<TI, kN, kR, false, false>), dim3(a.total_blocks), dim3(kRows), lds, s, a);
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_scan_fwd: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

// ------------------------------------------------------------------ host dispatch
template <typename TI, int kN, int kG, bool kPBC, bool kPU, int kMinW>
static int launch_fwd_v(const FwdArgs& a, bool aligned, hipStream_t s) {
  const size_t lds = (size_t)kRows * RowLayout<TI>::kStride + (size_t)kT * 2 * kN * 4;
  auto fits = [&](int64_t ds) {
    return ((int64_t)(kRows - 1) * (ds < 0 ? -ds : ds) + a.seqlen) * (int64_t)sizeof(TI) < ((int64_t)1 << 31);
  };
  const bool span32 = fits(a.o_ds) && fits(a.u_ds) && fits(a.dt_ds) && (!a.z || fits(a.z_ds)) &&
                      (!a.out_y || fits(a.y_ds));
#define MC_FWD_LAUNCH(AL, SP) \
  hipLaunchKernelGGL((scan_fwd_kernel<TI, kN, AL, kG, kPBC, kPU, kMinW, SP>), dim3(a.total_blocks), dim3(kRows), lds, s, a)
  const bool sp = a.softplus != 0;
  if (aligned && a.seqlen % kT == 0 && span32) { if (sp) MC_FWD_LAUNCH(2, true); else MC_FWD_LAUNCH(2, false); }
  else if (aligned) { if (sp) MC_FWD_LAUNCH(1, true); else MC_FWD_LAUNCH(1, false); }
  else { if (sp) MC_FWD_LAUNCH(0, true); else MC_FWD_LAUNCH(0, false); }
#undef MC_FWD_LAUNCH
  const hipError_t e = hipGetLastError();
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_scan_fwd: launch failed: %s", hipGetErrorString(e));
  return MC_OK;
}

// Kernel choice, measured on MI355X (tools/ab_scan_fwd.sh; ms, bf16, z, softplus):
//                                         C4 64x3072x4096   C2 256x1536x80
//   scan_fwd_kernel (kG 4, LDS B/C, 2 w/SIMD)     3.17 (r01: 3.35) 0.204
//   scan_fwd_mc_kernel R=1 (SGPR B/C, 16-pos)     3.87             0.152
//   scan_fwd_mc_kernel R=3 (1 w/SIMD)             3.66             0.180
// Rejected (kept in git history): per-position LDS broadcast at 3 w/SIMD
// 3.96 / 0.188; two-wave state split with SGPR half-rows 6.41 / 0.266; two-wave
// state split with LDS-staged rows and LDS partial-y sums (no 2+1 tail: 6
// half-tasks per SIMD) 3.92 at C4 -- the per-position work both waves repeat
// (row reads, softplus, y hand-off) costs more than the tail it removes;
// vector-load B/C rings spill at the occupancy they need.  With short
// sequences the grid is many short-lived waves and the SGPR-fed kernel wins;
// with long ones the LDS-staged kernel's deeper prefetch wins.
// A/B variants of this choice are built under tools/ (git history has the rejected kernels).
template <typename TI, int kN>
static int launch_fwd_n(const FwdArgs& a, bool aligned, hipStream_t s) {
  if (a.seqlen <= 512) return launch_fwd_mc<TI, kN, 1>(a, aligned, s);
  return launch_fwd_v<TI, kN, 4, true, true, sizeof(TI) == 4 ? 1 : 2>(a, aligned, s);   // fp32: see launch_fwd_dirs
}

template <typename TI>
static int launch_fwd_dirs(const FwdArgs& a, bool aligned, hipStream_t s) {
  // fp32 rows double the prefetch registers: one wave per SIMD keeps them out of scratch
  // (the SS2D grids are a few hundred waves, occupancy buys nothing there)
  constexpr int kW = sizeof(TI) == 4 ? 1 : 2;
  const int np = padded_dstate(a.dstate);
  if (np == 8) return launch_fwd_v<TI, 8, 4, true, true, kW>(a, aligned, s);
  if (np == 16) return launch_fwd_v<TI, 16, 4, true, true, kW>(a, aligned, s);
  return launch_fwd_v<TI, 32, 4, true, true, kW>(a, aligned, s);
}

template <typename TI>
static int launch_fwd_t(const FwdArgs& a, bool aligned, hipStream_t s) {
  const int np = padded_dstate(a.dstate);
  if (np == 8) return launch_fwd_n<TI, 8>(a, aligned, s);
  if (np == 16) return launch_fwd_n<TI, 16>(a, aligned, s);
  return launch_fwd_n<TI, 32>(a, aligned, s);
}

int validate_common(int batch, int dim, int seqlen, int dstate, int n_groups, int itype, int wtype, const char* who) {
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

bool vec_ok(const void* p, int64_t s0, int64_t s1, int64_t s2, int elem_bytes) {
  const int64_t v = 16 / elem_bytes;
  return p == nullptr || (aligned16(p) && s0 % v == 0 && s1 % v == 0 && s2 % v == 0);
}

}  // namespace scan
}  // namespace mc

// ------------------------------------------------------------------ C ABI
using namespace mc;
using namespace mc::scan;

extern "C" int32_t mc_scan_n_chunks(int32_t seqlen) { return seqlen <= 0 ? 0 : (seqlen + kS - 1) / kS; }

extern "C" int32_t mc_scan_n_states(int32_t seqlen, int32_t state_interval) {
  const int S = state_interval > 0 ? state_interval : kS;
  return seqlen <= 0 ? 0 : (seqlen + S - 1) / S;
}

extern "C" size_t mc_scan_chunk_states_bytes(int32_t batch, int32_t dim, int32_t seqlen, int32_t dstate) {
  return (size_t)batch * dim * mc_scan_n_chunks(seqlen) * dstate * sizeof(float);
}

extern "C" size_t mc_scan_fwd_workspace_bytes(int32_t batch, int32_t seqlen, int32_t dstate, int32_t n_groups) {
  return bct_bytes(batch, seqlen, dstate, n_groups);
}

static bool fill_fwd_args(const mc_scan_fwd_params* p, FwdArgs& a, bool& aligned);

extern "C" int mc_scan_fwd(const mc_scan_fwd_params* p, void* stream) {
  MC_CHECK(p != nullptr, MC_ERR_INVALID, "mc_scan_fwd: null params");
  int rc = validate_common(p->batch, p->dim, p->seqlen, p->dstate, p->n_groups, p->itype, p->wtype, "mc_scan_fwd");
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (p->batch == 0 || p->seqlen == 0) {
    // nothing to scan; a zero-length sequence leaves the state at zero
    if (p->last_state && p->batch > 0)
      (void)hipMemsetAsync(p->last_state, 0, (size_t)p->batch * p->dim * p->dstate * 4, s);
    return MC_OK;
  }
  const bool proj = p->delta_proj_w != nullptr;
  MC_CHECK(p->u && (p->delta || proj) && p->A && p->B && p->C && p->out, MC_ERR_INVALID,
           "mc_scan_fwd: u, delta (or delta_proj_w / delta_proj_x), A, B, C and out must be non-null");
  if (proj) {
    const int64_t L = p->seqlen, R = p->delta_rank;
    MC_CHECK(p->delta_proj_x && R >= 16 && R <= 256 && R % 16 == 0, MC_ERR_SHAPE,
             "mc_scan_fwd: projected delta needs delta_proj_x and delta_rank in [16, 256], a multiple of 16 (got %d)",
             p->delta_rank);
    MC_CHECK(p->dpx_token_stride >= R && p->dpx_token_stride % 4 == 0 && p->dpx_batch_stride % 4 == 0 &&
                 p->dpw_dim_stride >= R && p->dpw_dim_stride % 4 == 0 &&
                 reinterpret_cast<uintptr_t>(p->delta_proj_x) % 8 == 0 &&
                 reinterpret_cast<uintptr_t>(p->delta_proj_w) % 8 == 0 &&
                 ((L - 1) * p->dpx_token_stride + R) * 2 < ((int64_t)1 << 31) &&
                 (31 * p->dpw_dim_stride + R) * 2 < ((int64_t)1 << 31),
             MC_ERR_SHAPE, "mc_scan_fwd: projected delta operands need 8-B aligned rows (strides %% 4 == 0), "
             "token stride >= delta_rank and 32-bit spans");
  }
  const size_t need = bct_bytes(p->batch, p->seqlen, p->dstate, p->n_groups);
  MC_CHECK(p->workspace && p->workspace_bytes >= need && aligned16(p->workspace), MC_ERR_WORKSPACE,
           "mc_scan_fwd: workspace must be >= %zu bytes and 16-B aligned (got %zu)", need, p->workspace_bytes);

  const bool dirs = p->reverse_groups != 0 || p->u_groups != 0;
  if (dirs) {
    MC_CHECK(!p->z && p->u_groups >= 0 && p->u_groups <= p->n_groups && p->n_groups <= 31 &&
                 (p->reverse_groups >> p->n_groups) == 0,
             MC_ERR_SHAPE, "mc_scan_fwd: reverse_groups / u_groups need no z, 0 <= u_groups <= n_groups <= 31 and "
             "a mask within n_groups (got mask 0x%x, u_groups %d, n_groups %d)", p->reverse_groups, p->u_groups,
             p->n_groups);
  }
  FwdArgs a;
  bool aligned = false;
  const bool pair = fill_fwd_args(p, a, aligned);
  const int ib = p->itype == MC_DTYPE_F32 ? 4 : 2;
  (void)dirs;
  MC_CHECK(p->state_interval == 0 || p->state_interval == kS || (p->state_interval == kFineS && pair), MC_ERR_SHAPE,
           "mc_scan_fwd: state_interval %d: 0 / %d, or %d on the pair kernel's shapes (mc_scan_fwd_state_interval)",
           p->state_interval, kS, kFineS);
  // 16-bit rows, N = 16: state-split lane pairs (scan_fwd_pair.hip; C4 2.78 vs 3.22 ms, C2 training
  // forward 0.166 vs 0.183 ms per layer).  It reads B / C rows itself: no relayout pre-pass.
  if (pair) return launch_fwd_pair(a, p->itype, s);
  hipError_t e = relayout_bc(p->wtype, p->B, p->C, p->B_batch_stride, p->B_group_stride, p->B_dstate_stride,
                             p->C_batch_stride, p->C_group_stride, p->C_dstate_stride, p->batch, p->n_groups,
                             p->seqlen, p->dstate, dirs ? p->reverse_groups : 0,
                             reinterpret_cast<float*>(p->workspace), s);
  MC_CHECK(e == hipSuccess, MC_ERR_LAUNCH, "mc_scan_fwd: B/C relayout launch failed: %s", hipGetErrorString(e));
  if (dirs) {   // per-group addressing lives in the LDS-staged kernel (vector modes: seqlen % VI == 0)
    MC_CHECK(!proj, MC_ERR_SHAPE, "mc_scan_fwd: projected delta and grouped directions do not combine");
    const bool al = aligned && p->seqlen % (16 / ib) == 0;
    if (p->itype == MC_DTYPE_F32) return launch_fwd_dirs<float>(a, al, s);
    if (p->itype == MC_DTYPE_BF16) return launch_fwd_dirs<bf16_t>(a, al, s);
    return launch_fwd_dirs<f16_t>(a, al, s);
  }
  MC_CHECK(!proj, MC_ERR_SHAPE, "mc_scan_fwd: projected delta needs the pair kernel's shapes (16-bit rows, "
           "dstate 16, seqlen %% 8 == 0, 16-B aligned rows, no grouped directions)");
  if (p->itype == MC_DTYPE_F32) return launch_fwd_t<float>(a, aligned, s);
  if (p->itype == MC_DTYPE_BF16) return launch_fwd_t<bf16_t>(a, aligned, s);
  return launch_fwd_t<f16_t>(a, aligned, s);
}

extern "C" int32_t mc_scan_fwd_kernel(const mc_scan_fwd_params* p) {
  if (!p || p->batch == 0 || p->seqlen == 0) return MC_SCAN_KERNEL_NONE;
  if (p->reverse_groups != 0 || p->u_groups != 0) return MC_SCAN_KERNEL_DIRS;
  FwdArgs a;
  bool aligned = false;
  return fill_fwd_args(p, a, aligned) ? MC_SCAN_KERNEL_PAIR : MC_SCAN_KERNEL_GENERIC;
}

extern "C" int32_t mc_scan_fwd_state_interval(const mc_scan_fwd_params* p) {
  if (!p || p->state_interval != kFineS) return kS;
  FwdArgs a;
  bool aligned = false;
  return fill_fwd_args(p, a, aligned) ? kFineS : kS;
}

// FwdArgs from validated params; returns whether the pair kernel takes the call.  a.state_interval is
// the fine interval only when requested and the pair kernel runs (the others save every kS).
static bool fill_fwd_args(const mc_scan_fwd_params* p, FwdArgs& a, bool& aligned) {
  const bool proj = p->delta_proj_w != nullptr;
  const bool dirs = p->reverse_groups != 0 || p->u_groups != 0;
  a.batch = p->batch; a.dim = p->dim; a.seqlen = p->seqlen; a.dstate = p->dstate; a.n_groups = p->n_groups;
  a.n_chunks = (p->seqlen + kT - 1) / kT;
  a.n_states = mc_scan_n_chunks(p->seqlen);
  const int H = p->dim / p->n_groups;
  a.nblk = (H + kRows - 1) / kRows;
  a.total_blocks = p->batch * p->n_groups * a.nblk;
  a.softplus = p->delta_softplus;
  a.u_bs = p->u_batch_stride; a.u_ds = p->u_dim_stride;
  a.dt_bs = p->delta_batch_stride; a.dt_ds = p->delta_dim_stride;
  a.z_bs = p->z_batch_stride; a.z_ds = p->z_dim_stride;
  a.o_bs = p->out_batch_stride; a.o_ds = p->out_dim_stride;
  a.u = p->u; a.delta = p->delta; a.A = p->A; a.bct = reinterpret_cast<const float*>(p->workspace);
  a.D = p->D; a.z = p->z; a.delta_bias = p->delta_bias;
  a.out = p->out; a.chunk_states = p->chunk_states; a.last_state = p->last_state;
  a.out_y = p->z ? p->out_y : nullptr; a.y_bs = p->out_y_batch_stride; a.y_ds = p->out_y_dim_stride;
  a.rev_groups = dirs ? p->reverse_groups : 0; a.u_groups = dirs ? p->u_groups : 0;
  a.dpx = p->delta_proj_x; a.dpw = p->delta_proj_w; a.rank = p->delta_rank;
  a.dpx_bs = p->dpx_batch_stride; a.dpx_ts = p->dpx_token_stride; a.dpw_ds = p->dpw_dim_stride;
  a.delta_out = proj ? p->delta_out : nullptr;
  a.B = p->B; a.C = p->C;
  a.B_bs = p->B_batch_stride; a.B_gs = p->B_group_stride; a.B_ns = p->B_dstate_stride;
  a.C_bs = p->C_batch_stride; a.C_gs = p->C_group_stride; a.C_ns = p->C_dstate_stride;

  const int ib = p->itype == MC_DTYPE_F32 ? 4 : 2;
  aligned = vec_ok(p->u, p->u_batch_stride, p->u_dim_stride, 0, ib) &&
            vec_ok(proj ? p->delta_out : p->delta, p->delta_batch_stride, p->delta_dim_stride, 0, ib) &&
            vec_ok(p->z, p->z_batch_stride, p->z_dim_stride, 0, ib) &&
            vec_ok(p->out, p->out_batch_stride, p->out_dim_stride, 0, ib) &&
            vec_ok(a.out_y, a.y_bs, a.y_ds, 0, ib);
  const bool pair = !dirs && fwd_pair_ok(a, aligned, ib, p->itype, p->wtype);
  a.state_interval = (pair && p->state_interval == kFineS) ? kFineS : kS;
  a.n_states = mc_scan_n_states(p->seqlen, a.state_interval);
  return pair;
}
