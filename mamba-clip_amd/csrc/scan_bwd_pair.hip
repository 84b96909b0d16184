// scan_bwd_pair.hip -- selective-scan backward with state-split lane pairs (every 16-bit, N = 16,
// L % 8 == 0 call: the C2 and C4 text towers).
//
// Reverse mode of scan_fwd_pair.hip (reference semantics /root/reference/src/mamba_clip/model.py:83-169;
// the op behind selective_scan_cuda.bwd that mamba_ssm's SelectiveScanFn calls, model.py:539-550):
//   gy_t = dout_t silu(z_t),  lam_t,n = C_t,n gy_t + a_{t+1},n lam_{t+1},n       (a_t = exp(dt_t A))
//   dC_t,n = sum_d gy_t x_t,n          dB_t,n = sum_d lam_t,n dt_t u_t
//   du_t = D gy_t + dt_t S_t,  S_t = sum_n lam_t,n B_t,n
//   ddelta_t = (u_t S_t + Q_t) sigmoid(delta_t + bias),  Q_t = sum_n lam_t,n a_t,n x_{t-1},n A_n
//   dz_t = dout_t silu'(z_t) (Y_t + D u_t),  Y_t = sum_n C_t,n x_t,n   (recomputed: the forward stores no y)
//   dA_n = sum_{b,t} lam a x_{t-1} dt,  dD = sum gy u,  dbias = sum ddelta
//
// Layout: the forward's lane pairs.  A wave owns 32 channels of one (batch, group);
// lane 2c + h keeps states [8h, 8h + 8) of channel c as 4 packed fp32 pairs, so every state-
// position op is one v_pk_* for two states, and a wave is one workgroup's quarter (kQW waves share
// the dB / dC reduction).  Per 32-position chunk (the forward's saved-state interval), in reverse:
//  * B / C of the chunk: 16-bit rows read once per wave (one 16-B vector per lane and array),
//    converted and laid out in LDS as {B_n, B_n+1, C_n, C_n+1} quads per (position, lane half, pair);
//  * the per-position scalars dt = softplus(delta + bias), dt u, gy: each lane converts its 4
//    positions of an 8-position sub-tile (8-B row loads), the pair partner's 4 arrive by DPP;
//  * recompute pass: states at the sub-tile starts 8 / 16 / 24 from the saved chunk state (VGPRs);
//  * sub-tiles in reverse, pairs one at a time: forward sweep (x_t, a_t in VGPRs), dC products,
//    reverse adjoint sweep with packed S / Q / Y / dA accumulators, dB products; dB / dC are summed
//    over the wave's 32 channels in registers (permlane swaps + DPP, packed adds) and over the
//    workgroup's waves in LDS once per chunk, then written to a per-workgroup slab (fixed order:
//    deterministic; scan_bwd.hip's reduce kernels sum the slabs);
//  * each lane finishes its own 4 positions of the sub-tile (S / Q / Y of the partner by DPP) and
//    stores du / ddelta / dz as 8-B row pieces.
// Requirements (host-checked): dstate == 16, 16-bit u / delta / z / dout / gradients with 16-B
// aligned rows, 16-B aligned B / C rows, seqlen % 8 == 0, 32-bit row spans, no grouped directions.
#include "scan_common.h"

namespace mc {
namespace scan {

constexpr int kQW = 4;            // waves per workgroup
constexpr int kQCh = 32;          // channels per wave
constexpr int kQN = 16;           // dstate
constexpr int kQP = 4;            // state pairs per lane
constexpr int kQT = 8;            // positions per sub-tile
constexpr int kQSub = kS / kQT;   // sub-tiles per chunk
static_assert(kS == 32 && kQSub == 4 && kFineS == kQT, "the pair backward walks the forward's 32-position chunks "
              "in 8-position sub-tiles (the fine saved-state interval)");

struct BwdPairArgs {
  int batch, dim, seqlen, n_groups, n_states, nblk, total_blocks;
  int state_ratio;    // saved states per 32-position chunk: 1 (interval 32) or 4 (interval 8: no recompute)
  int64_t u_bs, u_ds, dt_bs, dt_ds, z_bs, z_ds, go_bs, go_ds;
  int64_t du_bs, du_ds, ddt_bs, ddt_ds, dz_bs, dz_ds;
  int64_t B_bs, B_gs, B_ns, C_bs, C_gs, C_ns;
  const void* u; const void* delta; const void* z; const void* dout;
  const void* B; const void* C;
  const float* A; const float* D; const float* delta_bias; const float* chunk_states;
  void* du; void* ddelta; void* dz;
  float* slab_bc;     // [b*G+g][nblk][seqlen][2][16]: dB partials, then dC partials
  float* slab_a;      // [b][16][dim]
  float* slab_d;      // [b][dim]
  float* slab_bias;   // [b][dim]
  // projected delta (mc_scan.h): delta re-formed per chunk from dpx / dpw, as the forward did
  const void* dpx; const void* dpw; int rank;
  int64_t dpx_bs, dpx_ts, dpw_ds;
};

// quad_perm DPP move (bound_ctrl: a disabled source reads 0 -- never the case here)
template <int kCtrl>
__device__ __forceinline__ float qperm(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kCtrl, 0xF, 0xF, true));
}
constexpr int kQpEven = 0xA0;   // [0,0,2,2]: the even lane of each pair
constexpr int kQpOdd = 0xF5;    // [1,1,3,3]: the odd lane
constexpr int kQpXor1 = 0xB1;   // [1,0,3,2]
constexpr int kQpXor2 = 0x4E;   // [2,3,0,1]
__device__ __forceinline__ float row_xor8(float v) {   // row_ror:8 == lane ^ 8 inside a 16-lane row
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, true));
}
__device__ __forceinline__ float row_xor4(float v) {   // banks 0 / 2 take lane + 4, banks 1 / 3 lane - 4
  const int iv = __float_as_int(v);
  const int lo = __builtin_amdgcn_update_dpp(iv, iv, 0x104, 0xF, 0x5, false);
  return __int_as_float(__builtin_amdgcn_update_dpp(lo, iv, 0x114, 0xF, 0xA, false));
}

// Halving stages inside a 16-lane row with bank-masked DPP adds (inline asm: hipcc cannot express
// a write-masked DPP op).  halve_bit3: lanes with bit 3 clear return a + a[lane ^ 8], the others
// b + b[lane ^ 8]; halve_bit2: bit 2 clear -> a + a[lane + 4], set -> b + b[lane - 4].  The leading
// s_nop 1 covers the VALU-write -> DPP-read hazard (hipcc pads nothing inside asm).  Same sums,
// same order as the select form (own + partner).
#ifndef MC_BWD_SELECT_HALVES
__device__ __forceinline__ float halve_bit3(float a, float b) {
  float r;
  asm volatile("s_nop 1\n\t"
               "v_add_f32_dpp %0, %1, %1 row_ror:8 row_mask:0xf bank_mask:0x3\n\t"
               "v_add_f32_dpp %0, %2, %2 row_ror:8 row_mask:0xf bank_mask:0xc" MC_ASM_TAIL
               : "=&v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float halve_bit2(float a, float b) {
  float r;
  asm volatile("s_nop 1\n\t"
               "v_add_f32_dpp %0, %1, %1 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
               "v_add_f32_dpp %0, %2, %2 row_shr:4 row_mask:0xf bank_mask:0xa" MC_ASM_TAIL
               : "=&v"(r) : "v"(a), "v"(b));
  return r;
}
#else
// A/B (hazard audit): the same halvings as keep / send selects around compiler DPP moves
__device__ __forceinline__ float halve_bit3(float a, float b) {
  const bool hi = (__lane_id() >> 3) & 1;
  const float keep = hi ? b : a, send = hi ? a : b;
  return keep + row_xor8(send);
}
__device__ __forceinline__ float halve_bit2(float a, float b) {
  const bool hi = (__lane_id() >> 2) & 1;
  const float keep = hi ? b : a, send = hi ? a : b;
  return keep + row_xor4(send);
}
#endif

// Finishing of one position's state sums: lanes of half h keep pair (h ? b : a) and add the partner
// lane's (lane ^ 1) other pair, each pair summed over its two states first.  The two pair sums and
// the DPP add are asm so that the compiler neither SLP-packs the sums (it did, into more
// instructions) nor keeps the DPP move apart from the add: 2 adds, 2 selects, 1 DPP add instead
// of 4 selects, 2 adds, a DPP move and an add.  Same sums, same order as before.
#ifndef MC_BWD_C_FINISH
__device__ __forceinline__ float pair_finish(f32x2 a, f32x2 b, int h) {
  float sa, sb, r;
  asm(MC_ASM_HEAD "v_add_f32_e32 %0, %1, %2" MC_ASM_TAIL : "=v"(sa) : "v"(a.x), "v"(a.y));
  asm(MC_ASM_HEAD "v_add_f32_e32 %0, %1, %2" MC_ASM_TAIL : "=v"(sb) : "v"(b.x), "v"(b.y));
  const float keep = h ? sb : sa, send = h ? sa : sb;
  asm("s_nop 1\n\t"
      "v_add_f32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" MC_ASM_TAIL
      : "=v"(r) : "v"(send), "v"(keep));
  return r;
}
#else
__device__ __forceinline__ float pair_finish(f32x2 a, f32x2 b, int h) {   // A/B (hazard audit): compiler code
  const float sa = a.x + a.y, sb = b.x + b.y;
  const float keep = h ? sb : sa, send = h ? sa : sb;
  return keep + qperm<kQpXor1>(send);
}
#endif

// Sum of 16 per-lane values (8 packed pairs, value k = 2t + s in v[t].{x|y}) over the 32 lanes of
// the same lane bit 0 (the wave's 32 channels).  Lane l ends with value k = l >> 2 (lanes l and l ^ 2
// hold the same sum).  Halving stages over lane bits 5, 4 (permlane swaps, packed adds), 3, 2 (DPP),
// then a full add over bit 1.  (An LDS transpose -- 16 b32 writes, 4 b128 reads, 8 packed adds --
// cut the VALU count by a fifth but measured 9 % slower: the round trip sits on each pair's path.)
__device__ __forceinline__ float pair_reduce16(f32x2 (&v)[8], int lane) {
  // gfx950: v_permlane*_swap must not read a VGPR within 2 wait states of the VALU op that wrote it.  The
  // compiler pads its own producers (s_nop 1) but gives an inline-asm producer only 1 wait state, and
  // v[] comes from pk_mul_bcast (asm).  Routing the operands through an s_nop 1 that "defines" them puts
  // >= 2 wait states between the last product and the first swap (tools/hazard_scan.py).
  asm volatile("s_nop 1" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
               "+v"(v[7]));
#ifdef MC_BWD_BPERMUTE   // diagnostic: the two cross-row halvings through ds_bpermute, no permlane swaps
  {
    const bool up32 = lane & 32, up16 = lane & 16;
    const int p32 = (lane ^ 32) << 2, p16 = (lane ^ 16) << 2;
    auto xch = [](int addr, float v) { return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v))); };
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f32x2 keep = up32 ? v[t + 4] : v[t], send = up32 ? v[t] : v[t + 4];
      v[t] = keep + f32x2{xch(p32, send.x), xch(p32, send.y)};
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f32x2 keep = up16 ? v[t + 2] : v[t], send = up16 ? v[t] : v[t + 2];
      v[t] = keep + f32x2{xch(p16, send.x), xch(p16, send.y)};
    }
  }
#else
#pragma unroll
  for (int t = 0; t < 4; ++t) {   // bit 5: t <-> t + 4
    auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[t].x), __float_as_uint(v[t + 4].x), false, false);
    auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[t].y), __float_as_uint(v[t + 4].y), false, false);
#ifdef MC_PERMLANE_NOP
    asm volatile("s_nop 4" : "+v"(rx[0]), "+v"(rx[1]), "+v"(ry[0]), "+v"(ry[1]));
#endif
    v[t] = f32x2{__uint_as_float(rx[0]), __uint_as_float(ry[0])} + f32x2{__uint_as_float(rx[1]), __uint_as_float(ry[1])};
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {   // bit 4: t <-> t + 2
    auto rx = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[t].x), __float_as_uint(v[t + 2].x), false, false);
    auto ry = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[t].y), __float_as_uint(v[t + 2].y), false, false);
#ifdef MC_PERMLANE_NOP
    asm volatile("s_nop 4" : "+v"(rx[0]), "+v"(rx[1]), "+v"(ry[0]), "+v"(ry[1]));
#endif
    v[t] = f32x2{__uint_as_float(rx[0]), __uint_as_float(ry[0])} + f32x2{__uint_as_float(rx[1]), __uint_as_float(ry[1])};
  }
#endif
  // bit 3: t = 0 <-> 1 and bit 2: s = 0 <-> 1 as bank-masked DPP adds (each half of a 16-lane row
  // writes its own sum), instead of keep / send selects around a DPP move
  const float x = halve_bit3(v[0].x, v[1].x), y = halve_bit3(v[0].y, v[1].y);
  const float r = halve_bit2(x, y);
  return r + qperm<kQpXor2>(r);   // bit 1
}

// One global_load_lds_dwordx4: 16 B per lane from gsrc to LDS byte address m0v + 16 * lane (m0v wave-
// uniform).  asm, so the compiler's waitcnt pass does not drain it early; the caller waits with
// s_waitcnt vmcnt(0) before reading the slots.  M0 is compiler-reserved: saved and restored here.
__device__ __forceinline__ void glds16_asm(const void* gsrc, uint32_t m0v) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(m0v) : "memory");
}

template <typename TI>
__device__ __forceinline__ uint2 buf_ld8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ void buf_st8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint2 v) {
  typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, off, 0, 0);
}
template <typename TI>
__device__ __forceinline__ f32x2 elem2(uint2 w, int i) {   // elements 2i, 2i + 1 of 4 packed 16-bit values
  const uint4 q = make_uint4(w.x, w.y, 0u, 0u);
  return f32x2{elem_f<TI>(q, 2 * i), elem_f<TI>(q, 2 * i + 1)};
}

#ifdef MC_BWD_DEBUG
// Diagnostic build only: per (workgroup, wave, chunk, sub-tile, lane) snapshots of the reverse
// sweep's carries, written to a library-owned buffer that the host copies out (mc_debug_copy).
__device__ float* g_dbg = nullptr;
constexpr int kDbgVals = 32;   // floats per lane and sub-tile: hcar[4] (8), dA2[4] (8), A2[4] (8), entry state (8)
#endif

template <typename TI, bool kSP, bool kZ, bool kPD, bool kFine>
__global__ __launch_bounds__(64 * kQW, 2) void scan_bwd_pair_kernel(const BwdPairArgs a) {
  using TW = TI;                               // B / C in the activation dtype (x_dbl rows)
  constexpr int kWV = 16 / (int)sizeof(TW);   // B / C elements per 16-B vector
  constexpr int kWL = 8 / kWV;                 // vectors per lane and array (8 positions)
  constexpr int kDbcW = kS * 2 * kQN;          // dB / dC floats per wave and chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  f32x4* bcq = reinterpret_cast<f32x4*>(smem) + wave * (kS * 2 * kQP);                    // [t][h][p]
  float* dbc_base = reinterpret_cast<float*>(smem + (size_t)kQW * kS * 2 * kQP * 16);     // [buf][wave][t][2][16]
  f32x4* xst = reinterpret_cast<f32x4*>(dbc_base + 2 * kQW * kDbcW) + wave * ((kQSub - 1) * 2 * 64);   // [s][2][lane]
  // projected delta: this wave's chunk tile [channel][position] in the activation dtype (2 KB)
  char* dlt = reinterpret_cast<char*>(reinterpret_cast<f32x4*>(dbc_base + 2 * kQW * kDbcW) + kQW * ((kQSub - 1) * 2 * 64)) +
              wave * (kQCh * kS * 2);

  const int lin = xcd_remap(blockIdx.x, a.total_blocks);
  const int wblk = lin % a.nblk;
  const int bg = lin / a.nblk;
  const int g = bg % a.n_groups, b = bg / a.n_groups;
  const int H = a.dim / a.n_groups;
  const int row0 = wblk * (kQCh * kQW) + wave * kQCh;
  const int nrows = max(0, min(kQCh, H - row0));   // 0: the wave only joins the barriers (zero partials)
  const int ch = lane >> 1, h = lane & 1;
  const bool my_ok = ch < nrows;
  const int my_r = max(0, min(ch, nrows - 1));
  const int dbase = g * H + min(row0, H - 1);
  const int my_dc = dbase + my_r;
  const int L_ = a.seqlen;
  constexpr bool hasZ = kZ;

  auto rows_rsrc = [&](const void* base, int64_t bs, int64_t ds) __attribute__((always_inline)) {
    return make_rsrc(reinterpret_cast<const TI*>(base) + (int64_t)b * bs + (int64_t)dbase * ds,
                     nrows > 0 ? (uint32_t)(((int64_t)(nrows - 1) * ds + L_) * (int64_t)sizeof(TI)) : 0u);
  };
  const __amdgpu_buffer_rsrc_t rs_u = rows_rsrc(a.u, a.u_bs, a.u_ds);
  const __amdgpu_buffer_rsrc_t rs_d = rows_rsrc(a.delta, a.dt_bs, a.dt_ds);
  const __amdgpu_buffer_rsrc_t rs_z = rows_rsrc(hasZ ? a.z : a.u, hasZ ? a.z_bs : a.u_bs, hasZ ? a.z_ds : a.u_ds);
  const __amdgpu_buffer_rsrc_t rs_g = rows_rsrc(a.dout, a.go_bs, a.go_ds);
  const __amdgpu_buffer_rsrc_t rs_du = rows_rsrc(a.du, a.du_bs, a.du_ds);
  const __amdgpu_buffer_rsrc_t rs_dd = rows_rsrc(a.ddelta, a.ddt_bs, a.ddt_ds);
  const __amdgpu_buffer_rsrc_t rs_dz = rows_rsrc(hasZ ? a.dz : a.du, hasZ ? a.dz_bs : a.du_bs, hasZ ? a.dz_ds : a.du_ds);
  // element offsets of this lane's row; masked lanes write past every range (dropped)
  const uint32_t ro_u = (uint32_t)(my_r * a.u_ds), ro_d = (uint32_t)(my_r * a.dt_ds);
  const uint32_t ro_z = (uint32_t)(my_r * (hasZ ? a.z_ds : a.u_ds)), ro_g = (uint32_t)(my_r * a.go_ds);
  const uint32_t ro_du = (uint32_t)(my_r * a.du_ds), ro_dd = (uint32_t)(my_r * a.ddt_ds);
  const uint32_t ro_dz = (uint32_t)(my_r * (hasZ ? a.dz_ds : a.du_ds));
  const uint32_t st_mask = my_ok ? 0u : 0x80000000u;

  // B / C rows of this (batch, group): lane j reads state row j >> 2, positions [8 (j & 3), +8) of a chunk
  const __amdgpu_buffer_rsrc_t rs_B = make_rsrc(reinterpret_cast<const TW*>(a.B) + (int64_t)b * a.B_bs + (int64_t)g * a.B_gs,
                                                (uint32_t)((15 * a.B_ns + L_) * (int64_t)sizeof(TW)));
  const __amdgpu_buffer_rsrc_t rs_C = make_rsrc(reinterpret_cast<const TW*>(a.C) + (int64_t)b * a.C_bs + (int64_t)g * a.C_gs,
                                                (uint32_t)((15 * a.C_ns + L_) * (int64_t)sizeof(TW)));
  const uint32_t bo_B = (uint32_t)(((lane >> 2) * a.B_ns + 8 * (lane & 3)) * (int64_t)sizeof(TW));
  const uint32_t bo_C = (uint32_t)(((lane >> 2) * a.C_ns + 8 * (lane & 3)) * (int64_t)sizeof(TW));
  // saved chunk states of this wave's rows: [row][n_states][16]
  // saved states of this wave's rows: [b][row][n_states][16], or position-major [b][n_states][row][16] at the
  // fine interval (the forward's 32 rows of one position are then one contiguous 2 KB store)
  const uint32_t cs_rs = kFine ? (uint32_t)kQN : (uint32_t)(a.n_states * kQN);     // floats per row step
  const uint32_t cs_ks = kFine ? (uint32_t)(a.dim * kQN) : (uint32_t)kQN;          // floats per state step
  const __amdgpu_buffer_rsrc_t rs_cs =
      make_rsrc(a.chunk_states + (int64_t)b * a.dim * a.n_states * kQN + (int64_t)dbase * cs_rs,
                nrows > 0 ? ((uint32_t)(nrows - 1) * cs_rs + (uint32_t)(a.n_states - 1) * cs_ks + kQN) * 4u : 0u);

  // projected delta operands: token-major dpx rows of this batch, the wave's dpw rows
  const __amdgpu_buffer_rsrc_t rs_px =
      make_rsrc(kPD ? reinterpret_cast<const TI*>(a.dpx) + (int64_t)b * a.dpx_bs : reinterpret_cast<const TI*>(a.u),
                kPD ? (uint32_t)(((int64_t)(L_ - 1) * a.dpx_ts + a.rank) * (int64_t)sizeof(TI)) : 0u);
  const __amdgpu_buffer_rsrc_t rs_pw =
      make_rsrc(kPD ? reinterpret_cast<const TI*>(a.dpw) + (int64_t)dbase * a.dpw_ds : reinterpret_cast<const TI*>(a.u),
                kPD && nrows > 0 ? (uint32_t)(((int64_t)(nrows - 1) * a.dpw_ds + a.rank) * (int64_t)sizeof(TI)) : 0u);

  // ---- lane constants: pairs (8h + 2p, 8h + 2p + 1) of channel my_dc
  f32x2 A2[kQP], hcar[kQP], dA2[kQP];
#pragma unroll
  for (int p = 0; p < kQP; ++p) {
    const float* ap = a.A + (int64_t)my_dc * kQN + 8 * h + 2 * p;
    A2[p] = f32x2{ap[0], ap[1]} * kLog2e;
    hcar[p] = f32x2{0.f, 0.f};
    dA2[p] = f32x2{0.f, 0.f};
  }
  const float Dv = a.D ? a.D[my_dc] : 0.f;
  const float biasv = a.delta_bias ? a.delta_bias[my_dc] : 0.f;
  float dDacc = 0.f, dbacc = 0.f;

  // ---- software pipeline: B / C + chunk state of the next chunk; raw rows of the next sub-tile step
  uint4 pB[kWL], pC[kWL];
  f32x4 px[2];
  auto load_chunk = [&](int c) __attribute__((always_inline)) {   // c < 0: offsets out of range, reads 0
    const uint32_t lo = c >= 0 ? (uint32_t)(c * kS) * (uint32_t)sizeof(TW) : 0x80000000u;
#pragma unroll
    for (int k = 0; k < kWL; ++k) {
      pB[k] = buf_ld16(rs_B, (bo_B + lo) + (uint32_t)(k * 16));
      pC[k] = buf_ld16(rs_C, (bo_C + lo) + (uint32_t)(k * 16));
    }
    // state after chunk c - 1 (zero for c == 0): floats [8h, 8h + 8) of my row
    const uint32_t ox = c > 0 ? ((uint32_t)my_r * cs_rs + (uint32_t)(c * (kFine ? kS / kQT : 1) - 1) * cs_ks + 8 * h) * 4u
                              : 0x80000000u;
    px[0] = __builtin_bit_cast(f32x4, buf_ld16(rs_cs, ox));
    px[1] = __builtin_bit_cast(f32x4, buf_ld16(rs_cs, ox + 16));
  };
  uint2 nu, nd, nz, ng;   // raw rows (4 positions) of the next step
  auto load_raw = [&](int pos) __attribute__((always_inline)) {   // pos: first position of the sub-tile
    const uint32_t e = (uint32_t)(pos + 4 * h);
    nu = buf_ld8<TI>(rs_u, (ro_u + e) * 2u);
    if constexpr (!kPD) nd = buf_ld8<TI>(rs_d, (ro_d + e) * 2u);
    ng = buf_ld8<TI>(rs_g, (ro_g + e) * 2u);
    if constexpr (hasZ) {
      nz = buf_ld8<TI>(rs_z, (ro_z + e) * 2u);
    }
  };

  // per-position scalars of one sub-tile: this lane's 4 positions from its raw rows, the partner's by DPP
  struct Sc {
    f32x2 dt[4], dtu[4], gy[4];          // 8 positions as packed pairs
    f32x2 own_dt[2], own_gy[2];          // this lane's 4 positions (finishing)
  };
  auto scalars = [&](uint2 ru, uint2 rd, uint2 rz, uint2 rg, bool want_gy, Sc& sc) __attribute__((always_inline)) {
    f32x2 odt[2], odtu[2], ogy[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x2 r = elem2<TI>(rd, i) + biasv;
      const f32x2 dt = kSP ? softplus2_log1p(r) : r;
      odt[i] = dt;
      odtu[i] = my_ok ? dt * elem2<TI>(ru, i) : f32x2{0.f, 0.f};   // masked channels add nothing to dB / dC
      if (want_gy) {
        const f32x2 go = elem2<TI>(rg, i);
        const f32x2 gy = hasZ ? go * silu2(elem2<TI>(rz, i)) : go;
        ogy[i] = my_ok ? gy : f32x2{0.f, 0.f};
      }
    }
    // positions 0..3 of the sub-tile live in the even lane, 4..7 in the odd lane
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      sc.dt[i] = f32x2{qperm<kQpEven>(odt[i].x), qperm<kQpEven>(odt[i].y)};
      sc.dt[2 + i] = f32x2{qperm<kQpOdd>(odt[i].x), qperm<kQpOdd>(odt[i].y)};
      sc.dtu[i] = f32x2{qperm<kQpEven>(odtu[i].x), qperm<kQpEven>(odtu[i].y)};
      sc.dtu[2 + i] = f32x2{qperm<kQpOdd>(odtu[i].x), qperm<kQpOdd>(odtu[i].y)};
      if (want_gy) {
        sc.gy[i] = f32x2{qperm<kQpEven>(ogy[i].x), qperm<kQpEven>(ogy[i].y)};
        sc.gy[2 + i] = f32x2{qperm<kQpOdd>(ogy[i].x), qperm<kQpOdd>(ogy[i].y)};
        sc.own_gy[i] = ogy[i];
      }
      sc.own_dt[i] = odt[i];
    }
  };
  // B pair p / the {B, C} quad of pair p at chunk position t (LDS, two broadcast addresses per wave)
  auto bpair = [&](int t, int p) __attribute__((always_inline)) -> f32x2 {
    return reinterpret_cast<const f32x2*>(bcq + t * (2 * kQP) + h * kQP + p)[0];
  };
  auto bquad = [&](int t, int p) __attribute__((always_inline)) -> f32x4 { return bcq[t * (2 * kQP) + h * kQP + p]; };

  const int nch = (L_ + kS - 1) / kS;
  // raw rows walk: with recompute, the pass consumes sub-tiles 0 .. nsub - 2 forward and leaves the
  // last sub-tile's rows in flight; with fine saved states the main loop starts there directly
  constexpr bool fine = kFine;
  // fine states: the entries of sub-tiles 1 .. 3 of chunk c (states after positions 32 c + 8 s + 7)
  // land in the sub-tile-entry slots by LDS DMA, issued one chunk ahead (after the previous chunk's
  // sub-tile loop, when the slots are free) and waited for at the chunk start: no VGPRs held
  typedef __attribute__((address_space(3))) char lds_char_t;
  const uint32_t xst_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_char_t*)(reinterpret_cast<char*>(xst)));
  const float* cs_lane = a.chunk_states + (int64_t)b * a.dim * a.n_states * kQN + (int64_t)(dbase + my_r) * kQN + 8 * h;
  auto issue_fine = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < kQSub - 1; ++s) {
      const float* src = cs_lane + (int64_t)min(c * (kS / kQT) + s, a.n_states - 1) * cs_ks;
      glds16_asm(src, xst_lds + (uint32_t)(2 * s) * 1024u);
      glds16_asm(src + 4, xst_lds + (uint32_t)(2 * s + 1) * 1024u);
    }
  };
  if (fine) {
    issue_fine(nch - 1);
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
  }
  load_chunk(nch - 1);
  load_raw((nch - 1) * kS + (fine ? kQT * (min(kQSub, (L_ - (nch - 1) * kS) / kQT) - 1) : 0));
  int buf = 0;
  for (int c = nch - 1; c >= 0; --c) {
    const int l0 = c * kS;
    const int nsub = min(kQSub, (L_ - l0) / kQT);   // L % 8 == 0: whole sub-tiles
    float* dbc = dbc_base + (buf * kQW + wave) * kDbcW;   // double-buffered: one barrier per chunk

    // ---- B / C of the chunk -> LDS quads; chunk-start state
    {
      const int n = lane >> 2, q = lane & 3;
      float* dst = reinterpret_cast<float*>(bcq) + ((n >> 3) * kQP + ((n & 7) >> 1)) * 4 + (n & 1);
#pragma unroll
      for (int k = 0; k < kWL; ++k)
#pragma unroll
        for (int e = 0; e < kWV; ++e) {
          const int t = 8 * q + k * kWV + e;
          dst[t * (2 * kQP * 4)] = elem_f<TW>(pB[k], e);
          dst[t * (2 * kQP * 4) + 2] = elem_f<TW>(pC[k], e);
        }
    }
    if constexpr (kPD) {   // the chunk's delta tile, formed exactly as scan_fwd_pair_kernel does
      using MM = Mfma16<TI>;
      const int i16 = lane & 15, q4 = 4 * (lane >> 4);
      const int nr = max(nrows, 1);
      f32x4 dacc[2][2];
#pragma unroll
      for (int pb = 0; pb < 2; ++pb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) dacc[pb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const uint32_t xo0 = (uint32_t)((l0 + i16) * a.dpx_ts + q4) * (uint32_t)sizeof(TI);
      const uint32_t xo1 = (uint32_t)((l0 + 16 + i16) * a.dpx_ts + q4) * (uint32_t)sizeof(TI);
      const uint32_t wo0 = (uint32_t)(min(i16, nr - 1) * a.dpw_ds + q4) * (uint32_t)sizeof(TI);
      const uint32_t wo1 = (uint32_t)(min(16 + i16, nr - 1) * a.dpw_ds + q4) * (uint32_t)sizeof(TI);
#pragma unroll 2
      for (int r0 = 0; r0 < a.rank; r0 += 16) {
        const uint32_t ro = (uint32_t)r0 * (uint32_t)sizeof(TI);
        const auto x0v = __builtin_bit_cast(typename MM::v4, __builtin_amdgcn_raw_buffer_load_b64(rs_px, xo0 + ro, 0, 0));
        const auto x1v = __builtin_bit_cast(typename MM::v4, __builtin_amdgcn_raw_buffer_load_b64(rs_px, xo1 + ro, 0, 0));
        const auto w0 = __builtin_bit_cast(typename MM::v4, __builtin_amdgcn_raw_buffer_load_b64(rs_pw, wo0 + ro, 0, 0));
        const auto w1 = __builtin_bit_cast(typename MM::v4, __builtin_amdgcn_raw_buffer_load_b64(rs_pw, wo1 + ro, 0, 0));
        dacc[0][0] = MM::mma(x0v, w0, dacc[0][0]);
        dacc[0][1] = MM::mma(x0v, w1, dacc[0][1]);
        dacc[1][0] = MM::mma(x1v, w0, dacc[1][0]);
        dacc[1][1] = MM::mma(x1v, w1, dacc[1][1]);
      }
#pragma unroll
      for (int pb = 0; pb < 2; ++pb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const uint2 v = make_uint2(bits16<TI>(dacc[pb][cb][0]) | (bits16<TI>(dacc[pb][cb][1]) << 16),
                                     bits16<TI>(dacc[pb][cb][2]) | (bits16<TI>(dacc[pb][cb][3]) << 16));
          *reinterpret_cast<uint2*>(dlt + ((16 * cb + i16) * kS + 16 * pb + q4) * 2) = v;
        }
    }
    f32x2 x0[kQP];
    x0[0] = px[0].lo; x0[1] = px[0].hi; x0[2] = px[1].lo; x0[3] = px[1].hi;
    if (!my_ok) {
#pragma unroll
      for (int p = 0; p < kQP; ++p) x0[p] = f32x2{0.f, 0.f};
    }
    if (fine) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the DMA of this chunk's entries landed
    load_chunk(c - 1);
    wave_lds_sync();

    // ---- states at the starts of sub-tiles 1 .. nsub - 1 -> LDS: the forward's fine-interval states
    // (state_ratio 4: entry of sub-tile s + 1 = the state after position l0 + 8 s + 7), else recomputed
    if constexpr (fine) {   // already in LDS (issue_fine)
    } else {
      f32x2 x[kQP];
#pragma unroll
      for (int p = 0; p < kQP; ++p) x[p] = x0[p];
#pragma unroll 1
      for (int s = 0; s + 1 < nsub; ++s) {
        const uint2 ru = nu, rz = nz, rg = ng;
        const uint2 rd = kPD ? *reinterpret_cast<const uint2*>(dlt + (my_r * kS + kQT * s + 4 * h) * 2) : nd;
        load_raw(l0 + kQT * (s + 1));
        Sc sc;
        scalars(ru, rd, rz, rg, false, sc);
        // x = a x + B dt u: the product with B off the state chain (one pk_fma per step on it)
#pragma unroll
        for (int t = 0; t < kQT; ++t) {
#pragma unroll
          for (int p = 0; p < kQP; ++p) {
            const f32x2 arg = (t & 1) ? pk_mul_bcast_safe<1>(A2[p], sc.dt[t >> 1]) : pk_mul_bcast_safe<0>(A2[p], sc.dt[t >> 1]);
            const f32x2 aa = f32x2{fast_exp2(arg.x), fast_exp2(arg.y)};
            const f32x2 bb = bpair(kQT * s + t, p);
            const f32x2 bu = (t & 1) ? pk_mul_bcast_safe<1>(bb, sc.dtu[t >> 1]) : pk_mul_bcast_safe<0>(bb, sc.dtu[t >> 1]);
            x[p] = aa * x[p] + bu;
          }
        }
        xst[(2 * s) * 64 + lane] = f32x4{x[0].x, x[0].y, x[1].x, x[1].y};
        xst[(2 * s + 1) * 64 + lane] = f32x4{x[2].x, x[2].y, x[3].x, x[3].y};
      }
    }
    wave_lds_sync();

    // ---- sub-tiles in reverse
#pragma unroll 1
    for (int s = nsub - 1; s >= 0; --s) {
#ifdef MC_BWD_VM0
      __builtin_amdgcn_s_waitcnt(0x0F70);   // diagnostic: every VMEM op retired before the rows are read
#endif
      const uint2 ru = nu, rz = nz, rg = ng;
      const uint2 rd = kPD ? *reinterpret_cast<const uint2*>(dlt + (my_r * kS + kQT * s + 4 * h) * 2) : nd;
      // next step; after s = 0 the next chunk's first step (full chunk: its last sub-tile when fine)
      load_raw(s > 0 ? l0 + kQT * (s - 1) : (fine ? l0 - kQT : l0 - kS));
      Sc sc;
      scalars(ru, rd, rz, rg, true, sc);
      // state entering the sub-tile: the chunk start (registers) or the recompute pass's (LDS)
      f32x4 xi01, xi23;
      {
        const int sl = s > 0 ? s - 1 : 0;
        const f32x4 l01 = xst[(2 * sl) * 64 + lane], l23 = xst[(2 * sl + 1) * 64 + lane];
        xi01 = s > 0 ? l01 : f32x4{x0[0].x, x0[0].y, x0[1].x, x0[1].y};
        xi23 = s > 0 ? l23 : f32x4{x0[2].x, x0[2].y, x0[3].x, x0[3].y};
      }
      f32x2 S2[kQT], Q2[kQT];
      f32x2 Y2[kQT];
#pragma unroll
      for (int t = 0; t < kQT; ++t) Y2[t] = f32x2{0.f, 0.f};
#pragma unroll
      for (int t = 0; t < kQT; ++t) S2[t] = Q2[t] = f32x2{0.f, 0.f};

#pragma unroll
      for (int p = 0; p < kQP; ++p) {
        __builtin_amdgcn_sched_barrier(0);   // one pair at a time: bounded live ranges
        // Pin the pair order: this pair's inputs pass through empty volatile asm, so instruction
        // selection cannot hoist the next pair's sweep over this one (live ranges would explode).
        f32x2 a2p = A2[p];
        asm volatile("" : "+v"(a2p));
        const f32x2 xin = p == 0 ? xi01.lo : (p == 1 ? xi01.hi : (p == 2 ? xi23.lo : xi23.hi));
        // forward sweep over the sub-tile: decays and states
        f32x2 as[kQT], xs[kQT];
#pragma unroll
        for (int t = 0; t < kQT; ++t) {
          const f32x2 arg = (t & 1) ? pk_mul_bcast_safe<1>(a2p, sc.dt[t >> 1]) : pk_mul_bcast_safe<0>(a2p, sc.dt[t >> 1]);
          as[t] = f32x2{pexp2(arg.x), pexp2(arg.y)};
        }
        {   // (B dt u off the chain: one pk_fma per step on it)
          f32x2 x = xin;
#pragma unroll
          for (int t = 0; t < kQT; ++t) {
            const f32x2 bb = bpair(kQT * s + t, p);
            const f32x2 bu = (t & 1) ? pk_mul_bcast_safe<1>(bb, sc.dtu[t >> 1]) : pk_mul_bcast_safe<0>(bb, sc.dtu[t >> 1]);
            x = pfma(as[t], x, bu);
            xs[t] = x;
          }
        }
        // dC_t = sum over channels of gy_t x_t
        {
          f32x2 red[kQT];
#pragma unroll
          for (int t = 0; t < kQT; ++t)
            red[t] = (t & 1) ? pk_mul_bcast_safe<1>(xs[t], sc.gy[t >> 1]) : pk_mul_bcast_safe<0>(xs[t], sc.gy[t >> 1]);
          const float v = pair_reduce16(red, lane);
          if ((lane & 2) == 0)
            dbc[((kQT * s + (lane >> 3)) * 2 + 1) * kQN + 8 * h + 2 * p + ((lane >> 2) & 1)] = v;
        }
        __builtin_amdgcn_sched_barrier(0);
        // reverse sweep: lam_t = C_t gy_t + a_{t+1} lam_{t+1}
        {
          f32x2 lam, dap = dA2[p], ha;
          f32x2 red[kQT];
          f32x4 qn = bquad(kQT * s + kQT - 1, p);
#pragma unroll
          for (int t = kQT - 1; t >= 0; --t) {
            const f32x4 q = qn;
            if (t > 0) qn = bquad(kQT * s + t - 1, p);
            lam = (t & 1) ? pk_fma_bcast_safe<1>(q.hi, sc.gy[t >> 1], t == kQT - 1 ? hcar[p] : ha)
                          : pk_fma_bcast_safe<0>(q.hi, sc.gy[t >> 1], t == kQT - 1 ? hcar[p] : ha);
            if (hasZ) Y2[t] = pfma(q.hi, xs[t], Y2[t]);
            S2[t] = pfma(lam, q.lo, S2[t]);
            red[t] = (t & 1) ? pk_mul_bcast_safe<1>(lam, sc.dtu[t >> 1]) : pk_mul_bcast_safe<0>(lam, sc.dtu[t >> 1]);
            ha = pmul(lam, as[t]);
            const f32x2 hax = pmul(ha, t > 0 ? xs[t - 1] : xin);
            Q2[t] = pfma(hax, a2p, Q2[t]);
            dap = (t & 1) ? pk_fma_bcast_safe<1>(hax, sc.dt[t >> 1], dap) : pk_fma_bcast_safe<0>(hax, sc.dt[t >> 1], dap);
          }
          asm volatile("" : "+v"(ha), "+v"(dap));
#pragma unroll
          for (int t = 0; t < kQT; ++t) asm volatile("" : "+v"(S2[t]), "+v"(Q2[t]));
#pragma unroll
          for (int t = 0; t < kQT; ++t) asm volatile("" : "+v"(Y2[t]));
          hcar[p] = ha;   // a_t0 lam_t0: the carry into the previous sub-tile
          dA2[p] = dap;
          const float v = pair_reduce16(red, lane);
          if ((lane & 2) == 0)
            dbc[((kQT * s + (lane >> 3)) * 2 + 0) * kQN + 8 * h + 2 * p + ((lane >> 2) & 1)] = v;
        }
      }
      __builtin_amdgcn_sched_barrier(0);

      // ---- finish this lane's 4 positions [4h, 4h + 4) of the sub-tile
      float fS[4], fQ[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        fS[e] = pair_finish(S2[e], S2[4 + e], h);
        fQ[e] = pair_finish(Q2[e], Q2[4 + e], h) * kLn2;   // A2 carries log2(e)
      }
      float fY[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) fY[e] = pair_finish(Y2[e], Y2[4 + e], h);
      float o_du[4], o_dd[4], o_dz[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x2 uu = elem2<TI>(ru, i);
        const f32x2 rr = elem2<TI>(rd, i) + biasv;
        const f32x2 dt = sc.own_dt[i], gy = sc.own_gy[i];
        const f32x2 S = f32x2{fS[2 * i], fS[2 * i + 1]}, Q = f32x2{fQ[2 * i], fQ[2 * i + 1]};
        f32x2 sg = f32x2{1.f, 1.f};
        if (kSP) {   // softplus' = sigmoid (x > 20: torch's threshold, slope 1)
          const f32x2 ep = f32x2{fast_exp2(-rr.x * kLog2e), fast_exp2(-rr.y * kLog2e)} + 1.f;
          sg = f32x2{rr.x > 20.f ? 1.f : fast_rcp(ep.x), rr.y > 20.f ? 1.f : fast_rcp(ep.y)};
        }
        const f32x2 du = Dv * gy + dt * S;
        const f32x2 dd = (uu * S + Q) * sg;
        o_du[2 * i] = du.x; o_du[2 * i + 1] = du.y;
        o_dd[2 * i] = dd.x; o_dd[2 * i + 1] = dd.y;
        if (hasZ) {
          const f32x2 zz = elem2<TI>(rz, i), go = elem2<TI>(rg, i);
          const f32x2 ez = f32x2{fast_exp2(-zz.x * kLog2e), fast_exp2(-zz.y * kLog2e)} + 1.f;
          const f32x2 sz = f32x2{fast_rcp(ez.x), fast_rcp(ez.y)};
          const f32x2 gz = go * sz * (1.f + zz * (1.f - sz));
          const f32x2 dz = gz * (Dv * uu + f32x2{fY[2 * i], fY[2 * i + 1]});
          o_dz[2 * i] = dz.x; o_dz[2 * i + 1] = dz.y;
        }
        if (my_ok) {
          const f32x2 gu = gy * uu;
          dDacc += gu.x + gu.y;
          dbacc += dd.x + dd.y;
        }
      }
#ifdef MC_BWD_DEBUG
      if (g_dbg) {
        const int nch_ = (L_ + kS - 1) / kS;
        float* d = g_dbg + ((((int64_t)lin * kQW + wave) * nch_ + c) * kQSub + s) * 64 * kDbgVals + lane * kDbgVals;
#pragma unroll
        for (int p = 0; p < kQP; ++p) {
          d[2 * p] = hcar[p].x; d[2 * p + 1] = hcar[p].y;
          d[8 + 2 * p] = dA2[p].x; d[8 + 2 * p + 1] = dA2[p].y;
          d[16 + 2 * p] = A2[p].x; d[16 + 2 * p + 1] = A2[p].y;
        }
        d[24] = xi01.x; d[25] = xi01.y; d[26] = xi01.z; d[27] = xi01.w;
        d[28] = xi23.x; d[29] = xi23.y; d[30] = xi23.z; d[31] = xi23.w;
      }
#endif
      const uint32_t e0 = (uint32_t)(l0 + kQT * s + 4 * h);
      buf_st8(rs_du, ((ro_du + e0) * 2u) | st_mask, make_uint2(cvt_pk2<TI>(o_du[0], o_du[1]), cvt_pk2<TI>(o_du[2], o_du[3])));
      buf_st8(rs_dd, ((ro_dd + e0) * 2u) | st_mask, make_uint2(cvt_pk2<TI>(o_dd[0], o_dd[1]), cvt_pk2<TI>(o_dd[2], o_dd[3])));
      if (hasZ)
        buf_st8(rs_dz, ((ro_dz + e0) * 2u) | st_mask, make_uint2(cvt_pk2<TI>(o_dz[0], o_dz[1]), cvt_pk2<TI>(o_dz[2], o_dz[3])));
    }

    if (fine && c > 0) issue_fine(c - 1);   // the slots are free: this chunk's sub-tiles are done
    // ---- dB / dC of the chunk: sum over the workgroup's waves (fixed order) -> slab
    lds_barrier();
    {
      float* slab = a.slab_bc + (((int64_t)bg * a.nblk + wblk) * L_ + l0) * (2 * kQN);
      const float* src = dbc_base + buf * kQW * kDbcW;
      for (int f = tid; f < kDbcW / 4; f += 64 * kQW) {
        f32x4 acc = reinterpret_cast<const f32x4*>(src)[f];
#pragma unroll
        for (int w = 1; w < kQW; ++w) acc += reinterpret_cast<const f32x4*>(src + w * kDbcW)[f];
        if (4 * f < (L_ - l0) * 2 * kQN) reinterpret_cast<f32x4*>(slab)[f] = acc;
      }
    }
    buf ^= 1;   // the next barrier orders this chunk's reads before the buffer is written again
  }

  // ---- per-channel parameter gradients
  if (my_ok) {
#pragma unroll
    for (int p = 0; p < kQP; ++p) {
      const int n0 = 8 * h + 2 * p;
      a.slab_a[((int64_t)b * kQN + n0) * a.dim + my_dc] = dA2[p].x;
      a.slab_a[((int64_t)b * kQN + n0 + 1) * a.dim + my_dc] = dA2[p].y;
    }
  }
  const float dD2 = dDacc + qperm<kQpXor1>(dDacc), db2 = dbacc + qperm<kQpXor1>(dbacc);
  if (my_ok && h == 0) {
    a.slab_d[(int64_t)b * a.dim + my_dc] = dD2;
    a.slab_bias[(int64_t)b * a.dim + my_dc] = db2;
  }
}

// B / C quads, dB / dC partials (double-buffered), sub-tile states: 72 KB; + the projected-delta tiles
// (2 KB per wave): 80 KB, still two workgroups per CU
size_t bwd_pair_lds_bytes(bool proj) {
  return (size_t)kQW * kS * 2 * kQP * 16 + (size_t)2 * kQW * kS * 2 * kQN * 4 + (size_t)kQW * (kQSub - 1) * 2 * 64 * 16 +
         (proj ? (size_t)kQW * kQCh * kS * 2 : 0);
}
int bwd_pair_nblk(int H) { return (H + kQCh * kQW - 1) / (kQCh * kQW); }

// Eligibility (the host has validated shapes; strides in elements).
bool bwd_pair_ok(const mc_scan_bwd_params* p) {
  const int ib = p->itype == MC_DTYPE_F32 ? 4 : 2;
  const int wb = p->wtype == MC_DTYPE_F32 ? 4 : 2;
  if (ib != 2 || p->wtype != p->itype || p->dstate != kQN || p->seqlen % 8 || p->reverse_groups || p->u_groups)
    return false;
  auto rows = [&](const void* t, int64_t bs, int64_t ds) {
    return !t || (aligned16(t) && bs % 8 == 0 && ds % 8 == 0 &&
                  ((int64_t)(kQCh * kQW - 1) * (ds < 0 ? -ds : ds) + p->seqlen) * 2 < ((int64_t)1 << 31));
  };
  auto bc = [&](const void* t, int64_t bs, int64_t gs, int64_t ns) {
    const int64_t v = 16 / wb;
    return aligned16(t) && bs % v == 0 && gs % v == 0 && ns % v == 0 && ns >= 0 &&
           (15 * ns + p->seqlen) * wb < ((int64_t)1 << 31);
  };
  return rows(p->u, p->u_batch_stride, p->u_dim_stride) &&
         (p->delta_proj_w || rows(p->delta, p->delta_batch_stride, p->delta_dim_stride)) &&
         rows(p->z, p->z_batch_stride, p->z_dim_stride) && rows(p->dout, p->dout_batch_stride, p->dout_dim_stride) &&
         rows(p->du, p->du_batch_stride, p->du_dim_stride) &&
         rows(p->ddelta, p->ddelta_batch_stride, p->ddelta_dim_stride) &&
         rows(p->dz, p->dz_batch_stride, p->dz_dim_stride) &&
         bc(p->B, p->B_batch_stride, p->B_group_stride, p->B_dstate_stride) &&
         bc(p->C, p->C_batch_stride, p->C_group_stride, p->C_dstate_stride) &&
         (int64_t)kQCh * kQW * mc_scan_n_states(p->seqlen, p->state_interval) * kQN * 4 < ((int64_t)1 << 31);
}

template <typename TI, bool kPD>
static void launch_pair_pd(const BwdPairArgs& a, bool sp, bool zy, hipStream_t s) {
  const size_t lds = bwd_pair_lds_bytes(kPD);
  const dim3 grid(a.total_blocks), block(64 * kQW);
  if (a.state_ratio != 1) {
    if (sp && zy) hipLaunchKernelGGL((scan_bwd_pair_kernel<TI, true, true, kPD, true>), grid, block, lds, s, a);
    else if (sp) hipLaunchKernelGGL((scan_bwd_pair_kernel<TI, true, false, kPD, true>), grid, block, lds, s, a);
    else if (zy) hipLaunchKernelGGL((scan_bwd_pair_kernel<TI, false, true, kPD, true>), grid, block, lds, s, a);
    else hipLaunchKernelGGL((scan_bwd_pair_kernel<TI, false, false, kPD, true>), grid, block, lds, s, a);
    return;
  }
  if (sp && zy) hipLaunchKernelGGL((scan_bwd_pair_kernel<TI, true, true, kPD, false>), grid, block, lds, s, a);
  else if (sp) hipLaunchKernelGGL((scan_bwd_pair_kernel<TI, true, false, kPD, false>), grid, block, lds, s, a);
  else if (zy) hipLaunchKernelGGL((scan_bwd_pair_kernel<TI, false, true, kPD, false>), grid, block, lds, s, a);
  else hipLaunchKernelGGL((scan_bwd_pair_kernel<TI, false, false, kPD, false>), grid, block, lds, s, a);
}
template <typename TI>
static void launch_pair_t(const BwdPairArgs& a, bool sp, bool zy, hipStream_t s) {
  if (a.dpw) launch_pair_pd<TI, true>(a, sp, zy, s);
  else launch_pair_pd<TI, false>(a, sp, zy, s);
}

void launch_bwd_pair(const mc_scan_bwd_params* p, float* slab_bc, float* slab_a, float* slab_d, float* slab_bias,
                     int nblk, hipStream_t s) {
  BwdPairArgs a;
  a.batch = p->batch; a.dim = p->dim; a.seqlen = p->seqlen; a.n_groups = p->n_groups;
  a.n_states = mc_scan_n_states(p->seqlen, p->state_interval);
  a.state_ratio = p->state_interval == kFineS ? kS / kFineS : 1;
  a.nblk = nblk;
  a.total_blocks = p->batch * p->n_groups * nblk;
  a.u_bs = p->u_batch_stride; a.u_ds = p->u_dim_stride;
  a.dt_bs = p->delta_batch_stride; a.dt_ds = p->delta_dim_stride;
  a.z_bs = p->z_batch_stride; a.z_ds = p->z_dim_stride;
  a.go_bs = p->dout_batch_stride; a.go_ds = p->dout_dim_stride;
  a.du_bs = p->du_batch_stride; a.du_ds = p->du_dim_stride;
  a.ddt_bs = p->ddelta_batch_stride; a.ddt_ds = p->ddelta_dim_stride;
  a.dz_bs = p->dz_batch_stride; a.dz_ds = p->dz_dim_stride;
  a.B_bs = p->B_batch_stride; a.B_gs = p->B_group_stride; a.B_ns = p->B_dstate_stride;
  a.C_bs = p->C_batch_stride; a.C_gs = p->C_group_stride; a.C_ns = p->C_dstate_stride;
  a.u = p->u; a.delta = p->delta; a.z = p->z; a.dout = p->dout; a.B = p->B; a.C = p->C;
  a.A = p->A; a.D = p->D; a.delta_bias = p->delta_bias; a.chunk_states = p->chunk_states;
  a.du = p->du; a.ddelta = p->ddelta; a.dz = p->dz;
  a.slab_bc = slab_bc; a.slab_a = slab_a; a.slab_d = slab_d; a.slab_bias = slab_bias;
  a.dpx = p->delta_proj_x; a.dpw = p->delta_proj_w; a.rank = p->delta_rank;
  a.dpx_bs = p->dpx_batch_stride; a.dpx_ts = p->dpx_token_stride; a.dpw_ds = p->dpw_dim_stride;
  const bool sp = p->delta_softplus != 0, zy = p->z != nullptr;
  if (p->itype == MC_DTYPE_BF16) launch_pair_t<bf16_t>(a, sp, zy, s);
  else launch_pair_t<f16_t>(a, sp, zy, s);
}

}  // namespace scan
}  // namespace mc

#ifdef MC_BWD_DEBUG
extern "C" int mc_debug_alloc(size_t bytes) {
  static float* buf = nullptr;
  static size_t have = 0;
  if (bytes > have) {
    if (buf) (void)hipFree(buf);
    if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
    have = bytes;
  }
  (void)hipMemset(buf, 0, bytes);
  float* p = bytes ? buf : nullptr;
  return hipMemcpyToSymbol(HIP_SYMBOL(mc::scan::g_dbg), &p, sizeof(p)) == hipSuccess ? 0 : 2;
}
extern "C" int mc_debug_copy(void* dst, size_t bytes, void* stream) {
  float* p = nullptr;
  if (hipMemcpyFromSymbol(&p, HIP_SYMBOL(mc::scan::g_dbg), sizeof(p)) != hipSuccess || !p) return 1;
  return hipMemcpyAsync(dst, p, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream) == hipSuccess ? 0 : 2;
}
#endif
