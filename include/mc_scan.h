/*
 * mc_scan.h -- C ABI of the MI355X selective-scan kernels (libmamba_clip_amd.so).
 *
 * Replaces the native boundary the reference reaches through
 *   mamba_ssm.ops.selective_scan_interface.selective_scan_fn
 *     -> SelectiveScanFn.forward/backward -> selective_scan_cuda.fwd/bwd
 * (third-party, not vendored; imported at /root/reference/src/mamba_clip/model.py:27-28,
 *  called at model.py:539-550; reference semantics embedded at model.py:83-169).
 *
 *   mc_scan_fwd  <- selective_scan_cuda.fwd(u, delta, A, B, C, D, z, delta_bias, softplus)
 *   mc_scan_bwd  <- selective_scan_cuda.bwd(u, delta, A, B, C, D, z, delta_bias, dout,
 *                                           x_chunks, out, dz, softplus, recompute_out_z)
 *
 * Contract
 *   - Plain pointers and sizes only.  Every device buffer (inputs, outputs,
 *     chunk states, workspace) is allocated by the caller; the library never
 *     allocates, frees or synchronises.
 *   - Launches are asynchronous on the given stream (hipStream_t passed as void*).
 *   - Returns MC_OK (0) or a negative code; mc_last_error() gives a
 *     thread-local message (the Python layer raises RuntimeError with it, as
 *     the upstream TORCH_CHECKs do).
 *   - Re-entrant; no global mutable state.
 *   - Layout: u/delta/z/out/dout/du/ddelta/dz are (batch, dim, seqlen) with unit
 *     stride along seqlen; B/C (and dB/dC) are (batch, n_groups, dstate, seqlen)
 *     with unit stride along seqlen; A (dim, dstate) fp32; D, delta_bias
 *     (dim,) fp32.  Channel d reads group d / (dim / n_groups).
 */
#ifndef MAMBA_CLIP_AMD_MC_SCAN_H
#define MAMBA_CLIP_AMD_MC_SCAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum mc_dtype {
  MC_DTYPE_F32 = 0,
  MC_DTYPE_BF16 = 1,
  MC_DTYPE_F16 = 2,
  MC_DTYPE_FP8_E4M3 = 3, /* OCP e4m3fn (gfx950 native fp8); contrastive GEMM operands only */
  MC_DTYPE_U8 = 4         /* raw decoded image bytes; mc_patch_embed_input only */
} mc_dtype;

enum {
  MC_OK = 0,
  MC_ERR_INVALID = -1,   /* null pointer / bad argument */
  MC_ERR_DTYPE = -2,     /* unsupported dtype combination */
  MC_ERR_SHAPE = -3,     /* bad shape (dim % n_groups, dstate > MC_SCAN_MAX_DSTATE, ...) */
  MC_ERR_LAUNCH = -4,    /* kernel launch failed */
  MC_ERR_WORKSPACE = -5  /* workspace too small */
};

/* States are held in VGPRs, one channel per lane: dstate <= 32 (padded to 8/16/32).
 * Upstream mamba_ssm accepts up to 256; every reference call site and BASELINE
 * config uses 16 (model.py:357, 539-550).  Larger dstate returns MC_ERR_SHAPE. */
#define MC_SCAN_MAX_DSTATE 32
/* sequence positions per saved chunk state: the training forward writes the
 * fp32 state after every MC_SCAN_CHUNK positions (and after the last position);
 * the backward walks chunks of this length in reverse, recomputing the states
 * inside a chunk from the one saved at its start.  32 positions = 2 B per
 * (channel, position) at dstate 16, a quarter of the bf16 activations. */
#define MC_SCAN_CHUNK 32
/* the fine saved-state interval (mc_scan_fwd_params.state_interval) */
#define MC_SCAN_STATE_INTERVAL_FINE 8

typedef struct mc_scan_fwd_params {
  int32_t batch, dim, seqlen, dstate, n_groups;
  int32_t itype;            /* mc_dtype of u, delta, z, out */
  int32_t wtype;            /* mc_dtype of B, C */
  int32_t delta_softplus;   /* apply softplus(delta + delta_bias) */
  /* element strides (seqlen stride is 1 everywhere) */
  int64_t u_batch_stride, u_dim_stride;
  int64_t delta_batch_stride, delta_dim_stride;
  int64_t z_batch_stride, z_dim_stride;
  int64_t out_batch_stride, out_dim_stride;
  int64_t B_batch_stride, B_group_stride, B_dstate_stride;
  int64_t C_batch_stride, C_group_stride, C_dstate_stride;
  const void* u;
  const void* delta;
  const float* A;           /* (dim, dstate) contiguous */
  const void* B;
  const void* C;
  const float* D;           /* nullable, (dim,) */
  const void* z;            /* nullable: out = (y + D u) * silu(z) */
  const float* delta_bias;  /* nullable, (dim,) */
  void* out;
  float* chunk_states;      /* nullable: (batch, dim, n_chunks, dstate) fp32, state at END of each chunk
                               (the last entry: the state after position seqlen-1) */
  float* last_state;        /* nullable: (batch, dim, dstate) fp32 */
  void* workspace;          /* >= mc_scan_fwd_workspace_bytes(...) bytes, 16-B aligned */
  size_t workspace_bytes;
  /* nullable; used only when z is given: the pre-gate output y + D u (itype,
   * seqlen stride 1) -- the `out` upstream's forward returns next to out_z.
   * Not needed for training: mc_scan_bwd recomputes y for dz. */
  void* out_y;
  int64_t out_y_batch_stride, out_y_dim_stride;
  /* Grouped directions (SS2D's cross-scan, reference model.py:510-517, merged
   * at 553-565), both 0 = off:
   * reverse_groups  bitmask: group g scans its sequence backwards -- step l
   *                 reads and writes every per-position tensor (u, delta, B, C,
   *                 out) at position seqlen-1-l -- so a flipped direction needs
   *                 no flipped copy of its inputs or outputs;
   * u_groups        k > 0: u holds k blocks of dim/n_groups channel rows and
   *                 group g reads block g % k (SS2D: 4 directions share the 2
   *                 blocks [x, x^T]); 0 = u has dim rows as usual.
   * Either set: z must be NULL (the cross-scan has no gate). */
  int32_t reverse_groups, u_groups;
  /* Projected delta -- the Mamba mixer's dt_proj fused into the scan (reference
   * model.py:519-528 / 630-647; upstream's mamba_inner_fn analogue).  When
   * delta_proj_w is non-NULL, `delta` is not read; instead
   *     delta[b, d, l] = sum_r delta_proj_w[d * dpw_dim_stride + r]
   *                          * delta_proj_x[b * dpx_batch_stride + l * dpx_token_stride + r]
   * is formed per chunk on the matrix cores, rounded to itype (what a dt_proj
   * GEMM would store), so the (batch, dim, seqlen) delta stream never leaves
   * the chip.  Both operands are itype; delta_proj_x is token-major.
   * delta_rank % 16 == 0, 16..256; 8-B aligned operands, strides % 4 == 0.
   * Pair-kernel shapes only (16-bit rows, dstate 16, seqlen % 8 == 0, 16-B
   * aligned rows, no grouped directions), else MC_ERR_SHAPE.
   * delta_out (nullable): the formed delta, written with delta_batch_stride /
   * delta_dim_stride -- the input mc_scan_bwd needs for training. */
  const void* delta_proj_x;
  const void* delta_proj_w;
  int32_t delta_rank;
  int64_t dpx_batch_stride, dpx_token_stride, dpw_dim_stride;
  void* delta_out;
  /* Saved-state interval of a training call: chunk_states holds the state after
   * every state_interval positions (and after the last position), i.e.
   * mc_scan_n_states(seqlen, state_interval) entries per channel.  0 or
   * MC_SCAN_CHUNK (32): the default.  MC_SCAN_STATE_INTERVAL_FINE (8): the
   * backward reads the state entering each of its 8-position sub-tiles instead
   * of recomputing it (C2: scan backward -10 %) at 4x the state memory; pair-
   * kernel shapes only -- mc_scan_fwd_state_interval() resolves a request.
   * Layout: the default interval keeps (batch, dim, n_states, dstate); the fine
   * one is position-major, (batch, n_states, dim, dstate). */
  int32_t state_interval;
} mc_scan_fwd_params;

typedef struct mc_scan_bwd_params {
  int32_t batch, dim, seqlen, dstate, n_groups;
  int32_t itype, wtype, delta_softplus;
  /* inputs, same layout rules as forward (seqlen stride 1) */
  int64_t u_batch_stride, u_dim_stride;
  int64_t delta_batch_stride, delta_dim_stride;
  int64_t z_batch_stride, z_dim_stride;
  int64_t dout_batch_stride, dout_dim_stride;
  /* output strides of du / ddelta / dz (seqlen stride 1): a caller keeping
   * activations channel-major passes the strides of u / delta / z */
  int64_t du_batch_stride, du_dim_stride;
  int64_t ddelta_batch_stride, ddelta_dim_stride;
  int64_t dz_batch_stride, dz_dim_stride;
  int64_t B_batch_stride, B_group_stride, B_dstate_stride;
  int64_t C_batch_stride, C_group_stride, C_dstate_stride;
  const void* u;
  const void* delta;
  const float* A;
  const void* B;
  const void* C;
  const float* D;             /* nullable */
  const void* z;              /* nullable */
  const float* delta_bias;    /* nullable */
  const void* dout;           /* gradient of out (itype) */
  const float* chunk_states;  /* REQUIRED: produced by mc_scan_fwd on the same inputs */
  /* outputs: du/ddelta/dz (batch, dim, seqlen) in itype with the strides above; dB/dC
   * contiguous (batch, n_groups, dstate, seqlen) in wtype; dA (dim, dstate),
   * dD (dim,), ddelta_bias (dim,) fp32.  dz / dD / ddelta_bias nullable when
   * the corresponding input is absent. */
  void* du;
  void* ddelta;
  void* dz;
  void* dB;
  void* dC;
  float* dA;
  float* dD;
  float* ddelta_bias;
  void* workspace;            /* >= mc_scan_bwd_workspace_bytes(...) bytes, 256-B aligned */
  size_t workspace_bytes;
  /* ignored (kept for layout stability): the backward recomputes the pre-gate
   * output y + D u that dz = dout * y * silu'(z) needs from the chunk states */
  const void* out_y;
  int64_t out_y_batch_stride, out_y_dim_stride;
  /* reverse_groups / u_groups as in mc_scan_fwd_params (same values as the
   * forward).  dout, du, ddelta, dB, dC follow the same mirrored positions; with
   * u_groups > 0, du still has dim rows (one per group and channel): the caller
   * sums the groups that share a u block. */
  int32_t reverse_groups, u_groups;
  /* Projected delta (see mc_scan_fwd_params): when delta_proj_w is non-NULL,
   * `delta` is not read; the kernel re-forms it per chunk from the same
   * operands, bit-identical to the forward's.  Same requirements. */
  const void* delta_proj_x;
  const void* delta_proj_w;
  int32_t delta_rank;
  int64_t dpx_batch_stride, dpx_token_stride, dpw_dim_stride;
  /* the interval the forward saved chunk_states with (0 = MC_SCAN_CHUNK) */
  int32_t state_interval;
  /* Output strides of dB / dC (elements; seqlen stride 1).  All three 0: contiguous
   * (batch, n_groups, dstate, seqlen).  A caller whose B / C are row blocks of one
   * channel-major projection output (the Mamba mixer's x_proj rows) passes that
   * block's strides, and the gradients land in the projection's gradient buffer. */
  int64_t dB_batch_stride, dB_group_stride, dB_dstate_stride;
  int64_t dC_batch_stride, dC_group_stride, dC_dstate_stride;
} mc_scan_bwd_params;

/* number of MC_SCAN_CHUNK-long chunks covering seqlen */
int32_t mc_scan_n_chunks(int32_t seqlen);

/* bytes of fp32 chunk states the forward writes for a training call (default interval) */
size_t mc_scan_chunk_states_bytes(int32_t batch, int32_t dim, int32_t seqlen, int32_t dstate);

/* saved states per channel at a given interval (0 = MC_SCAN_CHUNK): ceil(seqlen / interval) */
int32_t mc_scan_n_states(int32_t seqlen, int32_t state_interval);

/* the interval mc_scan_fwd will save states with for these params: p->state_interval when
 * the call can honour it (MC_SCAN_STATE_INTERVAL_FINE needs the pair kernel's shapes),
 * else MC_SCAN_CHUNK.  Size chunk_states with mc_scan_n_states(seqlen, result) and pass
 * the result to both mc_scan_fwd and mc_scan_bwd. */
int32_t mc_scan_fwd_state_interval(const mc_scan_fwd_params* p);

/* workspace the forward needs (B/C re-laid out as fp32 [batch][group][seqlen][2*dstate']) */
size_t mc_scan_fwd_workspace_bytes(int32_t batch, int32_t seqlen, int32_t dstate, int32_t n_groups);

/* workspace the backward needs (partial-sum slabs; deterministic reductions) */
size_t mc_scan_bwd_workspace_bytes(int32_t batch, int32_t dim, int32_t seqlen, int32_t dstate,
                                   int32_t n_groups);

/* Which kernel family mc_scan_fwd / mc_scan_bwd run for these params (no launch; for tests and
 * tooling): the lane-pair kernels (16-bit rows, dstate 16, seqlen % 8 == 0, 16-B aligned rows:
 * scan_fwd_pair.hip / scan_bwd_pair.hip), the general chunked kernels, or the grouped-direction
 * (SS2D) path.  NONE for an empty call. */
#define MC_SCAN_KERNEL_NONE 0
#define MC_SCAN_KERNEL_PAIR 1
#define MC_SCAN_KERNEL_GENERIC 2
#define MC_SCAN_KERNEL_DIRS 3
int32_t mc_scan_fwd_kernel(const mc_scan_fwd_params* p);
int32_t mc_scan_bwd_kernel(const mc_scan_bwd_params* p);

int mc_scan_fwd(const mc_scan_fwd_params* p, void* stream);
int mc_scan_bwd(const mc_scan_bwd_params* p, void* stream);

/* thread-local text of the last error returned on this thread */
const char* mc_last_error(void);
/* library version string */
const char* mc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MAMBA_CLIP_AMD_MC_SCAN_H */
