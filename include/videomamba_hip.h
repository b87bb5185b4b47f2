/*
 * videomamba_hip.h — C ABI of libvideomamba_hip.so (gfx950 / MI355X).
 *
 * The drop-in boundary for the VideoMamba encoder hot path.  Each entry point
 * replaces one third-party kernel call of the reference (tannerhoalst/VideoMamba),
 * cited as `file:line` under /root/reference:
 *
 *   vm_selective_scan_fwd      <- mamba_ssm selective_scan_fn
 *                                 (models/videomamba/mamba_simple.py:122-152, stateless and
 *                                  initial_state forms; also replaces the per-token
 *                                  selective_state_update loop at :153-172)
 *   vm_selective_scan_dtproj_fwd <- dt_proj (mamba_simple.py:409-413) + selective_scan_fn,
 *                                 dt computed inside the scan on the matrix cores
 *   vm_selective_scan_bidir_fwd <- the forward + flipped backward scans of
 *                                 BiMambaRefinerBlock (models/refiner_backbone.py:98-135)
 *   vm_selective_state_update  <- mamba_ssm selective_state_update  (mamba_simple.py:483-494)
 *   vm_causal_conv1d_fwd       <- causal_conv1d_fn (+ conv_state prepend)
 *                                 (mamba_simple.py:381-404)
 *   vm_causal_conv1d_update    <- causal_conv1d_update  (mamba_simple.py:468-474)
 *   vm_conv_proj_fwd           <- causal_conv1d_fn + x_proj + dt_proj, fused, token-major
 *                                 (mamba_simple.py:381-416)
 *   vm_in_proj_conv_proj_fwd   <- in_proj + causal_conv1d_fn + x_proj + dt_proj at small
 *                                 batches, the conv and x_proj in in_proj's epilogue
 *                                 (mamba_simple.py:333-339, :381-416)
 *   vm_conv_proj_cm_fwd        <- the same three steps on the channel-major small-batch
 *                                 layout (mamba_simple.py:381-416)
 *   vm_add_norm_fwd            <- mamba_ssm rms_norm_fn / layer_norm_fn
 *                                 (models/videomamba/videomamba.py:152-166, :904-918)
 *   vm_norm_pool_fwd           <- final add + norm (videomamba.py:896-918) with the
 *                                 per-frame / whole-clip column sums of the pooling
 *   vm_pool_finish_fwd         <- the pooling tail: means, CLS add / concat and pool_norm
 *                                 LayerNorm (videomamba.py:983-1062, :702-751 masked)
 *   vm_linear_fwd              <- the mixer's in_proj / out_proj nn.Linear at every batch
 *                                 (mamba_simple.py:333-339, :445-446); vm_linear_fwd_form
 *                                 names the kernel form (tests, benches)
 *   vm_linear_add_norm_fwd     <- out_proj + the next Block's fused add + RMSNorm
 *                                 (mamba_simple.py:445-446, videomamba.py:141-166)
 *   vm_patch_embed_fwd         <- PatchEmbed Conv3d + pos/temporal embedding add
 *                                 (videomamba.py:359-368, :806-815)
 *
 * Conventions (all entry points):
 *   - Plain device pointers, element counts and element strides; no torch types.
 *   - The caller owns every buffer; the library never allocates device memory.
 *   - Sequence ("l") strides are 1; every other stride is passed explicitly.
 *   - dtype codes: VM_DTYPE_F32 / VM_DTYPE_BF16.  Small parameters (A, D, biases,
 *     norm / conv weights) are fp32.
 *   - Work is enqueued on `stream` (a hipStream_t); nothing synchronises, so calls are
 *     safe to capture into a hipGraph.
 *   - Return 0 on success, a negative VM_E* code otherwise; vm_last_error() gives the
 *     message.  Nothing is thrown across the ABI.
 *   - Outputs are deterministic (bitwise repeatable).  The only atomics are the one-launch
 *     segmented scan's block hand-off granules and launch counter (agent-scope, in the
 *     caller's sync buffer; see vm_selective_scan_sync_bytes) — they carry and order values,
 *     never accumulate them.
 */
#ifndef VIDEOMAMBA_HIP_H
#define VIDEOMAMBA_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define VM_ABI_VERSION 14

#define VM_DTYPE_F32 0
#define VM_DTYPE_BF16 1

#define VM_OK 0
#define VM_E_INVALID -1  /* bad argument (shape, dtype, null pointer) */
#define VM_E_LAUNCH -2   /* HIP launch / runtime error */

typedef void* vm_stream_t; /* hipStream_t */

int vm_abi_version(void);
const char* vm_last_error(void);

/*
 * Selective scan, fp32 state (mamba_simple.py:30-106 semantics):
 *   delta' = softplus?(delta + delta_bias)
 *   h_t    = exp(delta'_t * A) * h_{t-1} + delta'_t * u_t * B_t      (h_{-1} = h0 or 0)
 *   y_t    = <h_t, C_t> + D * u_t;   out = y * silu(z)   (z, D optional)
 * u, delta, z, out: (batch, dim, seqlen) with element strides (*_sb, *_sd, *_sl).
 * B, C: (batch, dstate, seqlen) with strides (*_sb, *_sn, *_sl).  All in `dtype`.
 * Two layouts are accepted:
 *   token-major   — unit channel stride (u/delta/z/out *_sd == 1; B/C any strides):
 *                   channel-per-lane sequential kernels (vm_scan_seq.hip);
 *   channel-major — unit step stride for every operand (*_sl == 1): time-parallel
 *                   kernels (vm_scan.hip).
 * A: (dim, dstate) fp32 contiguous.  D, delta_bias: (dim) fp32, nullable.
 * h0 (nullable) / h_last (nullable): (batch, dim, dstate) with strides (sb, sd, 1) in
 * their own dtype; h_last may alias h0 (in-place state update).  dstate <= 16.
 * Steps [seqlen, out_len) of every out row are written as 0 (padded token layouts).
 * segments: token-major only — 0 lets the cost model choose how many time segments the
 * sequence is cut into (small batches run summary / carry / final passes), > 0 forces that
 * count (tests and sweeps).  There is no other configuration channel (no environment).
 * workspace: scratch for the time-segmented token-major form, at least
 * vm_selective_scan_workspace_bytes(..., segments) bytes; with less (or NULL) a
 * single-pass kernel runs instead — same result, less parallelism.
 */
int vm_selective_scan_fwd(const void* u, long long u_sb, long long u_sd, long long u_sl,
                          const void* delta, long long dl_sb, long long dl_sd, long long dl_sl,
                          const float* A,
                          const void* B, long long b_sb, long long b_sn, long long b_sl,
                          const void* C, long long c_sb, long long c_sn, long long c_sl,
                          const float* D, const void* z, long long z_sb, long long z_sd,
                          long long z_sl, const float* delta_bias, int delta_softplus,
                          const void* h0, int h0_dtype, long long h0_sb, long long h0_sd,
                          void* h_last, int hl_dtype, long long hl_sb, long long hl_sd,
                          void* out, long long o_sb, long long o_sd, long long o_sl,
                          int out_len, int batch, int dim, int seqlen, int dstate, int dtype,
                          int segments, void* workspace, long long workspace_bytes,
                          void* sync, long long sync_bytes, vm_stream_t stream);

/*
 * Both directions of a bidirectional block in one scan (BiMambaRefinerBlock,
 * models/refiner_backbone.py:98-135, whose backward block scans torch.flip of the
 * sequence).  Arguments as vm_selective_scan_fwd over batch = 2*split rows on token-major
 * operands: rows [0, split) scan forward with (A, D, delta_bias, h0, h_last); rows
 * [split, 2*split) hold the backward direction's operands already in flipped step order
 * and use (A_bwd, D_bwd, delta_bias_bwd, h0_bwd, h_last_bwd) (state row b - split, same
 * dtypes / strides), and their step t output is stored at the un-flipped row
 * t + (L - F) - 2F*floor(t/F), F = frame_len (1 = plain time reversal; the frame size
 * reverses frame order and keeps token order within a frame).  Needs dstate == 16 with
 * unit state stride and, when the cost model segments the sequence, the
 * vm_selective_scan_workspace_bytes(batch, ...) workspace.
 */
int vm_selective_scan_bidir_fwd(
    const void* u, long long u_sb, long long u_sd, long long u_sl,
    const void* delta, long long dl_sb, long long dl_sd, long long dl_sl,
    const float* A,
    const void* B, long long b_sb, long long b_sn, long long b_sl,
    const void* C, long long c_sb, long long c_sn, long long c_sl,
    const float* D, const void* z, long long z_sb, long long z_sd, long long z_sl,
    const float* delta_bias, int delta_softplus,
    const void* h0, int h0_dtype, long long h0_sb, long long h0_sd,
    void* h_last, int hl_dtype, long long hl_sb, long long hl_sd,
    void* out, long long o_sb, long long o_sd, long long o_sl, int out_len,
    int batch, int dim, int seqlen, int dstate, int dtype,
    int split, const float* A_bwd, const float* D_bwd, const float* delta_bias_bwd,
    const void* h0_bwd, void* h_last_bwd, int frame_len,
    int segments, void* workspace, long long workspace_bytes, void* sync,
    long long sync_bytes, vm_stream_t stream);

/*
 * dt_proj folded into the scan (ABI v8): the mixer's  dt = dt_proj.weight @ x_dbl[:, :R]^T
 * (models/videomamba/mamba_simple.py:409-413, rounded to bf16 there) followed by
 * selective_scan_fn(u, dt, A, B, C, D, z, delta_bias, delta_softplus=True)
 * (:423-435), with dt never written to memory: each 16-step block's dt is computed on the
 * matrix cores from the x_dbl rows the scan already reads for B|C.
 *   dt_low: rows of the x_dbl buffer (batch stride dtl_sb, row stride dtl_sl elements;
 *           dt_low = the first dt_rank columns), 8-byte aligned rows;
 *   w_dt:   (dim, w_dt_ld) bf16 with columns >= dt_rank zero, w_dt_ld >= 16*ceil(r/16);
 * everything else as vm_selective_scan_fwd.  bf16, token-major, 16 states with C directly
 * after B in the x_dbl row (the mixer's layout), z present, delta_softplus = 1, dt_rank a
 * multiple of 4 (ABI v10: x_dbl columns >= dt_rank are never read as dt_low).
 *   Single pass (the cost model picks one segment: chip-filling batches): dim % 128 == 0,
 *   dt_rank <= 64; each 16-step block's dt by v_mfma_f32_16x16x16_bf16 over
 *   ceil(dt_rank / 16) k-steps.
 *   Segmented (ABI v11; segments, workspace and sync as vm_selective_scan_fwd): segments of
 *   at most 64 steps (vm_selective_scan_chunk_steps), w_dt_ld = 32 or 64 (the r_pad of
 *   vm_conv_proj_fwd's W_dt); each wave computes its segment's dt exactly as
 *   vm_conv_proj_fwd's dt_proj does (v_mfma_f32_16x16x32_bf16 over w_dt_ld / 32 k-steps,
 *   x_dbl columns >= dt_rank as 0), so it equals the dt rows that call would write, bit for
 *   bit — the streaming batches' replacement for conv_proj's dt rows
 *   (mamba_simple.py:409-416).
 * Each token's dt is computed from its own row in a fixed order (sequence-length
 * independent).
 */
int vm_selective_scan_dtproj_fwd(
    const void* u, long long u_sb, long long u_sd, long long u_sl,
    const void* dt_low, long long dtl_sb, long long dtl_sl, int dt_rank,
    const void* w_dt, int w_dt_ld, const float* A,
    const void* B, long long b_sb, long long b_sn, long long b_sl,
    const void* C, long long c_sb, long long c_sn, long long c_sl,
    const float* D, const void* z, long long z_sb, long long z_sd, long long z_sl,
    const float* delta_bias, int delta_softplus,
    const void* h0, int h0_dtype, long long h0_sb, long long h0_sd,
    void* h_last, int hl_dtype, long long hl_sb, long long hl_sd,
    void* out, long long o_sb, long long o_sd, long long o_sl, int out_len,
    int batch, int dim, int seqlen, int dstate, int dtype,
    int segments, void* workspace, long long workspace_bytes, void* sync,
    long long sync_bytes, vm_stream_t stream);

/* Steps per segment the token-major scan would run for this shape and segment request
 * (0 = the single pass), ABI v11: vm_selective_scan_dtproj_fwd's segmented form takes
 * segments of at most 64 steps. */
int vm_selective_scan_chunk_steps(int batch, int dim, int seqlen, int dstate, int segments);

/* Scratch bytes vm_selective_scan_fwd wants for token-major operands of this shape and
 * segment request (0 = the cost model's choice). */
long long vm_selective_scan_workspace_bytes(int batch, int dim, int seqlen, int dstate,
                                            int segments);

/* Sync-buffer bytes for the one-launch segmented form (0 when the single pass runs).
 * `sync` (ABI v7, both scan entry points; NULL = the two-launch segmented form) must be
 * zero-filled before its first use and then left alone: every launch leaves it valid for the
 * next (ABI v9: word 1 is an epoch each launch advances, and blocks hand their aggregates on
 * as {tag = epoch, value} granules, so stale granules of any earlier launch — of any shape —
 * never match; tags wrap after 2^32 - 1 launches on one buffer).  One sync buffer must not
 * serve two launches that can run at the same time (e.g. on two streams).
 * The one-launch form runs when the buffer is large enough and the segmented grid fits one
 * workgroup per CU of the stream's device (blocks then wait on earlier, resident blocks'
 * published aggregates); results are identical to the two-launch form.
 * ABI v8: word 0 of the buffer is a sticky error word.  Each wait is bounded (it never
 * hangs the GPU); a block whose wait runs out sets word 0 and writes NaN for every output
 * and last state it owns.  The library never clears word 0: read it with
 * vm_selective_scan_sync_status on a host copy, and zero it to re-arm. */
long long vm_selective_scan_sync_bytes(int batch, int dim, int seqlen, int dstate,
                                       int segments);

/* Host-side check of a sync buffer: `sync_host` is a HOST copy of at least the first 16
 * bytes of the device buffer.  Returns 0 (no hand-off ever timed out), 1 (some launch timed
 * out: its outputs are NaN), or VM_E_INVALID.  Pure host code (no HIP call). */
int vm_selective_scan_sync_status(const void* sync_host, long long bytes);

/*
 * One-token scan step on `state` (updated in place, own dtype; fp32 math).
 * x, dt, z, out: (batch, dim) strides (*_sb, 1); B, C: (batch, dstate) strides (*_sb, 1).
 * state: (batch, dim, dstate) strides (s_sb, s_sd, 1).
 */
int vm_selective_state_update(void* state, int state_dtype, long long s_sb, long long s_sd,
                              const void* x, long long x_sb, const void* dt, long long dt_sb,
                              const float* A, const void* B, long long b_sb,
                              const void* C, long long c_sb, const float* D,
                              const void* z, long long z_sb, const float* dt_bias,
                              int dt_softplus, void* out, long long o_sb,
                              int batch, int dim, int dstate, int dtype, vm_stream_t stream);

/*
 * Depthwise causal conv1d (+bias, optional SiLU) over the virtual sequence
 * [conv_state_in (width values) | x], keeping the last `seqlen` outputs.
 * x, out: (batch, dim, seqlen) with element strides (*_sb, *_sd, *_sl): either unit step
 * stride (channel-major rows) or unit channel stride (token-major rows).  Steps
 * [seqlen, out_len) of out are written as 0.  weight: (dim, width) fp32; bias: (dim) fp32
 * nullable.  conv_state_in / conv_state_out: (batch, dim, width) strides (sb, sd, 1), own
 * dtype, nullable; out state = last `width` raw inputs.  conv_state_out must not alias
 * conv_state_in.  width <= 8.
 */
int vm_causal_conv1d_fwd(const void* x, long long x_sb, long long x_sd, long long x_sl,
                         const float* weight, const float* bias,
                         const void* cs_in, int cs_in_dtype, long long csi_sb, long long csi_sd,
                         void* cs_out, int cs_out_dtype, long long cso_sb, long long cso_sd,
                         void* out, long long o_sb, long long o_sd, long long o_sl, int out_len,
                         int batch, int dim, int seqlen, int width, int silu, int dtype,
                         vm_stream_t stream);

/*
 * Fused token-major mixer middle (bf16): per token row of the flattened (batch, out_len)
 * axis,  u = silu(conv1d([conv_state_in | x]))  ->  x_dbl = u @ W_x^T  ->
 * dt = x_dbl[:, :r] @ W_dt^T, rounded to bf16 at each of the three (the reference's
 * rounding points).  x: the first `dim` columns of xz rows (strides xz_sb, xz_sl; unit
 * channel stride).  u, dt: (rows, dim), x_dbl: (rows, e), all batch-contiguous
 * (sb == out_len * sl).  wx_pad: (e_pad, dim) with rows >= e zero (e_pad % 16 == 0,
 * e_pad <= 128); wdt_pad: (dim, r_pad) with columns >= r zero (r_pad 32 or 64).  Rows
 * with step >= seqlen are written as 0.  conv state as vm_causal_conv1d_fwd (width <= 4).
 * dim % 64 == 0, seqlen >= 1.
 * dt == NULL skips dt_proj (conv + x_proj only; wdt_pad may then be NULL too).
 * batch <= 8 runs a split-K form (fixed 128-channel splits of the x_proj reduction, so
 * every token's bits are independent of the sequence length) that needs `workspace` of
 * vm_conv_proj_workspace_bytes() bytes; larger batches need none (NULL, 0), and address
 * x rows, u rows and the conv state through 31-bit buffer offsets: VM_E_INVALID when the xz
 * rows of the sequences one 64-row tile touches span 2 GiB (about 230k tokens at dim 1152)
 * or the conv state does.
 * dt_softplus != 0: `dt` receives the scan's activated step instead,
 *   delta = softplus(float(bf16(dt)) + dt_bias[d])  (dt_bias nullable = 0), rounded to bf16
 *   — selective_scan_fn's delta_bias / delta_softplus prologue (mamba_simple.py:30-106),
 *   moved into the producer; pass delta_softplus = 0 and no delta_bias to the scan then.
 */
int vm_conv_proj_fwd(const void* xz, long long xz_sb, long long xz_sl,
                     const float* conv_weight, const float* conv_bias,
                     const void* cs_in, int cs_in_dtype, long long csi_sb, long long csi_sd,
                     void* cs_out, int cs_out_dtype, long long cso_sb, long long cso_sd,
                     const void* wx_pad, int e, int e_pad, const void* wdt_pad, int r, int r_pad,
                     void* u, long long u_sb, long long u_sl,
                     void* xdbl, long long xd_sb, long long xd_sl,
                     void* dt, long long dt_sb, long long dt_sl,
                     const float* dt_bias, int dt_softplus,
                     int out_len, int batch, int dim, int seqlen, int width, int dtype,
                     void* workspace, long long workspace_bytes, vm_stream_t stream);

/* Scratch bytes vm_conv_proj_fwd needs for this shape (0 above the split-K batch). */
long long vm_conv_proj_workspace_bytes(int batch, int out_len, int dim, int e);

/* ABI v10: 1 when vm_conv_proj_fwd accepts this shape's buffer extents (the small-batch forms
 * always do; the wide form needs its 31-bit buffer offsets to cover the operands, see above),
 * 0 when it would return VM_E_INVALID for them — a caller then takes the unfused conv +
 * projection path instead.  Pure host code. */
int vm_conv_proj_fits(int batch, int out_len, int seqlen, int dim, int e, int r_pad,
                      int dt_softplus, long long xz_sb, long long xz_sl, int has_conv_state_in,
                      int cs_in_dtype, long long csi_sb, long long csi_sd, int width,
                      long long u_sl);

/*
 * ABI v14.  in_proj + the mixer middle in two launches at small batches (token-major, bf16):
 *   xz = hn @ w_in^T (mamba_simple.py:333-339) — only its z half is written, to `z`
 *   (ntok, dim), row stride ldz; the x half stays in the GEMM's LDS tiles, where
 *   u = silu(conv1d([conv_state_in | x])) (:381-404), written to `u` (row stride u_tl), and
 *   the fixed 128-channel split partials of x_dbl = u @ W_x^T (:409) are formed; then
 *   x_dbl (row stride xd_tl) and, when `dt` is not NULL, dt = x_dbl[:, :r] @ W_dt^T
 *   (:410-413; row stride dt_tl) — every output bit-identical to vm_linear_fwd followed by
 *   vm_conv_proj_fwd (its small-batch forms), so chunked == full stays exact.
 * hn: (batch * out_len, k) bf16, row stride ldh; w_in: (2 dim, k) bf16, row stride ldw;
 * k in {192, 384, 576, 768, 1152, 1536}; batch <= 8, out_len >= 56 (even), dim % 128 == 0
 * and <= 2048, R + 2N <= 76 (e_pad <= 80), width <= 4; conv weights / state, wx_pad,
 * wdt_pad as vm_conv_proj_fwd.  Rows with step >= seqlen get u = 0.  `workspace`:
 * vm_in_proj_conv_proj_workspace_bytes() bytes (the x_dbl partials).
 * vm_in_proj_conv_proj_fits: 1 when the shape is accepted (pure host code).
 */
int vm_in_proj_conv_proj_fwd(const void* hn, long long ldh, const void* w_in, long long ldw, int k,
                             void* z, long long ldz, const float* conv_weight,
                             const float* conv_bias, const void* cs_in, int cs_in_dtype,
                             long long csi_sb, long long csi_sd, void* cs_out, int cs_out_dtype,
                             long long cso_sb, long long cso_sd, const void* wx_pad, int e,
                             int e_pad, const void* wdt_pad, int r, int r_pad, void* u,
                             long long u_tl, void* xdbl, long long xd_tl, void* dt,
                             long long dt_tl, int out_len, int batch, int dim, int seqlen,
                             int width, void* workspace, long long workspace_bytes,
                             vm_stream_t stream);
long long vm_in_proj_conv_proj_workspace_bytes(int batch, int out_len, int dim, int e);
int vm_in_proj_conv_proj_fits(int k, int batch, int out_len, int dim, int e, int e_pad,
                              int r_pad, int width, int has_dt);

/*
 * Channel-major mixer middle (bf16, small batches; the (D, B*L) layout of
 * mamba_simple.py:333-416):  u = silu(conv1d([conv_state_in | x])) -> x_dbl = W_x @ u ->
 * dt = W_dt @ x_dbl[:r], each rounded to bf16 (the reference's rounding points).
 * x: the first `dim` rows of xz, row stride x_sd, columns = batch * out_len tokens (batch b's
 * steps at columns b*out_len + t, unit stride).  u, dt: (dim, batch*out_len) row strides
 * u_sd / dt_sd; x_dbl: (e, batch*out_len) row stride xd_sd.  Columns with t >= seqlen are
 * written as 0.  wx_pad / wdt_pad / conv weights and state as vm_conv_proj_fwd.
 * The x_proj reduction over channels runs in a fixed split order (fp32 partials in
 * `workspace`, vm_conv_proj_cm_workspace_bytes() bytes), so every token's outputs are
 * independent of the sequence length and batch (chunked == full-sequence, bitwise).
 * dim % 64 == 0, out_len % 8 == 0, seqlen >= 1, width <= 4.
 */
int vm_conv_proj_cm_fwd(const void* xz, long long x_sd, const float* conv_weight,
                        const float* conv_bias,
                        const void* cs_in, int cs_in_dtype, long long csi_sb, long long csi_sd,
                        void* cs_out, int cs_out_dtype, long long cso_sb, long long cso_sd,
                        const void* wx_pad, int e, int e_pad, const void* wdt_pad, int r,
                        int r_pad, void* u, long long u_sd, void* xdbl, long long xd_sd,
                        void* dt, long long dt_sd, int out_len, int batch, int dim,
                        int seqlen, int width, void* workspace, long long workspace_bytes,
                        vm_stream_t stream);

/* Scratch bytes vm_conv_proj_cm_fwd needs for this shape (its x_proj partials). */
long long vm_conv_proj_cm_workspace_bytes(int batch, int out_len, int dim, int e);

/*
 * One-token conv step: shift conv_state left by one, append x, dot with weight (+bias),
 * optional SiLU.  x, out: (batch, dim) strides (*_sb, 1); conv_state in place.
 */
int vm_causal_conv1d_update(const void* x, long long x_sb, void* conv_state, int cs_dtype,
                            long long cs_sb, long long cs_sd, const float* weight,
                            const float* bias, void* out, long long o_sb,
                            int batch, int dim, int width, int silu, int dtype,
                            vm_stream_t stream);

/*
 * Fused residual add + RMSNorm / LayerNorm over contiguous rows of `cols`:
 *   s = x (+ residual) in fp32;  y = norm(s) * weight (+ bias)  -> out (out_dtype)
 *   residual_out (nullable) = s in res_out_dtype.
 * residual (nullable) and residual_out may alias.
 */
int vm_add_norm_fwd(const void* x, int x_dtype, const void* residual, int res_dtype,
                    const float* weight, const float* bias, void* out, int out_dtype,
                    void* residual_out, int res_out_dtype, long long rows, int cols,
                    float eps, int is_rms, vm_stream_t stream);

/*
 * Final add + norm fused with the pooling front half.  Per batch row b, rows
 * [0, rows) of x (+ residual) at x + b*in_batch_stride are normalised into out + b *
 * out_batch_stride (rows contiguous).  rev_frame > 0 reads rows [head, rows) in reversed
 * frame order (frames of rev_frame rows, row order kept within a frame): the flipped
 * input of BiMambaRefinerBlock's backward block (models/refiner_backbone.py:98-135).  Rows [0, head) (the CLS row) are only normalised;
 * rows [head, rows) form `groups` pooling groups: equal groups of `group_rows` rows when
 * bounds == NULL (head + groups*group_rows == rows, max_group_rows == group_rows), else
 * bounds (batch, groups+1) int32 row bounds with bounds[b][0] == head and
 * bounds[b][groups] == rows and every group at most max_group_rows rows.  With a
 * workspace (>= vm_norm_pool_workspace_bytes) the fp32 column sums of the rounded outputs
 * of each group are written there for vm_pool_finish_fwd; NULL skips them.
 * cols % 4 == 0, cols <= 2048, 16-byte aligned x / residual / out / weight.
 */
long long vm_norm_pool_workspace_bytes(int batch, int groups, int max_group_rows, int cols);
int vm_norm_pool_fwd(const void* x, int x_dtype, const void* residual, int res_dtype,
                     long long in_batch_stride, const float* weight, const float* bias,
                     float eps, int is_rms, void* out, int out_dtype,
                     long long out_batch_stride, int batch, int rows, int cols, int head,
                     int groups, int group_rows, const int* bounds, int max_group_rows,
                     int rev_frame, void* workspace, long long workspace_bytes,
                     vm_stream_t stream);

/*
 * Pool tail over vm_norm_pool_fwd's workspace (same batch / groups / group_rows /
 * bounds / max_group_rows).  mode: 0 avg, 1 cls+avg, 2 cls_cat_avg, 3 cls.  The average
 * is per group (keep_temporal) or over all groups, rounded to xp_dtype; cls+avg adds the
 * CLS row (cls + b*cls_batch_stride, rounded again); cls_cat_avg puts the CLS row first.
 * Each pooled row then gets LayerNorm(ln_weight, ln_bias, ln_eps) -> x_pool
 * (batch, P, cols) with P = 1 (cls), groups or 1 (avg, cls+avg), 1 + that (cls_cat_avg).
 */
int vm_pool_finish_fwd(const void* workspace, int batch, int groups, int group_rows,
                       const int* bounds, int max_group_rows, const void* cls, int cls_dtype,
                       long long cls_batch_stride, int mode, int keep_temporal,
                       const float* ln_weight, const float* ln_bias, float ln_eps,
                       void* x_pool, int xp_dtype, int cols, vm_stream_t stream);

/*
 * out (m, n) = x (m, k) @ w (n, k)^T (+ bias (n), fp32, nullable): bf16 operands, fp32
 * accumulation, rows K-contiguous with leading dimensions ldx / ldw / ldo (elements).
 * n, k and the leading dimensions multiples of 8, 16-byte aligned operands.  Each output
 * row is computed in the same order for every m (sequence-length independent).
 */
int vm_linear_fwd(const void* x, long long ldx, const void* w, long long ldw,
                  const float* bias, void* out, long long ldo, int m, int n, int k, int dtype,
                  vm_stream_t stream);

/*
 * vm_linear_fwd with the kernel form named (ABI v10): 0 = chosen by shape (what
 * vm_linear_fwd does), 1 = the LDS-DMA tile kernel (128-row tiles, one launch wave), 2 = the
 * persistent 256-row tile kernel (one workgroup per CU walking XCD-contiguous runs of
 * 256 x 256 or 256 x 192 tiles; needs bias == NULL and n a multiple of 256 or 192).  Every
 * form computes each output element as the same chain of MFMAs (K in 64-wide steps, in
 * order), so their outputs are bit-identical and a row never depends on m — the form only
 * changes speed.  Form 0 takes the persistent kernel from 1.5 tiles per CU up (the mixer's
 * projections above a few clips: in_proj / out_proj at 448 clips, mamba_simple.py:333-339,
 * :445-446).
 */
int vm_linear_fwd_form(const void* x, long long ldx, const void* w, long long ldw,
                       const float* bias, void* out, long long ldo, int m, int n, int k,
                       int dtype, int form, vm_stream_t stream);

/*
 * out_proj fused with the NEXT block's residual add + RMSNorm (mamba_simple.py:445-446, then
 * videomamba.py:141-166 with fused_add_norm, rms_norm, residual_in_fp32):
 *   h = bf16(x @ w^T);  residual += h (fp32, in place);  hn = bf16(rmsnorm(residual) * nw)
 * with vm_add_norm_fwd's exact arithmetic (bit-identical to vm_linear_fwd + vm_add_norm_fwd).
 * x (m, k), w (n, k), h (m, n), hn (m, n) bf16; residual (m, n) fp32; norm_weight (n) fp32.
 * ONE launch when the 128 x 64-tile grid fits the stream's device at one workgroup per CU
 * (ABI v13; B = 1 out_proj shapes): after its tile every workgroup normalises a share of the
 * rows, waiting (bounded) on per-128-row-tile counters that the tiles' producers add to
 * after agent-coherent h stores; a timeout sets word 0 of `counters` and makes the rows NaN.
 * Chip-filling row counts (where vm_linear_fwd picks the persistent tile kernel) with
 * (n, k) = (192, 384), (384, 768) or (576, 1152) — the Ti / S / M out_proj — run the
 * persistent kernel's NORM form: the workgroup of a 256-row block's last column tile, after
 * the other column tiles' producers count in, normalises the block (any row count, operands
 * past 2 GB).  Other larger grids run vm_linear_fwd + vm_add_norm_fwd (contiguous h /
 * residual / hn rows).  Every form gives the bits of the two separate calls; both fused
 * forms measured slower than the separate calls on MI355X, so the model
 * uses this entry point only when options.fuse_out_norm is set.
 * `counters`: vm_linear_add_norm_counter_bytes(m) zeroed bytes, left zeroed; one buffer must
 * not serve two launches that can run at the same time.  n % 8 == 0, n <= 1024, k as
 * vm_linear_fwd.
 */
long long vm_linear_add_norm_counter_bytes(int m);
int vm_linear_add_norm_fwd(const void* x, long long ldx, const void* w, long long ldw,
                           void* h, long long ldo, float* residual, long long ldr,
                           const float* norm_weight, float eps, void* hn, long long ldh,
                           int m, int n, int k, void* counters, long long counter_bytes,
                           vm_stream_t stream);

/*
 * Tubelet patch embed + positional embeddings (Conv3d with kernel = stride = (kt,Ph,Pw);
 * rectangular patches as the reference's PatchEmbed(patch_size=(ph, pw)), :340-364):
 *   tok[b, t*Gh*Gw + gh*Gw + gw, c] = e(e(e(conv + bias) + spos[gh*Gw+gw, c]) + tpos[t, c])
 * where e() rounds to the model dtype (the reference's rounding points).
 * video: (batch, cin, frames, height, width) contiguous, dtype `dtype`.
 * weight: (embed, cin*kt*P*P) contiguous, dtype `dtype`; bias: (embed) fp32.
 * spos: (Gh*Gw, embed), tpos: (frames/kt, embed), dtype `dtype`, contiguous.
 * out: token rows of `embed` elements; token j of batch b at out + b*out_sb + (row0+j)*embed.
 * ABI v12: cls / cls_pos (embed elements of `dtype`, both or neither) also write the rows
 * [0, row0) of every batch as e(cls + cls_pos) — the reference's CLS token plus its
 * positional embedding (videomamba.py:806-815) — and pad_rows zero rows follow the last
 * token (the padded buffer's tail), inside the same launch.
 */
int vm_patch_embed_fwd(const void* video, const void* weight, const float* bias,
                       const void* spos, const void* tpos, void* out, long long out_sb,
                       int row0, int batch, int cin, int frames, int height, int width,
                       int kt, int patch_h, int patch_w, int embed, int dtype,
                       const void* cls, const void* cls_pos, int pad_rows,
                       vm_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* VIDEOMAMBA_HIP_H */
