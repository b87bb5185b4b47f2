// Split-K mixer middle for small batches: depthwise causal conv1d + SiLU -> x_proj ->
// dt_proj, token-major (the mixer's layout at every batch) and channel-major.
//
// Replaces the three steps the reference runs between in_proj and the scan
// (models/videomamba/mamba_simple.py:381-416):
//     u     = silu(conv1d(x [+ conv_state]))            (causal_conv1d_fn)
//     x_dbl = u @ W_x^T                                   (x_proj, R + 2N outputs)
//     dt    = x_dbl[:, :R] @ W_dt^T                       (dt_proj weight; bias -> scan)
// with the reference's rounding points (u, x_dbl, dt rounded to bf16; fp32 accumulation).
//
// Why a split-K form: at B = 1 (the streaming-chunk latency path, 3,144 token rows) the
// one-workgroup-per-64-rows kernel of vm_conv_proj.hip has 49 workgroups for 256 CUs and
// sweeps all 1,152 channels serially (94 us per layer, profiles/r02_b1_*), and the library
// GEMMs for x_proj / dt_proj are latency-bound (12-14 us each for 7 MB) and pick split-K
// forms whose accumulation order depends on the token count — which broke chunked ==
// full-sequence bit-equality (scripts/diag/chunk_invariance.py: 5.4e-4 relative at M-32f).
// Here the channels split into FIXED 128-channel ranges (split s = channels 128s..128s+127,
// partials summed in split order), so every token's x_dbl / dt bits are independent of
// the sequence length and batch, and 49 x 9 = 441 workgroups fill the chip at B = 1.
//
//   conv_xproj_*_kernel  grid (token tiles of 64, channel splits): the x tile (+ conv halo)
//     and the split's W_x slice are staged in LDS, conv + SiLU writes u (global, and an LDS
//     [token][channel] tile), v_mfma_f32_16x16x32_bf16 accumulates the split's x_dbl
//     partial; partials go to an fp32 workspace.
//   xdbl_dt_*_kernel     grid (token tiles of 64, 128-channel blocks): sums the partials
//     in split order (block 0 also writes x_dbl in bf16), stages x_dbl[:R] as an MFMA
//     operand and computes dt for its 128 channels; dt leaves through an LDS tile as
//     contiguous row segments.
// HBM traffic per token: x in, u / dt out (2 * D * 2 B each) + the partials
// (D/128 * E * 4 B, L2 / infinity-cache resident at small batch).

#include "vm_conv_proj.h"

namespace vm {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct ConvProjCmParams {
  const bf16_t* x;  // rows = channels (stride x_sd), columns = batch * out_len tokens
  const float* cw; const float* cb;
  const void* csi; void* cso;
  const bf16_t* wx;   // (e_pad, D) zero-padded rows
  const bf16_t* wdt;  // (D, r_pad) zero-padded columns
  bf16_t* u; bf16_t* xdbl; bf16_t* dt;
  float* part;        // [nsplit][e][ntok] fp32 partials of x_dbl
  long long x_sd, u_sd, xd_sd, dt_sd, csi_sb, csi_sd, cso_sb, cso_sd;
  int batch, dim, seqlen, lp, ntok, e, e_pad, r, r_pad, width, csi_dtype, cso_dtype;
  int nsplit, split_ch;  // channel splits of the x_proj reduction, channels per split
};

constexpr int kCmTok = 64;    // token columns per workgroup
constexpr int kCmPitch = 72;  // LDS row pitch in bf16 (144 B): 16-B aligned rows
constexpr int kCmHalo = 8;    // tokens staged before the tile (>= width - 1, 16-B aligned)

// ---------------------------------------------------------------- conv + x_proj partials
template <int NB>  // NB = e_pad / 16 output row blocks of x_proj
__global__ __launch_bounds__(256) void conv_xproj_cm_kernel(const ConvProjCmParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t sX[64 * kCmPitch];      // [ch][halo + tok]
  __shared__ __attribute__((aligned(16))) bf16_t sU[kCmTok * kCmPitch];  // [tok][ch]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int tok0 = blockIdx.x * kCmTok;
  const int split = blockIdx.y;
  const int c_beg = split * p.split_ch;
  const int c_end = min(p.dim, c_beg + p.split_ch);
  const int W = p.width;

  // conv role: channel (lane) x 16 consecutive tokens (wave)
  const int ct0 = wave * 16;
  f32x4 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = c_beg; c0 < c_end; c0 += 64) {
    // ---- stage x[c0 .. c0+63][tok0 - 8 .. tok0 + 63] (16-B pieces, zero outside) ----
    for (int i = tid; i < 64 * 9; i += 256) {
      const int row = i / 9, seg = i - row * 9;
      const int t = tok0 - kCmHalo + seg * 8;
      uint4 q = make_uint4(0, 0, 0, 0);
      if (t >= 0 && t + 8 <= p.ntok)
        q = *reinterpret_cast<const uint4*>(p.x + (long long)(c0 + row) * p.x_sd + t);
      else if (t + 8 > 0 && t < p.ntok) {  // ragged end of the token axis
        uint16_t h[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
          h[k] = (t + k >= 0 && t + k < p.ntok) ? p.x[(long long)(c0 + row) * p.x_sd + t + k] : 0;
        q = make_uint4(h[0] | (uint32_t(h[1]) << 16), h[2] | (uint32_t(h[3]) << 16),
                       h[4] | (uint32_t(h[5]) << 16), h[6] | (uint32_t(h[7]) << 16));
      }
      *reinterpret_cast<uint4*>(&sX[row * kCmPitch + seg * 8]) = q;
    }
    __syncthreads();
    // ---- conv + SiLU: channel c0 + lane, tokens ct0 .. ct0 + 15 ----
    {
      const int c = c0 + lane;
      float w[4], bias = p.cb ? p.cb[c] : 0.0f;
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = k < W ? p.cw[c * W + k] : 0.0f;
      const bf16_t* xr = &sX[lane * kCmPitch + kCmHalo + ct0];
      uint16_t outv[16];
      int b = (tok0 + ct0) / p.lp;
      int step = tok0 + ct0 - b * p.lp;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (i > 0 && ++step == p.lp) {  // next batch row (out_len >= 8: at most 2 wraps)
          step = 0;
          ++b;
        }
        const int tok = tok0 + ct0 + i;
        float a = bias;
        if (step >= W - 1) {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (k < W) a = fmaf(w[k], to_f32(xr[i - (W - 1) + k]), a);
        } else {  // taps before the sequence start: conv state (or zeros)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (k < W) {
              const int j = step - (W - 1) + k;  // input index in the virtual sequence
              float v = 0.0f;
              if (j >= 0) v = to_f32(xr[i - (W - 1) + k]);
              else if (p.csi && tok < p.ntok)
                v = load_dyn(p.csi, b * p.csi_sb + (long long)c * p.csi_sd + W + j, p.csi_dtype);
              a = fmaf(w[k], v, a);
            }
          }
        }
        const float uval = (step < p.seqlen && tok < p.ntok)
                               ? a * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-a * kLog2e))
                               : 0.0f;
        outv[i] = from_f32<bf16_t>(uval);
        sU[(ct0 + i) * kCmPitch + lane] = outv[i];
      }
      // u row segment: 16 tokens = 32 B
      if (tok0 + ct0 + 16 <= p.ntok) {
        uint4* dst = reinterpret_cast<uint4*>(p.u + (long long)c * p.u_sd + tok0 + ct0);
        dst[0] = make_uint4(outv[0] | (uint32_t(outv[1]) << 16), outv[2] | (uint32_t(outv[3]) << 16),
                            outv[4] | (uint32_t(outv[5]) << 16), outv[6] | (uint32_t(outv[7]) << 16));
        dst[1] = make_uint4(outv[8] | (uint32_t(outv[9]) << 16), outv[10] | (uint32_t(outv[11]) << 16),
                            outv[12] | (uint32_t(outv[13]) << 16), outv[14] | (uint32_t(outv[15]) << 16));
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (tok0 + ct0 + i < p.ntok) p.u[(long long)c * p.u_sd + tok0 + ct0 + i] = outv[i];
      }
    }
    __syncthreads();
    // ---- x_proj partial: wave = tokens 16w .. 16w+15, all e_pad rows, K = 64 channels ----
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(
          &sU[(wave * 16 + (lane & 15)) * kCmPitch + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(
            p.wx + (long long)(j * 16 + (lane & 15)) * p.dim + c0 + ks * 32 + (lane >> 4) * 8);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[j], 0, 0, 0);
      }
    }
    __syncthreads();  // sX / sU are restaged by the next chunk
  }
  // ---- partials: part[split][e][tok], 16 consecutive tokens per (e) ----
  const int tok = tok0 + wave * 16 + (lane & 15);
  if (tok < p.ntok) {
    float* dst = p.part + (long long)split * p.e * p.ntok + tok;
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int e = j * 16 + (lane >> 4) * 4 + rr;
        if (e < p.e) dst[(long long)e * p.ntok] = acc[j][rr];
      }
  }
}

// ---------------------------------------------------------------- x_dbl reduce + dt_proj
__global__ __launch_bounds__(256) void xdbl_dt_cm_kernel(const ConvProjCmParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t sXD[kCmTok * kCmPitch];   // [tok][k]
  __shared__ __attribute__((aligned(16))) bf16_t sDT[128 * kCmPitch];      // [ch][tok]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int tok0 = blockIdx.x * kCmTok;
  const int cb = blockIdx.y;  // 128-channel block
  const bool writer = cb == 0;
  const int rows = writer ? p.e : p.r;
  // zero the K padding of the dt operand
  for (int i = tid; i < kCmTok * kCmPitch / 8; i += 256)
    reinterpret_cast<uint4*>(sXD)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  for (int idx = tid; idx < rows * kCmTok; idx += 256) {
    const int e = idx / kCmTok, t = idx - e * kCmTok;
    const int tok = tok0 + t;
    if (tok >= p.ntok) continue;
    float s = 0.0f;
    for (int sp = 0; sp < p.nsplit; ++sp) s += p.part[((long long)sp * p.e + e) * p.ntok + tok];
    const bf16_t v = from_f32<bf16_t>(s);
    if (e < p.r) sXD[t * kCmPitch + e] = v;
    if (writer) p.xdbl[(long long)e * p.xd_sd + tok] = v;
  }
  __syncthreads();
  // ---- dt for channels cb*128 + 32w .. +31 (2 row tiles) x 64 tokens (4 column tiles) ----
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ksteps = p.r_pad / 32;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    if (ks < ksteps) {
      bf16x8 av[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ch = min(cb * 128 + wave * 32 + i * 16 + (lane & 15), p.dim - 1);
        av[i] = *reinterpret_cast<const bf16x8*>(p.wdt + (long long)ch * p.r_pad + ks * 32 +
                                                 (lane >> 4) * 8);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(
            &sXD[(j * 16 + (lane & 15)) * kCmPitch + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv, acc[i][j], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        sDT[(wave * 32 + i * 16 + (lane >> 4) * 4 + rr) * kCmPitch + j * 16 + (lane & 15)] =
            from_f32<bf16_t>(acc[i][j][rr]);
  __syncthreads();
  // ---- 128 channel rows x 64 tokens out, 16 B per lane-store ----
  for (int i = tid; i < 128 * 8; i += 256) {
    const int row = i >> 3, q = i & 7;
    const int ch = cb * 128 + row;
    const int tok = tok0 + q * 8;
    if (ch >= p.dim) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(&sDT[row * kCmPitch + q * 8]);
    if (tok + 8 <= p.ntok) {
      *reinterpret_cast<uint4*>(p.dt + (long long)ch * p.dt_sd + tok) = v;
    } else {
      const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
      for (int k = 0; k < 8; ++k)
        if (tok + k < p.ntok) p.dt[(long long)ch * p.dt_sd + tok + k] = h[k];
    }
  }
}

// New conv state (B, D, width): the last `width` raw inputs of each channel (mamba_simple.py
// :383-399) — steps L - width .. L - 1 of x, or of the old state before the sequence start.
__global__ __launch_bounds__(256) void conv_state_cm_kernel(const ConvProjCmParams p) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (c >= p.dim) return;
  for (int s = 0; s < p.width; ++s) {
    const int te = p.seqlen - p.width + s;
    float val = 0.0f;
    if (te >= 0) val = to_f32(p.x[(long long)c * p.x_sd + (long long)b * p.lp + te]);
    else if (p.csi) val = load_dyn(p.csi, b * p.csi_sb + (long long)c * p.csi_sd + p.width + te,
                                   p.csi_dtype);
    store_dyn(p.cso, b * p.cso_sb + (long long)c * p.cso_sd + s, p.cso_dtype, val);
  }
}

// ================================================================ token-major split-K
constexpr int kTmPitch = 136;  // LDS row pitch in bf16 (272 B): 128 channels + 16-B pad
constexpr int kSkCh = 128;     // channels per split (fixed: see the file header)
// conv-state rows staged per tile: sequences whose first 3 steps touch a 64-token tile
// (out_len >= 8: at most 64 / 8 + 1)
constexpr int kSkCsRows = kCmTok / 8 + 1;
constexpr int kSkCsLoads = (kSkCsRows * 3 * kSkCh + 255) / 256;

struct SkTmParams {
  ConvProjTmArgs a;
  float* part;  // [nsplit][ntok][ep] fp32 partials of x_dbl, ep = round_up(e, 4)
  int ntok, nsplit, ep;
};

// x tile rows tok0 - 8 .. tok0 + 63 (zero outside [0, ntok)), channels c0 .. c0 + 127.
// Latency shape (what bounds these kernels at B = 1, where a CU holds ~2 workgroups and
// nothing overlaps them): every global load the workgroup needs is issued up front and
// waited for once; the u and partial stores go out last, so no barrier drains them.
template <int NB>  // NB = e_pad / 16 output column blocks of x_proj
__global__ __launch_bounds__(256) void conv_xproj_tm_kernel(const SkTmParams q) {
  const ConvProjTmArgs& p = q.a;
  extern __shared__ __attribute__((aligned(16))) bf16_t sm[];
  bf16_t* sX = sm;                         // [72][kTmPitch]
  bf16_t* sU = sX + 72 * kTmPitch;         // [64][kTmPitch]
  bf16_t* sW = sU + kCmTok * kTmPitch;     // [e_pad][kTmPitch]
  float* sC = reinterpret_cast<float*>(sW + p.e_pad * kTmPitch);  // [kSkCsRows][3][128]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int tok0 = blockIdx.x * kCmTok;
  const int split = blockIdx.y;
  const int c0 = split * kSkCh;
  const int W = p.width;
  const int nch = min(kSkCh, p.dim - c0);  // 128, or 64 for the last split of dim % 128 == 64
  const bool cact = 2 * lane < nch;
  const int c = c0 + 2 * (cact ? lane : 0);
  // ---- one round of global loads: x tile, W_x slice, this thread's conv taps ----
  constexpr int kXI = (72 * 16 + 255) / 256;  // 16-B x pieces per thread (5)
  uint4 xv[kXI];
#pragma unroll
  for (int k = 0; k < kXI; ++k) {
    const int i = tid + k * 256;
    const int rr = i >> 4, qd = i & 15;
    const int tok = tok0 - kCmHalo + rr;
    xv[k] = make_uint4(0, 0, 0, 0);
    if (i < 72 * 16 && tok >= 0 && tok < q.ntok && qd * 8 < nch)
      xv[k] = *reinterpret_cast<const uint4*>(p.x + (long long)tok * p.x_tl + c0 + qd * 8);
  }
  constexpr int kWI = (NB * 16 * 16 + 255) / 256;  // 16-B W_x pieces per thread
  uint4 wv[kWI];
#pragma unroll
  for (int k = 0; k < kWI; ++k) {
    const int i = tid + k * 256;
    const int e = i >> 4, qd = i & 15;
    wv[k] = make_uint4(0, 0, 0, 0);
    if (i < NB * 16 * 16 && qd * 8 < nch)
      wv[k] = *reinterpret_cast<const uint4*>(p.wx + (long long)e * p.dim + c0 + qd * 8);
  }
  // taps right-aligned to 4 (a width-W filter is a 4-tap filter with 4 - W leading zeros),
  // so tap k of token i always reads window row i + k
  float wl[4], wh[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    static_assert(4 * 16 * kSkMaxEp * 4 <= 72 * kTmPitch * 2, "partial rows exceed the x tile");
    wl[k] = k >= 4 - W ? p.cw[c * W + k - (4 - W)] : 0.0f;
    wh[k] = k >= 4 - W ? p.cw[(c + 1) * W + k - (4 - W)] : 0.0f;
  }
  const float bl = p.cb ? p.cb[c] : 0.0f, bh = p.cb ? p.cb[c + 1] : 0.0f;
  // old conv-state taps (steps -3 .. -1) of every sequence whose first steps fall in this
  // tile, staged with the same load round: read inside the conv loop they were dependent
  // round trips that held the tile containing a sequence start for several microseconds
  const int b_lo = tok0 / p.out_len;
  const int nbs = p.csi ? min(p.batch - 1, (tok0 + kCmTok - 1) / p.out_len) - b_lo + 1 : 0;
  float cv[kSkCsLoads];
#pragma unroll
  for (int k = 0; k < kSkCsLoads; ++k) {
    const int i = tid + k * 256;
    const int bb = i / (3 * kSkCh), m = (i / kSkCh) % 3, ch = i % kSkCh;
    const int tap = W - 1 - m;  // state column of step -(m + 1)
    cv[k] = 0.0f;
    if (bb < nbs && ch < nch && tap >= 0)
      cv[k] = load_dyn(p.csi, (b_lo + bb) * p.csi_sb + (long long)(c0 + ch) * p.csi_sd + tap,
                       p.csi_dtype);
  }
#pragma unroll
  for (int k = 0; k < kSkCsLoads; ++k) {
    const int i = tid + k * 256;
    if (i / (3 * kSkCh) < nbs) sC[i] = cv[k];
  }
#pragma unroll
  for (int k = 0; k < kXI; ++k) {
    const int i = tid + k * 256;
    if (i < 72 * 16) *reinterpret_cast<uint4*>(&sX[(i >> 4) * kTmPitch + (i & 15) * 8]) = xv[k];
  }
#pragma unroll
  for (int k = 0; k < kWI; ++k) {
    const int i = tid + k * 256;
    if (i < NB * 16 * 16) *reinterpret_cast<uint4*>(&sW[(i >> 4) * kTmPitch + (i & 15) * 8]) = wv[k];
  }
  __syncthreads();
  // ---- new conv state: the last `width` raw inputs of every sequence ending in this tile
  // (mamba_simple.py:383-399), from the staged rows (width - 1 <= halo) or the old state ----
  if (p.cso && tid < nch) {
    const int b1 = min(p.batch - 1, (tok0 + kCmTok - 1) / p.out_len);
    for (int b = tok0 / p.out_len; b <= b1; ++b) {
      const int tl = b * p.out_len + p.seqlen - 1;
      if (tl < tok0 || tl >= tok0 + kCmTok) continue;
      const int ch = c0 + tid;
      for (int s = 0; s < W; ++s) {
        const int te = p.seqlen - W + s;
        float v = 0.0f;
        if (te >= 0)
          v = to_f32(sX[(kCmHalo + b * p.out_len + te - tok0) * kTmPitch + tid]);
        else if (p.csi)
          v = load_dyn(p.csi, b * p.csi_sb + (long long)ch * p.csi_sd + W + te, p.csi_dtype);
        store_dyn(p.cso, b * p.cso_sb + (long long)ch * p.cso_sd + s, p.cso_dtype, v);
      }
    }
  }
  // ---- conv + SiLU: channels c, c + 1 (one packed word), tokens 16w .. 16w+15 ----
  // The wave's 16 tokens read a 19-row window, loaded from LDS up front (a uniform branch
  // per tap made every token a chain of LDS round trips: 7.6 us of the kernel at B = 1).
  // Tokens in the first 3 steps of their sequence are redone below with the taps before
  // the sequence (old conv state staged in sC, or zeros).
  const int t0 = wave * 16;
  uint32_t xw[19];
#pragma unroll
  for (int r = 0; r < 19; ++r)
    xw[r] = *reinterpret_cast<const uint32_t*>(&sX[(kCmHalo + t0 - 3 + r) * kTmPitch + 2 * lane]);
  const int bw = (tok0 + t0) / p.out_len;  // batch row and step of the wave's first token
  const int sw = tok0 + t0 - bw * p.out_len;
  auto token_pos = [&](int i, int& b, int& st) {  // out_len >= 8: at most 2 wraps in 16
    b = bw;
    st = sw + i;
    if (st >= p.out_len) { st -= p.out_len; ++b; }
    if (st >= p.out_len) { st -= p.out_len; ++b; }
  };
  auto pack = [&](float al, float ah, bool live) -> uint32_t {
    const float ul = live ? al * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-al * kLog2e)) : 0.0f;
    const float uh = live ? ah * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-ah * kLog2e)) : 0.0f;
    return static_cast<uint32_t>(from_f32<bf16_t>(ul)) |
           (static_cast<uint32_t>(from_f32<bf16_t>(uh)) << 16);
  };
  uint32_t upk[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float al = bl, ah = bh;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      al = fmaf(wl[k], __uint_as_float(xw[i + k] << 16), al);
      ah = fmaf(wh[k], __uint_as_float(xw[i + k] & 0xffff0000u), ah);
    }
    int b, st;
    token_pos(i, b, st);
    upk[i] = pack(al, ah, st < p.seqlen && tok0 + t0 + i < q.ntok && cact);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    int b, st;
    token_pos(i, b, st);
    if (st < 3) {  // uniform: a sequence starts at or just before this token
      float al = bl, ah = bh;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int j = st - 3 + k;  // input step in the virtual sequence
        float vl = __uint_as_float(xw[i + k] << 16), vh = __uint_as_float(xw[i + k] & 0xffff0000u);
        if (j < 0) {
          vl = vh = 0.0f;
          if (p.csi && tok0 + t0 + i < q.ntok && k >= 4 - W) {
            const float2 cs = *reinterpret_cast<const float2*>(
                &sC[((b - b_lo) * 3 - j - 1) * kSkCh + 2 * lane]);
            vl = cs.x;
            vh = cs.y;
          }
        }
        al = fmaf(wl[k], vl, al);
        ah = fmaf(wh[k], vh, ah);
      }
      upk[i] = pack(al, ah, st < p.seqlen && tok0 + t0 + i < q.ntok && cact);
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i)
    *reinterpret_cast<uint32_t*>(&sU[(t0 + i) * kTmPitch + 2 * lane]) = upk[i];
  __syncthreads();
  // ---- x_proj partial: wave = tokens 16w .. 16w+15 x all e_pad columns, K = 128 ----
  f32x4 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const bf16x8 av = *reinterpret_cast<const bf16x8*>(
        &sU[(wave * 16 + (lane & 15)) * kTmPitch + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(
          &sW[(j * 16 + (lane & 15)) * kTmPitch + ks * 32 + (lane >> 4) * 8]);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[j], 0, 0, 0);
    }
  }
  // ---- stores last: u rows (256 B per wave-store) and the partials ----
  if (cact) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int tok = tok0 + t0 + i;
      if (tok < q.ntok) *reinterpret_cast<uint32_t*>(p.u + (long long)tok * p.u_tl + c) = upk[i];
    }
  }
  // partials: D[token 4(lane/16) + r][column lane % 16] through this wave's own rows of the
  // (now unused) x tile, then whole part[split][token][0 .. ep) rows as 16-byte stores
  // (20 scattered 4-byte stores per lane were 4.6 us of the kernel at B = 1)
  constexpr int kPP = kSkMaxEp;  // fp32 pitch of the staged rows: 4 x 16 rows fit the x tile
  float* sP = reinterpret_cast<float*>(sX) + wave * 16 * kPP;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int e = j * 16 + (lane & 15);
      if (e < q.ep) sP[((lane >> 4) * 4 + rr) * kPP + e] = acc[j][rr];
    }
  __builtin_amdgcn_wave_barrier();
  const int nq = q.ep >> 2;  // float4 per row
  for (int i = lane; i < 16 * nq; i += 64) {
    const int r = i / nq, qd = i - r * nq;
    const int tok = tok0 + wave * 16 + r;
    if (tok < q.ntok)
      *reinterpret_cast<float4*>(q.part + ((long long)split * q.ntok + tok) * q.ep + 4 * qd) =
          *reinterpret_cast<const float4*>(&sP[r * kPP + 4 * qd]);
  }
}

// x_dbl = bf16(sum of the partials in split order); dt = bf16(x_dbl[:, :R] @ W_dt^T).
// All loads (W_dt fragments, every split's partials) are issued before the first wait.
template <int NSPL>  // splits (dim / 128 rounded up), 1 .. 16
__global__ __launch_bounds__(256) void xdbl_dt_tm_kernel(const SkTmParams q) {
  const ConvProjTmArgs& p = q.a;
  __shared__ __attribute__((aligned(16))) bf16_t sXD[kCmTok * kCmPitch];   // [tok][k]
  __shared__ __attribute__((aligned(16))) bf16_t sDT[kCmTok * kTmPitch];   // [tok][128 ch]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int tok0 = blockIdx.x * kCmTok;
  const int cb = blockIdx.y;  // 128-channel block
  const bool writer = cb == 0;
  const bool do_dt = p.wdt != nullptr;
  bf16x8 bw[2][2];
  if (do_dt) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ch = min(cb * 128 + wave * 32 + i * 16 + (lane & 15), p.dim - 1);
        bw[i][ks] = ks * 32 < p.r_pad
                        ? *reinterpret_cast<const bf16x8*>(p.wdt + (long long)ch * p.r_pad +
                                                           ks * 32 + (lane >> 4) * 8)
                        : bf16x8{};
      }
  }
  // reduction items: (token, 4 consecutive columns) over rows R (the dt operand) or E (the
  // writer block, which also stores x_dbl); every split's float4 of a round of kIt items is
  // in flight together
  const int rows = writer ? p.e : p.r;
  const int q4 = (rows + 3) >> 2;
  const long long sstride = (long long)q.ntok * q.ep;
  constexpr int kIt = 3;
  for (int it0 = 0; it0 < kCmTok * q4; it0 += kIt * 256) {
    float4 part[kIt][NSPL];
#pragma unroll
    for (int k = 0; k < kIt; ++k) {
      const int it = it0 + tid + k * 256;
      const int t = it / q4, e0 = (it - t * q4) * 4;
      const bool ok = it < kCmTok * q4 && tok0 + t < q.ntok;
      const float* src = q.part + (long long)(tok0 + t) * q.ep + e0;
#pragma unroll
      for (int sp = 0; sp < NSPL; ++sp)
        part[k][sp] = ok ? *reinterpret_cast<const float4*>(src + sp * sstride)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < kIt; ++k) {
      const int it = it0 + tid + k * 256;
      if (it >= kCmTok * q4) continue;
      const int t = it / q4, e0 = (it - t * q4) * 4;
      float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int sp = 0; sp < NSPL; ++sp) {
        sum.x += part[k][sp].x; sum.y += part[k][sp].y; sum.z += part[k][sp].z; sum.w += part[k][sp].w;
      }
      const float sv[4] = {sum.x, sum.y, sum.z, sum.w};
      const int tok = tok0 + t;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int e = e0 + kk;
        if (e >= rows) break;
        const bf16_t v = from_f32<bf16_t>(sv[kk]);
        if (e < p.r) sXD[t * kCmPitch + e] = v;
        if (writer && tok < q.ntok) p.xdbl[(long long)tok * p.xd_tl + e] = v;
      }
    }
  }
  // zero K padding of the dt operand (columns r .. r_pad)
  for (int i = tid; i < kCmTok * (p.r_pad - p.r); i += 256) {
    const int t = i / (p.r_pad - p.r);
    sXD[t * kCmPitch + p.r + (i - t * (p.r_pad - p.r))] = bf16_t(0);
  }
  if (!do_dt) return;
  __syncthreads();
  // ---- dt: tokens (4 tiles of 16) x channels cb*128 + 32w .. +31 (2 tiles), K = r_pad ----
  f32x4 acc[4][2];
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[jt][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    if (ks * 32 < p.r_pad) {
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(
            &sXD[(jt * 16 + (lane & 15)) * kCmPitch + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[jt][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bw[i][ks], acc[jt][i], 0, 0, 0);
      }
    }
  }
  // D[token 4(lane/16) + r][channel lane % 16] -> sDT[token][channel]
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        sDT[(jt * 16 + (lane >> 4) * 4 + rr) * kTmPitch + wave * 32 + i * 16 + (lane & 15)] =
            from_f32<bf16_t>(acc[jt][i][rr]);
  __syncthreads();
  // 64 token rows x 128 channels out, 16 B per lane-store
  const int nch = min(128, p.dim - cb * 128);
  for (int i = tid; i < kCmTok * 16; i += 256) {
    const int t = i >> 4, qd = i & 15;
    const int tok = tok0 + t;
    if (tok >= q.ntok || qd * 8 >= nch) continue;
    *reinterpret_cast<uint4*>(p.dt + (long long)tok * p.dt_tl + cb * 128 + qd * 8) =
        *reinterpret_cast<const uint4*>(&sDT[t * kTmPitch + qd * 8]);
  }
}

// ================================================================ fused small-batch form
// One launch for conv + SiLU -> x_proj -> dt_proj at small batches (B <= 8, dim <= 1152):
// a workgroup owns kFuTok = 16 token rows and all channels, one wave per fixed 128-channel
// split (the split-K form's splits).  Each wave runs its split's conv and its x_proj
// partial on MFMA exactly as conv_xproj_tm_kernel does, the partials are summed through LDS
// in split order (exactly the xdbl_dt_tm_kernel sum), and the same waves then run dt_proj
// for their 128 channels — so u / x_dbl / dt are bit-identical to the two-kernel split-K
// form, without its fp32 partials round trip through L2 / infinity cache and with one
// launch fewer per layer.  B = 1 M-16f: 197 workgroups.
//   Loads: every global load of a wave (19 x-rows of its 128 channels, its W_x fragments,
//   conv taps, the conv-state taps of a sequence start) is issued in one round; W_dt
//   fragments are issued right after the x_proj MFMAs and land during the LDS reduction.
constexpr int kFuTok = 16;     // token rows per workgroup
constexpr int kFuMaxSpl = 9;   // splits (waves) per workgroup: dim <= 1152
constexpr int kFuUPitch = 136; // bf16 pitch of a wave's [16 tok][128 ch] u tile
constexpr int kFuXdPitch = 72; // bf16 pitch of the [16 tok][64] x_dbl[:R] operand
constexpr int kFuXRows = 20;   // x rows staged per wave (tok0 - 3 .. tok0 + 16)

// Workgroup barrier over LDS traffic only: __syncthreads() also waits vmcnt(0), which
// drained the W_dt fragment loads (issued to land during the partial reduction) and every
// u / x_dbl store at the first barrier after the x_proj MFMAs (timestamps,
// scripts/diag/stamp_conv_proj.py: that phase took 8.9 us of the 20.9 us kernel at B = 1).
// Register operands still get their own counted waits from the compiler at first use.
__device__ __forceinline__ void fu_lds_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

template <int NB, bool CS32>  // NB = e_pad / 16 x_proj column blocks; CS32: fp32 conv state in
__global__ __launch_bounds__(64 * kFuMaxSpl) void conv_proj_fused_kernel(const SkTmParams q) {
  const ConvProjTmArgs& p = q.a;
  // LDS: per-wave u tiles, then (aliased) the split partials [split][tok][ep], then
  // (aliased) the dt tile [tok][dim]; the x_dbl operand after them
  extern __shared__ __attribute__((aligned(16))) char fsm[];
  constexpr int kUBytes = kFuMaxSpl * kFuTok * kFuUPitch * 2;
  constexpr int kPBytes = kFuMaxSpl * kFuTok * kSkMaxEp * 4;
  constexpr int kArea = kUBytes > kPBytes ? kUBytes : kPBytes;
  bf16_t* sU = reinterpret_cast<bf16_t*>(fsm);
  float* sP = reinterpret_cast<float*>(fsm);
  bf16_t* sXD = reinterpret_cast<bf16_t*>(fsm + kArea);
  bf16_t* sDT = reinterpret_cast<bf16_t*>(fsm);  // [16][dim + 8], after the partials
  const int dtp = p.dim + 8;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;           // = split
  const int nspl = blockDim.x >> 6;
  const int tok0 = blockIdx.x * kFuTok;
  const int c0 = wave * kSkCh;
  const int W = p.width;
  const int nch = min(kSkCh, p.dim - c0);
  const bool cact = 2 * lane < nch;
  const int c = c0 + 2 * (cact ? lane : 0);
  const int ntok = q.ntok;

  // Every global load and store of the tile is a buffer access whose out-of-range offset
  // (rows outside [0, ntok), idle lanes, padding k-steps) reads 0 / stores nothing, so none
  // sits behind a branch: a per-element "load or zero" select made hipcc branch around each
  // access and wait vmcnt(0) after it — 16 dependent round trips for the W_dt fragments,
  // most of the 8.9 us between the conv and the x_proj partials at B = 1
  // (scripts/diag/stamp_conv_proj.py).
  const auto xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p.x), 0, static_cast<int>((long long)ntok * p.x_tl * 2), 0x00020000);
  const auto wxr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p.wx), 0, static_cast<int>((long long)p.e_pad * p.dim * 2), 0x00020000);
  const auto wdr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p.wdt), 0,
      p.wdt ? static_cast<int>((long long)p.dim * p.r_pad * 2) : 0, 0x00020000);
  const auto ur = __builtin_amdgcn_make_buffer_rsrc(
      p.u, 0, static_cast<int>((long long)ntok * p.u_tl * 2), 0x00020000);
  constexpr int kOut = 0x7ffffff0;  // an offset past every range above
  // the offset select stays a select: seen through, hipcc splits the access into a load
  // per arm of a divergent branch and waits vmcnt(0) at the join
  auto opaque = [](int off) {
    asm volatile("" : "+v"(off));
    return off;
  };
  // ---- one round of loads ----
  // the (at most one: out_len >= 24) sequence starting in tok0 - 2 .. tok0 + 15, whose
  // first 3 steps may lie in this tile: its old conv-state taps for steps -1, -2, -3
  // (state columns W - 1, W - 2, W - 3)
  const int bs = (tok0 - 2 + p.out_len - 1) / p.out_len;  // tok0 - 2 + out_len - 1 >= 0
  const int ts = bs * p.out_len;
  const bool has_start = ts < tok0 + kFuTok && bs < p.batch;
  // Loaded first and unconditionally as 16-bit buffer pieces (offsets out of range where
  // unused): no load sits in a branch whose join makes hipcc drain vmcnt, and the counted
  // waits for them never cover the W_x round issued later.
  float csl[3], csh[3];
  {
    constexpr int es = CS32 ? 4 : 2;
    const long long span = p.csi ? ((long long)(p.batch - 1) * p.csi_sb +
                                    (long long)(p.dim - 1) * p.csi_sd + W) * es
                                 : 0;
    const auto csr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.csi), 0,
                                                       static_cast<int>(span), 0x00020000);
    auto tap = [&](long long idx, bool ok) {
      const int off = opaque(ok ? static_cast<int>(idx * es) : kOut);
      if constexpr (CS32)
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(csr, off, 0, 0));
      else
        return __uint_as_float(static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b16(csr, off, 0, 0)) << 16);
    };
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int col = W - 1 - m;
      const bool ok = has_start && p.csi && col >= 0;
      const long long base = (long long)bs * p.csi_sb + (long long)c * p.csi_sd + col;
      csl[m] = tap(base, ok);
      csh[m] = tap(base + p.csi_sd, ok);
    }
  }

  __builtin_amdgcn_sched_barrier(0);
  // x rows tok0 - 3 .. tok0 + 16 of this split's 128 channels go to the wave's own LDS
  // slice by buffer_load ... lds, 4 rows x 256 B per instruction (5 instead of 19 per-lane
  // 4-byte loads: with 9 waves per CU issuing ~70 memory instructions each, their issue
  // backed up; per-wave stamps, scripts/diag/stamp_conv_proj.py --waves).  Rows outside
  // [0, ntok) read as zero or hold stale bytes: their taps are replaced (sequence starts
  // take the conv state) or their outputs dropped (tokens past ntok).
  char* sXw = fsm + kArea + kFuTok * kFuXdPitch * 2 + wave * (kFuXRows * 256);
#pragma unroll
  for (int i = 0; i < kFuXRows / 4; ++i) {
    const int row = 4 * i + (lane >> 4);
    dma16(xr, sXw + i * 1024, ((tok0 - 3 + row) * static_cast<int>(p.x_tl) + c0) * 2 + (lane & 15) * 16);
  }
  __builtin_amdgcn_sched_barrier(0);
  // W_x fragments of this split: column block j, k-step ks (rows e, 8 channels per lane);
  // k-steps 0-1 with the first round, 2-3 once the x rows are consumed (register budget)
  bf16x8 wv[4][NB];
  auto wx_load = [&](int ks) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int kc = ks * 32 + (lane >> 4) * 8;
      wv[ks][j] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                      wxr, opaque(kc < nch ? ((j * 16 + (lane & 15)) * p.dim + c0 + kc) * 2 : kOut),
                      0, 0));
    }
  };
  // conv taps and bias: unconditional loads (clamped index), zeroed by a select
  float wl[4], wh[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int kk = k - (4 - W) > 0 ? k - (4 - W) : 0;
    const float vl = p.cw[c * W + kk], vh = p.cw[(c + 1) * W + kk];
    wl[k] = k >= 4 - W ? vl : 0.0f;
    wh[k] = k >= 4 - W ? vh : 0.0f;
  }
  const float* cbp = p.cb ? p.cb : p.cw;
  const float bl0 = cbp[c], bh0 = cbp[c + 1];
  const float bl = p.cb ? bl0 : 0.0f, bh = p.cb ? bh0 : 0.0f;
  __builtin_amdgcn_sched_barrier(0);
  wx_load(0);
  wx_load(1);
  __builtin_amdgcn_sched_barrier(0);
  // the x rows (and the taps) have landed once only the 2 * NB W_x loads are in flight;
  // each wave reads only the rows its own DMA wrote
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  if constexpr (2 * NB == 2) __builtin_amdgcn_s_waitcnt(0x0F72);
  else if constexpr (2 * NB == 4) __builtin_amdgcn_s_waitcnt(0x0F74);
  else if constexpr (2 * NB == 6) __builtin_amdgcn_s_waitcnt(0x0F76);
  else if constexpr (2 * NB == 8) __builtin_amdgcn_s_waitcnt(0x0F78);
  else __builtin_amdgcn_s_waitcnt(0x0F7A);  // vmcnt(10)
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  uint32_t xw[kFuTok + 3];
#pragma unroll
  for (int r = 0; r < kFuTok + 3; ++r)
    xw[r] = cact ? *reinterpret_cast<const uint32_t*>(sXw + r * 256 + 4 * lane) : 0u;
  // ---- conv + SiLU: channels c, c + 1, tokens tok0 .. tok0 + 15 ----
  auto pack = [&](float al, float ah, bool live) -> uint32_t {
    const float ul = live ? al * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-al * kLog2e)) : 0.0f;
    const float uh = live ? ah * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-ah * kLog2e)) : 0.0f;
    return static_cast<uint32_t>(from_f32<bf16_t>(ul)) |
           (static_cast<uint32_t>(from_f32<bf16_t>(uh)) << 16);
  };
  const int b0 = tok0 / p.out_len;  // batch row and step of the tile's first token
  const int s0 = tok0 - b0 * p.out_len;
  // the channel pair's taps as packed operands: v_pk_fma_f32 does per lane exactly the
  // scalar fmaf chain (same taps, same order), half the VALU issue
  typedef __attribute__((ext_vector_type(2))) float fp2;
  fp2 wp[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) wp[k] = fp2{wl[k], wh[k]};
  uint32_t upk[kFuTok];
#pragma unroll
  for (int i = 0; i < kFuTok; ++i) {
    fp2 acc2 = fp2{bl, bh};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      acc2 = __builtin_elementwise_fma(
          wp[k], fp2{__uint_as_float(xw[i + k] << 16), __uint_as_float(xw[i + k] & 0xffff0000u)}, acc2);
    float al = acc2.x, ah = acc2.y;
    int st = s0 + i;
    if (st >= p.out_len) st -= p.out_len;  // out_len >= 16: at most one wrap
    if (st < 3) {  // uniform: the taps before the sequence start come from the old state
      al = bl;
      ah = bh;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int j = st - 3 + k;  // input step in the virtual sequence
        float vl = __uint_as_float(xw[i + k] << 16), vh = __uint_as_float(xw[i + k] & 0xffff0000u);
        if (j < 0) {
          vl = vh = 0.0f;
          if (p.csi && tok0 + i < ntok && k >= 4 - W) {
            vl = csl[-j - 1];
            vh = csh[-j - 1];
          }
        }
        al = fmaf(wl[k], vl, al);
        ah = fmaf(wh[k], vh, ah);
      }
    }
    upk[i] = pack(al, ah, st < p.seqlen && tok0 + i < ntok && cact);
  }
  wx_load(2);
  wx_load(3);
  // ---- u: global rows and this wave's LDS tile ----
  bf16_t* myU = sU + wave * kFuTok * kFuUPitch;
#pragma unroll
  for (int i = 0; i < kFuTok; ++i)
    *reinterpret_cast<uint32_t*>(&myU[i * kFuUPitch + 2 * lane]) = upk[i];
  __builtin_amdgcn_wave_barrier();
  // ---- x_proj partial of this split: tokens x e_pad columns, K = 128 ----
  f32x4 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const bf16x8 av = *reinterpret_cast<const bf16x8*>(
        &myU[(lane & 15) * kFuUPitch + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
    for (int j = 0; j < NB; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, wv[ks][j], acc[j], 0, 0, 0);
  }
  // u rows leave from the LDS tile as 16-byte pieces (4 stores per lane instead of 16)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int id = k * 64 + lane, row = id >> 4, ch = (id & 15) * 8;
    typedef __attribute__((__vector_size__(4 * sizeof(int)))) int v4i;
    const v4i v = *reinterpret_cast<const v4i*>(&myU[row * kFuUPitch + ch]);
    __builtin_amdgcn_raw_buffer_store_b128(
        v, ur,
        opaque(ch < nch && tok0 + row < ntok ? ((tok0 + row) * static_cast<int>(p.u_tl) + c0 + ch) * 2
                                             : kOut),
        0, 0);
  }
  // W_dt fragments for this wave's dt channels (128 per wave, 8 column tiles x 2 k-steps),
  // in flight during the reduction
  const bool do_dt = p.wdt != nullptr;
  bf16x8 bw[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = min(c0 + i * 16 + (lane & 15), p.dim - 1);
      bw[i][ks] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                      wdr, opaque(ks * 32 < p.r_pad ? (ch * p.r_pad + ks * 32 + (lane >> 4) * 8) * 2
                                                  : kOut),
                      0, 0));
    }
  fu_lds_barrier();  // every wave's u tile is consumed: the area becomes the partials
  const int ep = q.ep;
  float* myP = sP + wave * kFuTok * ep;
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int e = j * 16 + (lane & 15);
      if (e < ep) myP[((lane >> 4) * 4 + rr) * ep + e] = acc[j][rr];
    }
  // zero the K padding of the dt operand
  for (int i = tid; i < kFuTok * (p.r_pad - p.r); i += blockDim.x) {
    const int t = i / (p.r_pad - p.r);
    sXD[t * kFuXdPitch + p.r + (i - t * (p.r_pad - p.r))] = bf16_t(0);
  }
  fu_lds_barrier();
  // ---- x_dbl = bf16(sum of the partials in split order) ----
  for (int i = tid; i < kFuTok * p.e; i += blockDim.x) {
    const int t = i / p.e, e = i - t * p.e;
    float sum = 0.0f;
    for (int sp = 0; sp < nspl; ++sp) sum += sP[(sp * kFuTok + t) * ep + e];
    const bf16_t v = from_f32<bf16_t>(sum);
    if (e < p.r) sXD[t * kFuXdPitch + e] = v;
    if (tok0 + t < ntok) p.xdbl[(long long)(tok0 + t) * p.xd_tl + e] = v;
  }
  // ---- new conv state of a sequence ending in this tile: its last W raw inputs (from the
  // staged x rows), written last: after the conv, the branch's join made hipcc wait
  // vmcnt(0) there, serialising the two W_x load rounds ----
  auto write_conv_state = [&]() {
    if (p.cso && cact) {
      const int be1 = min(p.batch - 1, (tok0 + kFuTok - 1) / p.out_len);
      for (int be = b0; be <= be1; ++be) {  // the tile's (at most two) sequences
        const int tl = be * p.out_len + p.seqlen - 1;
        if (tl < tok0 || tl >= tok0 + kFuTok) continue;
        for (int s2 = 0; s2 < W; ++s2) {
          const int te = p.seqlen - W + s2;
          float vl = 0.0f, vh = 0.0f;
          if (te >= 0) {
            const int r = be * p.out_len + te - (tok0 - 3);  // 0 .. kFuTok + 2
            const uint32_t v = *reinterpret_cast<const uint32_t*>(sXw + r * 256 + 4 * lane);
            vl = __uint_as_float(v << 16);
            vh = __uint_as_float(v & 0xffff0000u);
          } else if (p.csi) {
            const long long base = (long long)be * p.csi_sb + (long long)c * p.csi_sd + W + te;
            vl = load_dyn(p.csi, base, p.csi_dtype);
            vh = load_dyn(p.csi, base + p.csi_sd, p.csi_dtype);
          }
          const long long ob = (long long)be * p.cso_sb + (long long)c * p.cso_sd + s2;
          store_dyn(p.cso, ob, p.cso_dtype, vl);
          store_dyn(p.cso, ob + p.cso_sd, p.cso_dtype, vh);
        }
      }
    }
  };
  if (!do_dt) {
    write_conv_state();
    return;
  }
  fu_lds_barrier();
  // ---- dt for channels c0 .. c0 + 127: tokens x 8 column tiles, K = r_pad ----
  f32x4 dacc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    if (ks * 32 < p.r_pad) {
      const bf16x8 av = *reinterpret_cast<const bf16x8*>(
          &sXD[(lane & 15) * kFuXdPitch + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        dacc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bw[i][ks], dacc[i], 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int ch = c0 + i * 16 + (lane & 15);
    if (ch < p.dim) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        sDT[((lane >> 4) * 4 + rr) * dtp + ch] = from_f32<bf16_t>(dacc[i][rr]);
    }
  }
  fu_lds_barrier();
  // 16 token rows x dim channels out, 16 B per lane-store
  const int q8 = p.dim >> 3;
  for (int i = tid; i < kFuTok * q8; i += blockDim.x) {
    const int t = i / q8, qd = i - t * q8;
    if (tok0 + t < ntok)
      *reinterpret_cast<uint4*>(p.dt + (long long)(tok0 + t) * p.dt_tl + qd * 8) =
          *reinterpret_cast<const uint4*>(&sDT[t * dtp + qd * 8]);
  }
  write_conv_state();
}

bool conv_proj_fused_ok(const ConvProjTmArgs& a) {
  // e_pad <= 80 (R + 2N <= 80, every VideoMamba size up to d_model 768): wider x_proj
  // outputs exceed the register budget of the 576-thread workgroup; buffer byte offsets
  // (x and u rows) must fit 31 bits
  const long long ntok = static_cast<long long>(a.batch) * a.out_len;
  return a.dim <= kFuMaxSpl * kSkCh && a.out_len >= 24 && a.e_pad <= 80 &&
         (a.e + 3) / 4 * 4 <= kSkMaxEp && (a.wdt == nullptr || a.r_pad <= 64) &&
         (ntok + 3) * a.x_tl * 2 < (1ll << 31) && (ntok + 3) * a.u_tl * 2 < (1ll << 31);
}

void conv_proj_fused_launch(const ConvProjTmArgs& a, hipStream_t s) {
  SkTmParams q{};
  q.a = a;
  q.part = nullptr;
  q.ntok = a.batch * a.out_len;
  q.nsplit = (a.dim + kSkCh - 1) / kSkCh;
  q.ep = (a.e + 3) / 4 * 4;
  const unsigned tiles = static_cast<unsigned>((q.ntok + kFuTok - 1) / kFuTok);
  constexpr int kUBytes = kFuMaxSpl * kFuTok * kFuUPitch * 2;
  constexpr int kPBytes = kFuMaxSpl * kFuTok * kSkMaxEp * 4;
  const size_t lds = static_cast<size_t>(kUBytes > kPBytes ? kUBytes : kPBytes) +
                     kFuTok * kFuXdPitch * 2 + kFuMaxSpl * kFuXRows * 256;
  static_assert(kFuTok * (kFuMaxSpl * kSkCh + 8) * 2 <= kPBytes, "dt tile exceeds the area");
  const dim3 grid(tiles), block(64 * q.nsplit);
  const bool cs32 = a.csi != nullptr && a.csi_dtype != VM_DTYPE_BF16;
  switch (a.e_pad / 16) {
#define VM_FU_CASE(NBV)                                                                    \
    case NBV:                                                                              \
      if (cs32) hipLaunchKernelGGL((conv_proj_fused_kernel<NBV, true>), grid, block, lds, s, q); \
      else hipLaunchKernelGGL((conv_proj_fused_kernel<NBV, false>), grid, block, lds, s, q);   \
      break;
    VM_FU_CASE(1) VM_FU_CASE(2) VM_FU_CASE(3) VM_FU_CASE(4) VM_FU_CASE(5)
#undef VM_FU_CASE
  }
}

long long conv_proj_sk_workspace_bytes(int batch, int out_len, int dim, int e) {
  if (batch <= 0 || out_len <= 0 || dim <= 0 || e <= 0) return 0;
  const long long ntok = 1LL * batch * out_len;
  const long long nsplit = (dim + kSkCh - 1) / kSkCh;
  return nsplit * ntok * ((e + 3) / 4 * 4) * static_cast<long long>(sizeof(float));
}

void conv_proj_sk_launch(const ConvProjTmArgs& a, float* part, hipStream_t s) {
  SkTmParams q{};
  q.a = a;
  q.part = part;
  q.ntok = a.batch * a.out_len;
  q.nsplit = (a.dim + kSkCh - 1) / kSkCh;
  q.ep = (a.e + 3) / 4 * 4;
  const unsigned tiles = static_cast<unsigned>((q.ntok + kCmTok - 1) / kCmTok);
  const size_t lds = static_cast<size_t>(72 + kCmTok + a.e_pad) * kTmPitch * sizeof(bf16_t) +
                    static_cast<size_t>(kSkCsRows) * 3 * kSkCh * sizeof(float);
  dim3 g1(tiles, q.nsplit);
  switch (a.e_pad / 16) {
#define VM_SK_CASE(NBV) \
    case NBV: hipLaunchKernelGGL(conv_xproj_tm_kernel<NBV>, g1, dim3(256), lds, s, q); break;
    VM_SK_CASE(1) VM_SK_CASE(2) VM_SK_CASE(3) VM_SK_CASE(4)
    VM_SK_CASE(5) VM_SK_CASE(6) VM_SK_CASE(7) VM_SK_CASE(8)
#undef VM_SK_CASE
  }
  conv_proj_sk_reduce_launch(a, part, s);
}

// The split-K form's second kernel alone: x_dbl from the partials, dt_proj (a.wdt) — also
// the tail of vm_in_proj_conv_proj_fwd, whose in_proj epilogue writes the same partials.
void conv_proj_sk_reduce_launch(const ConvProjTmArgs& a, float* part, hipStream_t s) {
  SkTmParams q{};
  q.a = a;
  q.part = part;
  q.ntok = a.batch * a.out_len;
  q.nsplit = (a.dim + kSkCh - 1) / kSkCh;
  q.ep = (a.e + 3) / 4 * 4;
  const unsigned tiles = static_cast<unsigned>((q.ntok + kCmTok - 1) / kCmTok);
  const unsigned cblocks = a.wdt ? static_cast<unsigned>((a.dim + 127) / 128) : 1u;
  const dim3 g2(tiles, cblocks);
  switch (q.nsplit) {
#define VM_SK2(NS) case NS: hipLaunchKernelGGL(xdbl_dt_tm_kernel<NS>, g2, dim3(256), 0, s, q); break;
    VM_SK2(1) VM_SK2(2) VM_SK2(3) VM_SK2(4) VM_SK2(5) VM_SK2(6) VM_SK2(7) VM_SK2(8)
    VM_SK2(9) VM_SK2(10) VM_SK2(11) VM_SK2(12) VM_SK2(13) VM_SK2(14) VM_SK2(15) VM_SK2(16)
#undef VM_SK2
  }
}

// Split count: a FIXED channel split (128 channels per split) so the x_proj reduction order,
// and with it every token's x_dbl bits, never depends on the token count — a chunk-
// dependent split (more splits for shorter sequences) broke chunked == full bitwise.
// At B = 1 (3,144 tokens, D = 1152) that is 49 x 9 = 441 workgroups.
constexpr int kCmSplitCh = 128;
static int cm_splits(int ntok, int dim) {
  (void)ntok;
  return (dim + kCmSplitCh - 1) / kCmSplitCh;
}

}  // namespace vm

using namespace vm;

extern "C" long long vm_conv_proj_cm_workspace_bytes(int batch, int out_len, int dim, int e) {
  if (batch <= 0 || out_len <= 0 || dim <= 0 || dim % 64 != 0 || e <= 0) return 0;
  const int ntok = batch * out_len;
  return static_cast<long long>(cm_splits(ntok, dim)) * e * ntok * sizeof(float);
}

extern "C" int vm_conv_proj_cm_fwd(const void* xz, long long x_sd,
                                   const float* conv_weight, const float* conv_bias,
                                   const void* cs_in, int cs_in_dtype, long long csi_sb, long long csi_sd,
                                   void* cs_out, int cs_out_dtype, long long cso_sb, long long cso_sd,
                                   const void* wx_pad, int e, int e_pad,
                                   const void* wdt_pad, int r, int r_pad,
                                   void* u, long long u_sd, void* xdbl, long long xd_sd,
                                   void* dt, long long dt_sd, int out_len, int batch, int dim,
                                   int seqlen, int width, void* workspace,
                                   long long workspace_bytes, vm_stream_t stream) {
  if (!xz || !conv_weight || !wx_pad || !wdt_pad || !u || !xdbl || !dt) {
    vmhost::set_error("vm_conv_proj_cm_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (batch < 0 || dim <= 0 || dim % 64 != 0 || seqlen < 1 || out_len < seqlen || out_len % 8 ||
      width < 1 || width > 4 || e < 1 || e_pad % 16 != 0 || e_pad < e || e_pad > 128 ||
      r < 1 || r > e || (r_pad != 32 && r_pad != 64) || r_pad < r ||
      (cs_in && !vmhost::dtype_ok(cs_in_dtype)) || (cs_out && !vmhost::dtype_ok(cs_out_dtype))) {
    vmhost::set_error("vm_conv_proj_cm_fwd: unsupported shape (dim %% 64 == 0, out_len %% 8 == 0, "
                      "width <= 4, R + 2N <= 128, R <= 64, seqlen >= 1)");
    return VM_E_INVALID;
  }
  if (!vmhost::aligned16(xz) || !vmhost::aligned16(u) || !vmhost::aligned16(wx_pad) ||
      !vmhost::aligned16(wdt_pad) || !vmhost::aligned16(dt) || x_sd % 8 || u_sd % 8 || dt_sd % 8) {
    vmhost::set_error("vm_conv_proj_cm_fwd: x / u / dt rows and the weights must be 16-byte aligned");
    return VM_E_INVALID;
  }
  if (cs_out && cs_in == cs_out) {
    vmhost::set_error("vm_conv_proj_cm_fwd: conv_state_out must not alias conv_state_in");
    return VM_E_INVALID;
  }
  if (batch == 0) return VM_OK;
  const long long need = vm_conv_proj_cm_workspace_bytes(batch, out_len, dim, e);
  if (!workspace || workspace_bytes < need) {
    vmhost::set_error("vm_conv_proj_cm_fwd: workspace of %lld bytes required", need);
    return VM_E_INVALID;
  }
  ConvProjCmParams p{};
  p.x = static_cast<const bf16_t*>(xz); p.cw = conv_weight; p.cb = conv_bias;
  p.csi = cs_in; p.cso = cs_out;
  p.wx = static_cast<const bf16_t*>(wx_pad); p.wdt = static_cast<const bf16_t*>(wdt_pad);
  p.u = static_cast<bf16_t*>(u); p.xdbl = static_cast<bf16_t*>(xdbl); p.dt = static_cast<bf16_t*>(dt);
  p.part = static_cast<float*>(workspace);
  p.x_sd = x_sd; p.u_sd = u_sd; p.xd_sd = xd_sd; p.dt_sd = dt_sd;
  p.csi_sb = csi_sb; p.csi_sd = csi_sd; p.cso_sb = cso_sb; p.cso_sd = cso_sd;
  p.batch = batch; p.dim = dim; p.seqlen = seqlen; p.lp = out_len; p.ntok = batch * out_len;
  p.e = e; p.e_pad = e_pad; p.r = r; p.r_pad = r_pad; p.width = width;
  p.csi_dtype = cs_in_dtype; p.cso_dtype = cs_out_dtype;
  p.nsplit = cm_splits(p.ntok, dim);
  p.split_ch = kCmSplitCh;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned tiles = static_cast<unsigned>((p.ntok + kCmTok - 1) / kCmTok);
  dim3 g1(tiles, p.nsplit);
  switch (e_pad / 16) {
#define VM_CM_CASE(NBV) \
    case NBV: hipLaunchKernelGGL(conv_xproj_cm_kernel<NBV>, g1, dim3(256), 0, st, p); break;
    VM_CM_CASE(1) VM_CM_CASE(2) VM_CM_CASE(3) VM_CM_CASE(4)
    VM_CM_CASE(5) VM_CM_CASE(6) VM_CM_CASE(7) VM_CM_CASE(8)
#undef VM_CM_CASE
  }
  hipLaunchKernelGGL(xdbl_dt_cm_kernel, dim3(tiles, (dim + 127) / 128), dim3(256), 0, st, p);
  if (cs_out)
    hipLaunchKernelGGL(conv_state_cm_kernel, dim3((dim + 255) / 256, batch), dim3(256), 0, st, p);
  return vmhost::launch_status("vm_conv_proj_cm_fwd");
}
