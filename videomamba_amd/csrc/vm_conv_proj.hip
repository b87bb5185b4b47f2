// Fused token-major mixer middle: depthwise causal conv1d + SiLU -> x_proj -> dt_proj.
//
// Replaces, for the token-major (large-batch) mixer, the three steps the reference runs
// between in_proj and the scan (models/videomamba/mamba_simple.py:381-416):
//     u     = silu(conv1d(x [+ conv_state]))            (causal_conv1d_fn)
//     x_dbl = u @ W_x^T                                   (x_proj, (R + 2N) outputs)
//     dt    = x_dbl[:, :R] @ W_dt^T                       (dt_proj weight; bias -> scan)
// with the reference's rounding points (u, x_dbl, dt in bf16; fp32 accumulation).
// Optionally (dt_softplus) the dt epilogue also applies the scan's delta activation,
//     delta = softplus(float(bf16(dt)) + dt_bias)  -> bf16,
// the reference's selective_scan_fn(delta_bias=..., delta_softplus=True) prologue
// (mamba_simple.py:109-172 / :30-106), so the scan streams a ready delta and spends no
// transcendentals on it: the activation moves into a kernel whose VALU sits idle behind
// its memory waits, and the scan (issue-bound) drops ~7 % per launch.
//
// One workgroup (4 waves) owns 64 token rows of the flattened (batch * Lp) axis and sweeps
// the channels in chunks of 64:
//   conv   : thread = (8 adjacent channels, 2 tokens); x rows t-3..t from L1/L2, state or
//            zeros before the sequence start; u written to HBM (16 B per thread-row) and to
//            an LDS A-tile [64 tokens][64 ch];
//   x_proj : wave w = tokens 16w..16w+15, all (R+2N) outputs, v_mfma_f32_16x16x32_bf16
//            with W_x's chunk staged in LDS (rows padded to a multiple of 16 with zeros);
// then x_dbl (bf16) is written and its first R columns (zero-padded to K = 32 or 64) form
// the A operand of dt_proj: wave w = output-column blocks w, w+4, ..., all 64 tokens,
// W_dt fragments straight from L2 (each read by one wave of the workgroup).
// HBM traffic per token: x row in, u / dt rows out (+ x_dbl): 3 * D * 2 + 2 * (R + 2N) B.

#include <stdlib.h>

#include "vm_conv_proj.h"

namespace vm {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

struct ConvProjParams {
  const bf16_t* xz; const float* cw; const float* cb;
  const void* csi; void* cso;
  const bf16_t* wx;   // (e_pad, D) zero-padded rows
  const bf16_t* wdt;  // (D, r_pad) zero-padded columns
  bf16_t* u; bf16_t* xdbl; bf16_t* dt;
  const float* dtb;  // dt bias (nullable), used with SPD
  long long xz_sb, xz_sl, csi_sb, csi_sd, cso_sb, cso_sd;
  long long u_sb, u_sl, xd_sb, xd_sl, dt_sb, dt_sl;
  int batch, dim, seqlen, lp, rows, e, e_pad, r, r_pad, width, csi_dtype, cso_dtype;
};

constexpr int kCPTok = 64;   // token rows per workgroup
constexpr int kCPCh = 64;    // channels per chunk
constexpr int kCPPad = 72;   // LDS row pitch (bf16): 144 B rows keep b128 reads conflict-light
constexpr int kCPMaxNB = 8;  // (R + 2N) <= 128

__device__ __forceinline__ void unpack8(const uint4& q, float (&v)[8]) {
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
// two floats -> packed bf16 pair in one v_cvt_pk_bf16_f32 (round to nearest even, as
// from_f32<bf16_t>)
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const bf16x2 h = __builtin_convertvector(f32x2{a, b}, bf16x2);
  return __builtin_bit_cast(uint32_t, h);
}
__device__ __forceinline__ float silu_f(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x * kLog2e));
}
// silu_f on a packed pair: the multiplies and the add as packed ops, the same values
__device__ __forceinline__ f32x2 silu2(f32x2 x) {
  const f32x2 t = x * f32x2{-kLog2e, -kLog2e};
  const f32x2 d = f32x2{1.0f, 1.0f} + f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

// dt epilogue: bf16 dt (the reference's rounding point), or with SPD the activated
// delta = softplus(float(bf16(dt)) + bias) rounded to bf16
// softplus(x) = log1p(e^x) with log1p by the u = 1 + w correction (exact where 1 + w
// rounds to 1, a few ulp elsewhere): unlike softplus_fast it keeps full relative precision
// for small deltas — affordable here, where the VALU waits on memory anyway.
__device__ __forceinline__ float softplus_acc(float x) {
  if (x > 20.0f) return x;
  const float w = __builtin_amdgcn_exp2f(x * kLog2e);
  const float u = 1.0f + w;
  const float d = u - 1.0f;
  return d == 0.0f ? w : __builtin_amdgcn_logf(u) * 0.6931471805599453f * (w * __builtin_amdgcn_rcpf(d));
}
template <bool SPD>
__device__ __forceinline__ bf16_t dt_out(float acc, float bias) {
  const bf16_t v = from_f32<bf16_t>(acc);
  if constexpr (SPD) return from_f32<bf16_t>(softplus_acc(to_f32(v) + bias));
  return v;
}

template <bool SPD>
__device__ __forceinline__ void dt_phase_half(const ConvProjParams& p, const bf16_t* sA,
                                              bf16_t* sU, int row0, int lane, int wave);

// LDS: sA [64][72] bf16 (u chunk, then x_dbl[:, :R]);  sU [4 waves][64][72] bf16 (W_x
// chunk during the sweep, then per-wave output staging);  dynamic: conv weights (D, 4)
// and bias (D) as fp32.
// EXP (tools/probes/cp_lab.hip only; 0 in the library) removes pieces to price them:
// 1 W_x staging loads, 2 x_proj MFMAs, 4 u stores, 8 conv window loads, 16 loop barriers.
// SPD: the dt epilogue emits softplus(dt + bias) (see the header)
template <bool DT, int NB, int EXP = 0, bool SPD = false>  // DT: also run dt_proj here; NB = e_pad / 16 blocks
// 3 waves per SIMD = the 3 workgroups per CU the LDS budget allows (unbounded, hipcc spends
// ~176 registers on the in-flight prefetch and runs 2)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
void conv_proj_kernel(const ConvProjParams p) {
  // sU: W_x chunk (<= 128 rows x kCPPad) / x_dbl tile (64 x 2*kCPPad); with DT also the
  // per-wave dt staging (4 x 64 x kCPPad)
  constexpr int kSU = 2 * kCPTok * kCPPad;  // with DT the dt staging is 4 waves x 32 rows
  __shared__ __attribute__((aligned(16))) bf16_t sA[kCPTok * kCPPad];
  __shared__ __attribute__((aligned(16))) bf16_t sU[kSU];
  extern __shared__ __attribute__((aligned(16))) float sW[];  // [D][4] taps, then [D] bias
  bf16_t* sB = sU;  // W_x chunk: e_pad (<= 128) rows of kCPPad
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int row0 = blockIdx.x * kCPTok;
  const int D = p.dim;

  // conv weights, right-aligned into 4 taps, and bias -> LDS; taps of a channel pair
  // interleaved ([pair][tap][2]) so each tap's pair is one packed operand
  for (int i = tid; i < D * 4; i += 256) {
    const int ch = i >> 2, tap = (i & 3) - (4 - p.width);
    sW[(ch >> 1) * 8 + (i & 3) * 2 + (ch & 1)] = tap >= 0 ? p.cw[ch * p.width + tap] : 0.0f;
  }
  for (int i = tid; i < D; i += 256) sW[4 * D + i] = p.cb ? p.cb[i] : 0.0f;

  // conv role: 8 channels x 2 adjacent token rows (same sequence: rows 2k, 2k+1 never
  // straddle a batch boundary because out_len is even)
  const int cg = tid & 7;
  const int tg = tid >> 3;
  const int rowa = row0 + 2 * tg;
  const bool rva = rowa < p.rows, rvb = rowa + 1 < p.rows;
  const int rr = rva ? rowa : p.rows - 1;
  const int b = rr / p.lp;
  const int ta = rr - b * p.lp;  // step of the first row; window rows ta-3 .. ta+1
  // Every load of the sweep is unconditional, so none sits behind a branch whose join makes
  // hipcc drain vmcnt: window rows outside [0, seqlen) read a clamped (valid) row and are
  // zeroed at use, W_x padding pieces re-read its last row into LDS rows nothing reads.
  // Round 2's per-row "load or zero" select and runtime-bound W_x staging loop compiled to
  // a load + vmcnt(0) round trip per piece, exposing the window prefetch and three W_x
  // latencies in every chunk.  Both are buffer loads: a per-lane 32-bit offset fixed for
  // the sweep plus the chunk's channel offset in a scalar register.
  // x window rows: the workgroup's 64 rows touch sequences b0 .. b0 + 63 / out_len + 1
  // (a row pair never straddles two: out_len is even); the host checks the offsets fit
  // 31 bits
  const int b0 = row0 / p.lp;
  const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.xz + (long long)b0 * p.xz_sb), 0,
                                                    0x7fffffff, 0x00020000);
  int woff[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int te = min(max(ta - 3 + j, 0), p.seqlen - 1);
    woff[j] = static_cast<int>(((long long)(b - b0) * p.xz_sb + (long long)te * p.xz_sl + cg * 8) * 2);
  }
  auto load_win = [&](int c0, uint4 (&w)[5]) {
#pragma unroll
    for (int j = 0; j < 5; ++j)
      w[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, woff[j], c0 * 2, 0));
  };
  unsigned win_ok = 0;  // bit j: window row ta - 3 + j lies in [0, seqlen)
#pragma unroll
  for (int j = 0; j < 5; ++j)
    if (ta - 3 + j >= 0 && ta - 3 + j < p.seqlen) win_ok |= 1u << j;
  // conv state (B, D, W) of fp32 or bf16 through one buffer resource (its size is checked
  // on the host to fit 31-bit offsets)
  const bool cs_bf16 = p.csi_dtype == VM_DTYPE_BF16;
  const auto csr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.csi), 0,
      p.csi ? static_cast<int>(((long long)(p.batch - 1) * p.csi_sb + (long long)(D - 1) * p.csi_sd + p.width) *
                               (cs_bf16 ? 2 : 4))
            : 0,
      0x00020000);
  auto cs_off = [](bool ok, int off) {
    off = ok ? off : 0x7ffffff0;  // past the range: the load reads 0
    asm volatile("" : "+v"(off));  // keep it a select (seen through, hipcc branches per load)
    return off;
  };
  // W_x chunk [e_pad][64] as 16-B pieces, loaded one chunk ahead into registers and
  // written to LDS after the previous chunk's MFMAs
  constexpr int kWxIt = (NB * 128 + 255) / 256;
  uint4 wreg[kWxIt];
  const auto wxr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.wx), 0,
                                                     NB * 16 * D * 2, 0x00020000);
  int xoff[kWxIt];
#pragma unroll
  for (int i = 0; i < kWxIt; ++i) {
    const int idx = tid + 256 * i;
    xoff[i] = (min(idx >> 3, NB * 16 - 1) * D + (idx & 7) * 8) * 2;
  }
  auto load_wx = [&](int c0) {
#pragma unroll
    for (int i = 0; i < kWxIt; ++i)
      wreg[i] = (EXP & 1) ? make_uint4(i, c0, 0, 0)
                          : __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wxr, xoff[i], c0 * 2, 0));
  };

  // u rows of this workgroup (the range ends at the last valid row): the stores need no
  // branch, so the counted wait for the window prefetch at the end of a chunk can leave
  // them in flight
  const auto ur = __builtin_amdgcn_make_buffer_rsrc(
      p.u + (long long)row0 * p.u_sl, 0, static_cast<int>(min(kCPTok, p.rows - row0) * p.u_sl * 2),
      0x00020000);
  const int u_row = static_cast<int>(p.u_sl * 2);
  const int uoff = (2 * tg * static_cast<int>(p.u_sl) + cg * 8) * 2;

  f32x4 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 wa[5], wb[5];
  load_wx(0);
  load_win(0, wa);
  __syncthreads();  // sW ready
  // one 64-channel chunk; cur holds its window rows, nxt receives the next chunk's
  auto chunk = [&](int c0, uint4 (&cur)[5], uint4 (&nxt)[5]) {
    const int c = c0 + cg * 8;
    // ---- stage W_x[:, c0:c0+64] (rows < 128 <= kSU / kCPPad) ----
#pragma unroll
    for (int i = 0; i < kWxIt; ++i) {
      const int idx = tid + 256 * i;
      *reinterpret_cast<uint4*>(&sB[(idx >> 3) * kCPPad + (idx & 7) * 8]) = wreg[i];
    }
    // prefetch the next chunk (the last chunk re-reads its own: cache hits, no branch)
    const int cn = min(c0 + kCPCh, D - kCPCh);
    load_wx(cn);
    if (!(EXP & 8)) load_win(cn, nxt);
#pragma unroll
    for (int j = 0; j < 5; ++j) {  // zero rows outside the sequence (a mask, not a branch)
      const uint32_t m = 0u - ((win_ok >> j) & 1u);
      cur[j].x &= m; cur[j].y &= m; cur[j].z &= m; cur[j].w &= m;
    }
    // ---- conv + silu, one channel pair (one packed word of each window row) at a time ----
    if (ta < 3 && p.csi) {  // window reaches before the sequence start: conv state
      // rows te < 0 of the window are zero here; the state taps are OR-ed in, each a buffer
      // load whose offset is out of range (reads 0) where the row needs none: no branch
      // inside this (rare) one, a row's 8 loads issued together
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int te = ta - 3 + j;
        const int sj = p.width + te;
        const bool ok = te < 0 && sj >= 0;
        const int base = b * (int)p.csi_sb + c * (int)p.csi_sd + sj;
        uint32_t pk[4];
        if (cs_bf16) {
          uint32_t h[8];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            h[k] = __builtin_amdgcn_raw_buffer_load_b16(csr, cs_off(ok, (base + k * (int)p.csi_sd) * 2), 0, 0);
#pragma unroll
          for (int k = 0; k < 4; ++k) pk[k] = h[2 * k] | (h[2 * k + 1] << 16);
        } else {
          float sv[8];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            sv[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(csr, cs_off(ok, (base + k * (int)p.csi_sd) * 4), 0, 0));
#pragma unroll
          for (int k = 0; k < 4; ++k) pk[k] = pack2(sv[2 * k], sv[2 * k + 1]);
        }
        cur[j].x |= pk[0]; cur[j].y |= pk[1]; cur[j].z |= pk[2]; cur[j].w |= pk[3];
      }
    }
    const bool la = rva && ta < p.seqlen, lb = rvb && ta + 1 < p.seqlen;
    uint32_t pa[4], pb[4];
    // channel pairs (ch, ch + 1) as packed fp32 pairs: v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32
    // do per lane exactly what the scalar fmaf / * / + did (same taps in the same order, one
    // rounding each), at about 5.3 instead of 2 x 4 issue cycles — the conv + SiLU VALU
    // stream is most of this kernel's non-memory time
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x2 xv[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const uint32_t wd = q == 0 ? cur[j].x : q == 1 ? cur[j].y : q == 2 ? cur[j].z : cur[j].w;
        xv[j] = f32x2{__uint_as_float(wd << 16), __uint_as_float(wd & 0xffff0000u)};
      }
      const int ch = c + 2 * q;  // even
      const float4 t01 = *reinterpret_cast<const float4*>(&sW[ch * 4]);
      const float4 t23 = *reinterpret_cast<const float4*>(&sW[ch * 4 + 4]);
      const f32x2 bias2 = *reinterpret_cast<const f32x2*>(&sW[4 * D + ch]);
      const f32x2 w0 = f32x2{t01.x, t01.y}, w1 = f32x2{t01.z, t01.w}, w2 = f32x2{t23.x, t23.y},
                  w3 = f32x2{t23.z, t23.w};
      f32x2 ya = __builtin_elementwise_fma(w0, xv[0], bias2);
      f32x2 yb = __builtin_elementwise_fma(w0, xv[1], bias2);
      ya = __builtin_elementwise_fma(w1, xv[1], ya);
      yb = __builtin_elementwise_fma(w1, xv[2], yb);
      ya = __builtin_elementwise_fma(w2, xv[2], ya);
      yb = __builtin_elementwise_fma(w2, xv[3], yb);
      ya = __builtin_elementwise_fma(w3, xv[3], ya);
      yb = __builtin_elementwise_fma(w3, xv[4], yb);
      const f32x2 sa = silu2(ya), sb = silu2(yb);
      pa[q] = pack2(la ? sa.x : 0.f, la ? sa.y : 0.f);
      pb[q] = pack2(lb ? sb.x : 0.f, lb ? sb.y : 0.f);
    }
    const uint4 qa = make_uint4(pa[0], pa[1], pa[2], pa[3]);
    const uint4 qb = make_uint4(pb[0], pb[1], pb[2], pb[3]);
    if (!(EXP & 4)) {  // unconditional: rows past the end fall outside ur's range
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, qa), ur, uoff + c0 * 2, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, qb), ur, uoff + c0 * 2 + u_row, 0, 0);
    }
    *reinterpret_cast<uint4*>(&sA[(2 * tg) * kCPPad + cg * 8]) = qa;
    *reinterpret_cast<uint4*>(&sA[(2 * tg + 1) * kCPPad + cg * 8]) = qb;
    if (!(EXP & 16)) __syncthreads();
    // ---- x_proj MFMA: wave's 16 tokens x all e_pad outputs, K = 64 ----
#pragma unroll
    for (int ks = 0; ks < ((EXP & 2) ? 0 : 2); ++ks) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(
          &sA[(wave * 16 + (lane & 15)) * kCPPad + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(
            &sB[(j * 16 + (lane & 15)) * kCPPad + ks * 32 + (lane >> 4) * 8]);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bv, acc[j], 0, 0, 0);
      }
    }
    if (!(EXP & 16)) __syncthreads();
  };
  // (a two-chunk trip with the window buffers swapping roles saves the copy below but needs
  // ~220 registers: 2 waves per SIMD instead of 3)
  for (int c0 = 0; c0 < D; c0 += kCPCh) {
    chunk(c0, wa, wb);
#pragma unroll
    for (int j = 0; j < 5; ++j) wa[j] = wb[j];
  }

  // ---- x_dbl: bf16 tile [64][e_pad] in sU (stride kCPPad*2), x_dbl[:, :R] -> sA ----
  bf16_t* sX = sU;  // [64][2 * kCPPad] (e_pad <= 128 < 144)
  for (int idx = tid; idx < kCPTok * kCPPad / 8; idx += 256)
    *reinterpret_cast<uint4*>(&sA[idx * 8]) = make_uint4(0, 0, 0, 0);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int n = j * 16 + (lane & 15);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int lr = wave * 16 + (lane >> 4) * 4 + e;
      const bf16_t v = from_f32<bf16_t>(acc[j][e]);
      sX[lr * 2 * kCPPad + n] = v;
      if (n < p.r) sA[lr * kCPPad + n] = v;
    }
  }
  __syncthreads();
  // coalesced x_dbl rows: e (even) bf16 per row, 4-byte pieces
  {
    const int pieces = p.e / 2;
    for (int idx = tid; idx < kCPTok * pieces; idx += 256) {
      const int lr = idx / pieces, q = idx - lr * pieces;
      const int row = row0 + lr;
      if (row < p.rows)
        *reinterpret_cast<uint32_t*>(p.xdbl + (long long)row * p.xd_sl + 2 * q) =
            *reinterpret_cast<const uint32_t*>(&sX[lr * 2 * kCPPad + 2 * q]);
    }
  }
  if constexpr (DT) {
    __syncthreads();  // sU is reused below as per-wave output staging
    dt_phase_half<SPD>(p, sA, sU, row0, lane, wave);
  }
}

// dt_proj inside conv_proj (DT): wave = 64-column blocks wave, wave+4, ...; each block in
// two 32-row halves, so the per-wave staging is 32 rows and the fused kernel keeps conv_proj's LDS
// budget (3 workgroups per CU) and half the accumulators.
template <bool SPD>
__device__ __forceinline__ void dt_phase_half(const ConvProjParams& p, const bf16_t* sA,
                                              bf16_t* sU, int row0, int lane, int wave) {
  const int D = p.dim;
  const int ksteps = p.r_pad / 32;
  bf16_t* stg = sU + wave * 32 * kCPPad;
  for (int cb = wave; cb * 64 < D; cb += 4) {
    float bj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bj[j] = SPD && p.dtb ? p.dtb[cb * 64 + j * 16 + (lane & 15)] : 0.0f;
    bf16x8 bw[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        if (ks < ksteps)
          bw[j][ks] = *reinterpret_cast<const bf16x8*>(
              p.wdt + (long long)(cb * 64 + j * 16 + (lane & 15)) * p.r_pad + ks * 32 +
              (lane >> 4) * 8);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x4 d[2][4];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) d[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (ks < ksteps) {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(
                &sA[((2 * h + i) * 16 + (lane & 15)) * kCPPad + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
              d[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[j][ks], d[i][j], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            stg[(i * 16 + (lane >> 4) * 4 + e) * kCPPad + j * 16 + (lane & 15)] =
                dt_out<SPD>(d[i][j][e], bj[j]);
      // 32 rows x 128 B out, 16 B per lane-store
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int lr = it * 8 + (lane >> 3), q = lane & 7;
        const int row = row0 + h * 32 + lr;
        const uint4 val = *reinterpret_cast<const uint4*>(&stg[lr * kCPPad + q * 8]);
        if (row < p.rows)
          *reinterpret_cast<uint4*>(p.dt + (long long)row * p.dt_sl + cb * 64 + q * 8) = val;
      }
    }
  }
}

// New conv state (B, D, width): the last `width` raw inputs of each channel — steps
// L-width .. L-1 of x, or of the old state for steps before the sequence start
// (mamba_simple.py:383-399). Its own small launch keeps the chunk loop of conv_proj_kernel
// free of the one-row-per-sequence branch that held a workgroup per sequence back.
__global__ __launch_bounds__(256) void conv_state_out_kernel(const ConvProjParams p) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (c >= p.dim) return;
  const bf16_t* xrow = p.xz + b * p.xz_sb;
  for (int s = 0; s < p.width; ++s) {
    const int te = p.seqlen - p.width + s;
    float val = 0.0f;
    if (te >= 0) val = to_f32(xrow[(long long)te * p.xz_sl + c]);
    else if (p.csi) val = load_dyn(p.csi, b * p.csi_sb + (long long)c * p.csi_sd + p.width + te,
                                   p.csi_dtype);
    store_dyn(p.cso, b * p.cso_sb + (long long)c * p.cso_sd + s, p.cso_dtype, val);
  }
}

}  // namespace vm

using namespace vm;

extern "C" long long vm_conv_proj_workspace_bytes(int batch, int out_len, int dim, int e) {
  if (batch > kSkMaxBatch) return 0;
  return conv_proj_sk_workspace_bytes(batch, out_len, dim, e);
}

// Which form vm_conv_proj_fwd runs (the split-K / fused small-batch form for batch <=
// kSkMaxBatch, else the wide kernel), and whether the wide kernel's 31-bit buffer offsets
// cover the operands: the x rows of the sequences one workgroup's 64 rows touch, the conv
// state, the u rows.  Shared by the launcher and the host query vm_conv_proj_fits.
static bool conv_proj_small_form(int batch, int dim, int e, int r_pad, int spd, int out_len) {
  return batch <= kSkMaxBatch && !spd && dim <= 2048 && (e + 3) / 4 * 4 <= kSkMaxEp &&
         r_pad <= 80 && out_len >= 8;
}
static bool conv_proj_wide_offsets_ok(int batch, int out_len, int seqlen, int dim,
                                      long long xz_sb, long long xz_sl, bool has_cs_in,
                                      int cs_in_dtype, long long csi_sb, long long csi_sd,
                                      int width, long long u_sl) {
  constexpr long long kOff31 = 0x7fffff00LL;
  const int cs_es = has_cs_in && cs_in_dtype == VM_DTYPE_BF16 ? 2 : 4;
  return ((long long)(kCPTok / out_len + 1) * xz_sb + (long long)seqlen * xz_sl + dim) * 2 <=
             kOff31 &&
         (!has_cs_in ||
          ((long long)(batch - 1) * csi_sb + (long long)(dim - 1) * csi_sd + width) * cs_es <=
              kOff31) &&
         (long long)kCPTok * u_sl * 2 <= kOff31;
}

extern "C" int vm_conv_proj_fits(int batch, int out_len, int seqlen, int dim, int e, int r_pad,
                                 int dt_softplus, long long xz_sb, long long xz_sl,
                                 int has_conv_state_in, int cs_in_dtype, long long csi_sb,
                                 long long csi_sd, int width, long long u_sl) {
  if (batch <= 0 || out_len <= 0) return 1;
  if (conv_proj_small_form(batch, dim, e, r_pad, dt_softplus != 0, out_len)) return 1;
  return conv_proj_wide_offsets_ok(batch, out_len, seqlen, dim, xz_sb, xz_sl,
                                   has_conv_state_in != 0, cs_in_dtype, csi_sb, csi_sd, width,
                                   u_sl)
             ? 1
             : 0;
}

extern "C" int vm_conv_proj_fwd(const void* xz, long long xz_sb, long long xz_sl,
                                const float* conv_weight, const float* conv_bias,
                                const void* cs_in, int cs_in_dtype, long long csi_sb, long long csi_sd,
                                void* cs_out, int cs_out_dtype, long long cso_sb, long long cso_sd,
                                const void* wx_pad, int e, int e_pad,
                                const void* wdt_pad, int r, int r_pad,
                                void* u, long long u_sb, long long u_sl,
                                void* xdbl, long long xd_sb, long long xd_sl,
                                void* dt, long long dt_sb, long long dt_sl,
                                const float* dt_bias, int dt_softplus, int out_len, int batch, int dim, int seqlen, int width, int dtype,
                                void* workspace, long long workspace_bytes, vm_stream_t stream) {
  if (!xz || !conv_weight || !wx_pad || !u || !xdbl || (dt && !wdt_pad)) {
    vmhost::set_error("vm_conv_proj_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (dtype != VM_DTYPE_BF16 || batch < 0 || dim <= 0 || dim % kCPCh != 0 || seqlen < 1 ||
      out_len < seqlen || width < 1 || width > 4 || e < 1 || e_pad % 16 != 0 || e_pad < e ||
      e_pad > kCPMaxNB * 16 || r < 1 || r > e || (dt && ((r_pad != 32 && r_pad != 64) || r_pad < r)) ||
      (cs_in && !vmhost::dtype_ok(cs_in_dtype)) || (cs_out && !vmhost::dtype_ok(cs_out_dtype))) {
    vmhost::set_error("vm_conv_proj_fwd: unsupported shape (bf16, dim %% 64 == 0, width <= 4, "
                      "R + 2N <= 128, R <= 64, seqlen >= 1)");
    return VM_E_INVALID;
  }
  if (!vmhost::aligned16(xz) || !vmhost::aligned16(u) || !vmhost::aligned16(wx_pad) ||
      (dt && !vmhost::aligned16(wdt_pad)) || (dt && !vmhost::aligned16(dt)) || xz_sb % 8 || xz_sl % 8 ||
      u_sb % 8 || u_sl % 8 || dt_sl % 8 || out_len % 2 || e % 2 || xd_sl % 2 ||
      (reinterpret_cast<uintptr_t>(xdbl) & 3) || dim > 8192) {
    vmhost::set_error("vm_conv_proj_fwd: xz / u / dt / weights need 16-byte aligned rows, "
                      "x_dbl 4-byte aligned, even out_len and e, dim <= 8192");
    return VM_E_INVALID;
  }
  if (u_sb != out_len * u_sl || xd_sb != out_len * xd_sl || (dt && dt_sb != out_len * dt_sl)) {
    vmhost::set_error("vm_conv_proj_fwd: u / x_dbl / dt must be batch-contiguous "
                      "(sb == out_len * sl)");
    return VM_E_INVALID;
  }
  if (cs_out && cs_in == cs_out) {
    vmhost::set_error("vm_conv_proj_fwd: conv_state_out must not alias conv_state_in");
    return VM_E_INVALID;
  }
  if (batch == 0) return VM_OK;
  ConvProjParams p{};
  p.xz = static_cast<const bf16_t*>(xz); p.cw = conv_weight; p.cb = conv_bias;
  p.csi = cs_in; p.cso = cs_out;
  p.wx = static_cast<const bf16_t*>(wx_pad); p.wdt = static_cast<const bf16_t*>(wdt_pad);
  p.u = static_cast<bf16_t*>(u); p.xdbl = static_cast<bf16_t*>(xdbl);
  p.dt = static_cast<bf16_t*>(dt);
  p.dtb = dt_bias;
  p.xz_sb = xz_sb; p.xz_sl = xz_sl; p.csi_sb = csi_sb; p.csi_sd = csi_sd;
  p.cso_sb = cso_sb; p.cso_sd = cso_sd;
  p.u_sb = u_sb; p.u_sl = u_sl; p.xd_sb = xd_sb; p.xd_sl = xd_sl; p.dt_sb = dt_sb; p.dt_sl = dt_sl;
  p.batch = batch; p.dim = dim; p.seqlen = seqlen; p.lp = out_len;
  p.rows = batch * out_len; p.e = e; p.e_pad = e_pad; p.r = r; p.r_pad = r_pad;
  p.width = width; p.csi_dtype = cs_in_dtype; p.cso_dtype = cs_out_dtype;
  dim3 grid((p.rows + kCPTok - 1) / kCPTok);
  const size_t lds = static_cast<size_t>(dim) * 5 * sizeof(float);
  hipStream_t st = static_cast<hipStream_t>(stream);
  // dt_proj runs inside conv_proj (half-tile dt phase, same LDS budget); dt == nullptr
  // skips it (conv + x_proj only: a consumer that projects dt itself)
  const bool fused_dt = dt != nullptr;
  const bool spd = dt_softplus != 0;
  if (conv_proj_small_form(batch, dim, e, r_pad, spd, out_len)) {
    // small batch: the split-K form (vm_conv_proj_sk.hip) fills the chip and keeps the
    // x_proj reduction order fixed per token
    const long long need = conv_proj_sk_workspace_bytes(batch, out_len, dim, e);
    if (!workspace || workspace_bytes < need) {
      vmhost::set_error("vm_conv_proj_fwd: batch <= %d needs a workspace of %lld bytes "
                        "(vm_conv_proj_workspace_bytes)", kSkMaxBatch, need);
      return VM_E_INVALID;
    }
    ConvProjTmArgs a{};
    a.x = p.xz; a.x_tl = xz_sl; a.cw = conv_weight; a.cb = conv_bias;
    a.csi = cs_in; a.csi_dtype = cs_in_dtype; a.csi_sb = csi_sb; a.csi_sd = csi_sd;
    a.cso = cs_out; a.cso_dtype = cs_out_dtype; a.cso_sb = cso_sb; a.cso_sd = cso_sd;
    a.wx = p.wx; a.e = e; a.e_pad = e_pad; a.wdt = fused_dt ? p.wdt : nullptr; a.r = r;
    a.r_pad = r_pad; a.u = p.u; a.u_tl = u_sl; a.xdbl = p.xdbl; a.xd_tl = xd_sl; a.dt = p.dt;
    a.dt_tl = dt_sl; a.out_len = out_len; a.batch = batch; a.dim = dim; a.seqlen = seqlen;
    a.width = width;
    // one fused launch where it applies (bit-identical), else the two split-K launches;
    // both write the conv state
    if (conv_proj_fused_ok(a)) conv_proj_fused_launch(a, st);
    else conv_proj_sk_launch(a, static_cast<float*>(workspace), st);
    return vmhost::launch_status("vm_conv_proj_fwd");
  }
  if (!conv_proj_wide_offsets_ok(batch, out_len, seqlen, dim, xz_sb, xz_sl, cs_in != nullptr,
                                 cs_in_dtype, csi_sb, csi_sd, width, u_sl)) {
    vmhost::set_error("vm_conv_proj_fwd: batch > %d needs a sequence of xz under 1 GiB "
                      "(31-bit buffer offsets)", kSkMaxBatch);
    return VM_E_INVALID;
  }
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, p); };
  switch (e_pad / 16) {  // x_proj output blocks
#define VM_CP_CASE(NBV)                                              \
    case NBV:                                                        \
      if (fused_dt && spd) go(conv_proj_kernel<true, NBV, 0, true>); \
      else if (fused_dt) go(conv_proj_kernel<true, NBV>);            \
      else go(conv_proj_kernel<false, NBV>);                         \
      break;
    VM_CP_CASE(1) VM_CP_CASE(2) VM_CP_CASE(3) VM_CP_CASE(4)
    VM_CP_CASE(5) VM_CP_CASE(6) VM_CP_CASE(7) VM_CP_CASE(8)
#undef VM_CP_CASE
  }
  if (cs_out)
    hipLaunchKernelGGL(conv_state_out_kernel, dim3((dim + 255) / 256, batch), dim3(256), 0, st, p);
  return vmhost::launch_status("vm_conv_proj_fwd");
}
