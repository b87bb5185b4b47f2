// Fused token-major mixer middle: depthwise causal conv1d + SiLU -> x_proj -> dt_proj.
//
// Replaces, for the token-major (large-batch) mixer, the three steps the reference runs
// between in_proj and the scan (models/videomamba/mamba_simple.py:381-416):
//     u     = silu(conv1d(x [+ conv_state]))            (causal_conv1d_fn)
//     x_dbl = u @ W_x^T                                   (x_proj, (R + 2N) outputs)
//     dt    = x_dbl[:, :R] @ W_dt^T                       (dt_proj weight; bias -> scan)
// with the reference's rounding points (u, x_dbl, dt in bf16; fp32 accumulation).
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

#include "vm_common.h"

namespace vm {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct ConvProjParams {
  const bf16_t* xz; const float* cw; const float* cb;
  const void* csi; void* cso;
  const bf16_t* wx;   // (e_pad, D) zero-padded rows
  const bf16_t* wdt;  // (D, r_pad) zero-padded columns
  bf16_t* u; bf16_t* xdbl; bf16_t* dt;
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

__global__ __launch_bounds__(256) void conv_proj_kernel(const ConvProjParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t sA[kCPTok * kCPPad];
  __shared__ __attribute__((aligned(16))) bf16_t sB[kCPMaxNB * 16 * kCPPad];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int row0 = blockIdx.x * kCPTok;
  const int nb = p.e_pad / 16;

  // conv role: 8 channels x 2 token rows
  const int cg = tid & 7;
  const int tg = tid >> 3;
  int tb[2], tt[2];
  bool rv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = row0 + 2 * tg + i;
    rv[i] = row < p.rows;
    const int rr = rv[i] ? row : p.rows - 1;
    tb[i] = rr / p.lp;
    tt[i] = rr - tb[i] * p.lp;
  }

  f32x4 acc[kCPMaxNB];
#pragma unroll
  for (int j = 0; j < kCPMaxNB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = 0; c0 < p.dim; c0 += kCPCh) {
    // ---- stage W_x[:, c0:c0+64] (e_pad rows x 128 B) ----
    for (int idx = tid; idx < p.e_pad * 8; idx += 256) {
      const int n = idx >> 3, q = idx & 7;
      *reinterpret_cast<uint4*>(&sB[n * kCPPad + q * 8]) =
          *reinterpret_cast<const uint4*>(p.wx + (long long)n * p.dim + c0 + q * 8);
    }
    // ---- conv + silu for (2 tokens) x (8 channels) ----
    const int c = c0 + cg * 8;
    float w[4][8], bias[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int ch = c + k;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int tap = i - (4 - p.width);  // right-aligned taps
        w[i][k] = tap >= 0 ? p.cw[ch * p.width + tap] : 0.0f;
      }
      bias[k] = p.cb ? p.cb[ch] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int b = tb[i], t = tt[i];
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = bias[k];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int te = t - 3 + j;
        float v[8];
        if (te >= 0 && te < p.seqlen) {
          const uint4 q = *reinterpret_cast<const uint4*>(p.xz + b * p.xz_sb + te * p.xz_sl + c);
          unpack8(q, v);
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int sj = p.width + te;  // state column of virtual step te < 0
            v[k] = (te < 0 && p.csi && sj >= 0)
                       ? load_dyn(p.csi, b * p.csi_sb + (long long)(c + k) * p.csi_sd + sj,
                                  p.csi_dtype)
                       : 0.0f;
          }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = fmaf(w[j][k], v[k], o[k]);
      }
      const bool live = rv[i] && t < p.seqlen;
      uint32_t packed[4];
#pragma unroll
      for (int k = 0; k < 8; k += 2) {
        const float a0 = live ? silu(o[k]) : 0.0f;
        const float a1 = live ? silu(o[k + 1]) : 0.0f;
        packed[k / 2] = static_cast<uint32_t>(from_f32<bf16_t>(a0)) |
                        (static_cast<uint32_t>(from_f32<bf16_t>(a1)) << 16);
      }
      const uint4 pq = make_uint4(packed[0], packed[1], packed[2], packed[3]);
      if (rv[i]) *reinterpret_cast<uint4*>(p.u + (long long)(row0 + 2 * tg + i) * p.u_sl + c) = pq;
      *reinterpret_cast<uint4*>(&sA[(2 * tg + i) * kCPPad + cg * 8]) = pq;
      // new conv state: the last `width` raw inputs, from the row holding step L-1
      if (p.cso && live && t == p.seqlen - 1) {  // one row per sequence: reload
        for (int k = 0; k < 8; ++k)
          for (int s = 0; s < p.width; ++s) {
            const int te = t - p.width + 1 + s;
            float v = 0.0f;
            if (te >= 0) v = to_f32(p.xz[b * p.xz_sb + te * p.xz_sl + c + k]);
            else if (p.csi) v = load_dyn(p.csi, b * p.csi_sb + (long long)(c + k) * p.csi_sd +
                                                    p.width + te, p.csi_dtype);
            store_dyn(p.cso, b * p.cso_sb + (long long)(c + k) * p.cso_sd + s, p.cso_dtype, v);
          }
      }
    }
    __syncthreads();
    // ---- x_proj MFMA: wave's 16 tokens x all e_pad outputs, K = 64 ----
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(
          &sA[(wave * 16 + (lane & 15)) * kCPPad + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
      for (int j = 0; j < kCPMaxNB; ++j) {
        if (j < nb) {
          const bf16x8 bv = *reinterpret_cast<const bf16x8*>(
              &sB[(j * 16 + (lane & 15)) * kCPPad + ks * 32 + (lane >> 4) * 8]);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bv, acc[j], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }

  // ---- x_dbl: round to bf16, store, and stage x_dbl[:, :R] (zero-padded) as dt's A ----
  for (int idx = tid; idx < kCPTok * kCPPad / 8; idx += 256)
    *reinterpret_cast<uint4*>(&sA[idx * 8]) = make_uint4(0, 0, 0, 0);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kCPMaxNB; ++j) {
    if (j < nb) {
      const int n = j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int lr = wave * 16 + (lane >> 4) * 4 + e;
        const int row = row0 + lr;
        const bf16_t v = from_f32<bf16_t>(acc[j][e]);
        if (n < p.e && row < p.rows) p.xdbl[(long long)row * p.xd_sl + n] = v;
        if (n < p.r) sA[lr * kCPPad + n] = v;
      }
    }
  }
  __syncthreads();

  // ---- dt_proj MFMA: wave = column blocks wave, wave+4, ...; all 64 tokens ----
  const int ksteps = p.r_pad / 32;
  bf16x8 af[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      af[i][ks] = *reinterpret_cast<const bf16x8*>(
          &sA[(i * 16 + (lane & 15)) * kCPPad + ks * 32 + (lane >> 4) * 8]);
  const int rbase = row0 + (lane >> 4) * 4;  // + i * 16 + e
  bf16_t* __restrict__ dtp = p.dt + (long long)rbase * p.dt_sl;
  for (int nblk = wave; nblk * 16 < p.dim; nblk += 4) {
    const int n = nblk * 16 + (lane & 15);
    bf16x8 bf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      bf[ks] = ks < ksteps ? *reinterpret_cast<const bf16x8*>(
                                 p.wdt + (long long)n * p.r_pad + ks * 32 + (lane >> 4) * 8)
                           : bf16x8{};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        if (ks < ksteps) d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf[ks], d, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (rbase + i * 16 + e < p.rows)
          dtp[(long long)(i * 16 + e) * p.dt_sl + n] = from_f32<bf16_t>(d[e]);
    }
  }
}

}  // namespace vm

using namespace vm;

extern "C" int vm_conv_proj_fwd(const void* xz, long long xz_sb, long long xz_sl,
                                const float* conv_weight, const float* conv_bias,
                                const void* cs_in, int cs_in_dtype, long long csi_sb, long long csi_sd,
                                void* cs_out, int cs_out_dtype, long long cso_sb, long long cso_sd,
                                const void* wx_pad, int e, int e_pad,
                                const void* wdt_pad, int r, int r_pad,
                                void* u, long long u_sb, long long u_sl,
                                void* xdbl, long long xd_sb, long long xd_sl,
                                void* dt, long long dt_sb, long long dt_sl,
                                int out_len, int batch, int dim, int seqlen, int width, int dtype,
                                vm_stream_t stream) {
  if (!xz || !conv_weight || !wx_pad || !wdt_pad || !u || !xdbl || !dt) {
    vmhost::set_error("vm_conv_proj_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (dtype != VM_DTYPE_BF16 || batch < 0 || dim <= 0 || dim % kCPCh != 0 || seqlen < 1 ||
      out_len < seqlen || width < 1 || width > 4 || e < 1 || e_pad % 16 != 0 || e_pad < e ||
      e_pad > kCPMaxNB * 16 || r < 1 || r > e || (r_pad != 32 && r_pad != 64) || r_pad < r ||
      (cs_in && !vmhost::dtype_ok(cs_in_dtype)) || (cs_out && !vmhost::dtype_ok(cs_out_dtype))) {
    vmhost::set_error("vm_conv_proj_fwd: unsupported shape (bf16, dim %% 64 == 0, width <= 4, "
                      "R + 2N <= 128, R <= 64, seqlen >= 1)");
    return VM_E_INVALID;
  }
  if (!vmhost::aligned16(xz) || !vmhost::aligned16(u) || !vmhost::aligned16(wx_pad) ||
      !vmhost::aligned16(wdt_pad) || xz_sb % 8 || xz_sl % 8 || u_sb % 8 || u_sl % 8) {
    vmhost::set_error("vm_conv_proj_fwd: xz / u / weights need 16-byte aligned rows");
    return VM_E_INVALID;
  }
  if (u_sb != out_len * u_sl || xd_sb != out_len * xd_sl || dt_sb != out_len * dt_sl) {
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
  p.xz_sb = xz_sb; p.xz_sl = xz_sl; p.csi_sb = csi_sb; p.csi_sd = csi_sd;
  p.cso_sb = cso_sb; p.cso_sd = cso_sd;
  p.u_sb = u_sb; p.u_sl = u_sl; p.xd_sb = xd_sb; p.xd_sl = xd_sl; p.dt_sb = dt_sb; p.dt_sl = dt_sl;
  p.batch = batch; p.dim = dim; p.seqlen = seqlen; p.lp = out_len;
  p.rows = batch * out_len; p.e = e; p.e_pad = e_pad; p.r = r; p.r_pad = r_pad;
  p.width = width; p.csi_dtype = cs_in_dtype; p.cso_dtype = cs_out_dtype;
  dim3 grid((p.rows + kCPTok - 1) / kCPTok);
  hipLaunchKernelGGL(conv_proj_kernel, grid, dim3(256), 0, static_cast<hipStream_t>(stream), p);
  return vmhost::launch_status("vm_conv_proj_fwd");
}
