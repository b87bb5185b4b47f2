// Tubelet patch embed: Conv3d with kernel = stride = (kt, Ph, Pw) as an implicit GEMM,
// fused with the bias, the spatial and the temporal positional embedding adds.
// Replaces PatchEmbed.forward + the pos-embed adds of models/videomamba/videomamba.py
// (:359-368, :806-815).  The reference materialises the conv output, the +spatial and
// the +temporal sums in the model dtype; the epilogue rounds at the same three points.
//
//   tok[m, n] = sum_k video[gather(m, k)] * weight[n, k],  m = (b, t, gh, gw),
//   k = (ci, kt_, kh, kw) in the weight's (C, Cin, kt, Ph, Pw) order.  Rectangular
//   patches (Ph != Pw) are the reference's PatchEmbed(patch_size=(ph, pw)) (:340-364).
//
// bf16 path: v_mfma_f32_16x16x32_bf16, operands loaded straight into fragments (with
// Pw % 8 == 0 the 8 consecutive k of a lane are 8 contiguous pixels of one patch row:
// one 16-byte load), block tile 64 tokens x 64 channels (2x2 waves of 32x32).
// Other shapes / fp32: a scalar implicit-GEMM kernel (same math, fp32 accumulate).

#include <stdlib.h>

#include "vm_common.h"

namespace vm {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct PatchParams {
  const void* video; const void* w; const float* bias; const void* spos; const void* tpos;
  void* out;
  const void* cls; const void* cls_pos;  // head rows [0, row0) = e(cls + cls_pos) (nullable)
  long long out_sb;
  int row0, batch, cin, frames, height, width, kt, ph, pw, embed;
  int pad_rows;  // zero rows after the tokens (the padded buffer's tail)
  int tt, gh, gw, K, M;  // derived: temporal tokens, grid, reduction length, tokens
};

// The rows of the padded token buffer around the patch tokens, written by the launch's
// channel-tile-0 workgroups (block bx of nbx along the tokens, channel tile by) after their tiles (the scalar fallback: before) (grid-stride over batch x rows x channels):
// the CLS rows [0, row0) = e(cls + cls_pos) — the reference's cls_token + pos_embed[:, :1]
// in the model dtype (videomamba.py:806-815) — and pad_rows zero rows after the last token.
// Folded in here they cost no launches of their own (three small torch kernels before).
template <typename T>
__device__ __forceinline__ void patch_frame_rows(const PatchParams& p, int bx, int nbx, int by) {
  const int head = p.cls ? p.row0 : 0;
  const int per_b = head + p.pad_rows;
  if (by != 0 || per_b == 0) return;
  const int ntok = p.tt * p.gh * p.gw;
  const int total = p.batch * per_b * p.embed;  // < 2^31 (checked on the host)
  for (int i = bx * blockDim.x + threadIdx.x; i < total; i += nbx * blockDim.x) {
    const int br = i / p.embed;
    const int c = i - br * p.embed;
    const int b = br / per_b;
    const int r = br - b * per_b;
    float v = 0.0f;
    int row = p.row0 + ntok + (r - head);
    if (r < head) {
      row = r;
      v = to_f32(static_cast<const T*>(p.cls)[c]) + to_f32(static_cast<const T*>(p.cls_pos)[c]);
    }
    static_cast<T*>(p.out)[b * p.out_sb + static_cast<long long>(row) * p.embed + c] = from_f32<T>(v);
  }
}

template <typename T>
__device__ __forceinline__ void patch_store(const PatchParams& p, int m, int n, float acc) {
  const int hw = p.gh * p.gw;
  const int per_b = p.tt * hw;
  const int b = m / per_b;
  const int rem = m - b * per_b;
  const int t = rem / hw;
  const int s = rem - t * hw;
  float v = round_to<T>(acc + p.bias[n]);
  v = round_to<T>(v + to_f32(static_cast<const T*>(p.spos)[(long long)s * p.embed + n]));
  v = v + to_f32(static_cast<const T*>(p.tpos)[(long long)t * p.embed + n]);
  static_cast<T*>(p.out)[b * p.out_sb + (long long)(p.row0 + rem) * p.embed + n] = from_f32<T>(v);
}

__device__ __forceinline__ long long token_base(const PatchParams& p, int m) {
  const int hw = p.gh * p.gw;
  const int per_b = p.tt * hw;
  const int b = m / per_b;
  const int rem = m - b * per_b;
  const int t = rem / hw;
  const int s = rem - t * hw;
  const int gy = s / p.gw;
  const int gx = s - gy * p.gw;
  return ((long long)b * p.cin * p.frames + (long long)t * p.kt) * p.height * p.width +
         (long long)gy * p.ph * p.width + (long long)gx * p.pw;
}

__device__ __forceinline__ long long k_offset(const PatchParams& p, int k) {
  const int pp = p.ph * p.pw;
  const int per_c = p.kt * pp;
  const int ci = k / per_c;
  const int r1 = k - ci * per_c;
  const int kz = r1 / pp;
  const int r2 = r1 - kz * pp;
  const int ky = r2 / p.pw;
  const int kx = r2 - ky * p.pw;
  return ((long long)ci * p.frames + kz) * p.height * p.width + (long long)ky * p.width + kx;
}

__global__ __launch_bounds__(256) void patch_mfma_kernel(const PatchParams p) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 64 + (wave & 1) * 32;
  const int n0 = blockIdx.y * 64 + (wave >> 1) * 32;
  const int r = lane & 15;
  const int kg = lane >> 4;
  const bf16_t* vid = static_cast<const bf16_t*>(p.video);
  const bf16_t* wt = static_cast<const bf16_t*>(p.w);

  long long abase[2];
  bool mval[2], nval[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + i * 16 + r;
    mval[i] = m < p.M;
    abase[i] = token_base(p, mval[i] ? m : 0);
    nval[i] = (n0 + i * 16 + r) < p.embed;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16x8 zero = {};
  for (int kk = 0; kk < p.K; kk += 32) {
    const int k = kk + kg * 8;
    const bool kval = k < p.K;
    const long long koff = k_offset(p, kval ? k : 0);
    bf16x8 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      a[i] = (kval && mval[i]) ? *reinterpret_cast<const bf16x8*>(vid + abase[i] + koff) : zero;
      const int n = n0 + i * 16 + r;
      b[i] = (kval && nval[i]) ? *reinterpret_cast<const bf16x8*>(wt + (long long)n * p.K + k) : zero;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + i * 16 + kg * 4 + e;
        const int n = n0 + j * 16 + r;
        if (m < p.M && n < p.embed) patch_store<bf16_t>(p, m, n, acc[i][j][e]);
      }
  patch_frame_rows<bf16_t>(p, blockIdx.x, gridDim.x, blockIdx.y);  // after the tile: the head / padding rows never delay it
}

// 16x16 patches, bf16, embed % 192 == 0 (the VideoMamba shapes): workgroup tile
// 64 tokens x 192 channels (2x2 waves of 32 x 96, so each video patch row is read by 3
// workgroups instead of 9), im2col offsets advanced by shifts (one k-step of 32 = two
// patch rows of one channel), and the epilogue staged through LDS so the bias / spatial /
// temporal adds and the stores run on 8-channel vectors of whole output rows.
constexpr int kPT = 64, kPN = 192, kPJ = 6;  // tokens, channels per workgroup; 16-col tiles per wave
__global__ __launch_bounds__(256) void patch_mfma16_kernel(const PatchParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t stile[kPT * (kPN + 8)];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int mt0 = blockIdx.x * kPT;
  const int m0 = mt0 + (wave & 1) * 32;
  const int n0 = blockIdx.y * kPN + (wave >> 1) * 96;
  const int r = lane & 15;
  const int kg = lane >> 4;
  const bf16_t* vid = static_cast<const bf16_t*>(p.video);
  const bf16_t* wt = static_cast<const bf16_t*>(p.w);
  const long long plane = (long long)p.frames * p.height * p.width;  // one input channel
  // lane's k within a 32-wide k-step: patch row 2*step + (kg >> 1), columns (kg & 1) * 8
  const long long lane_k = (long long)(kg >> 1) * p.width + (kg & 1) * 8;

  long long abase[2];  // rows past the last token read token 0 (their outputs are never stored)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + i * 16 + r;
    abase[i] = token_base(p, m < p.M ? m : 0) + lane_k;
  }
  const bf16_t* wrow[kPJ];
#pragma unroll
  for (int j = 0; j < kPJ; ++j) wrow[j] = wt + (long long)(n0 + j * 16 + r) * p.K + kg * 8;
  f32x4 acc[2][kPJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < kPJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int steps_per_c = 8 * p.kt;  // 256 * kt k per input channel, 32 per step
  // two register sets of operands, ping-ponged: one k-step's loads are in flight while
  // the other's 12 MFMAs run.  16x16 patches make K = 256 * cin * kt, a whole number of
  // step pairs, so every load and MFMA is unconditional (the last pair's look-ahead load is
  // clamped to the last step): no register copies close the loop and nothing is sunk into a
  // branch, so the waits stay counted instead of draining every load each step.
  auto load = [&](int kk, bf16x8 (&ra)[2], bf16x8 (&rb)[kPJ]) {
    const int step = kk >> 5;
    const int ci = step / steps_per_c;
    const int sr = step - ci * steps_per_c;  // (kz, row pair) within the channel
    const int kz = sr >> 3;
    const long long koff = ci * plane + (long long)kz * p.height * p.width +
                           (long long)(2 * (sr & 7)) * p.width;
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = *reinterpret_cast<const bf16x8*>(vid + abase[i] + koff);
#pragma unroll
    for (int j = 0; j < kPJ; ++j) rb[j] = *reinterpret_cast<const bf16x8*>(wrow[j] + kk);
  };
  auto mma = [&](const bf16x8 (&ra)[2], const bf16x8 (&rb)[kPJ]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < kPJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra[i], rb[j], acc[i][j], 0, 0, 0);
  };
  const int klast = p.K - 32;
  bf16x8 a0[2], b0[kPJ], a1[2], b1[kPJ];
  load(0, a0, b0);
  for (int kk = 0; kk < p.K; kk += 64) {
    load(kk + 32, a1, b1);
    mma(a0, b0);
    load(min(kk + 64, klast), a0, b0);
    mma(a1, b1);
  }
  // stage round(acc + bias) (the conv output's rounding point) as bf16 [token][channel]
#pragma unroll
  for (int j = 0; j < kPJ; ++j) {
    const int nl = (wave >> 1) * 96 + j * 16 + r;
    const float bj = p.bias[blockIdx.y * kPN + nl];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ml = (wave & 1) * 32 + i * 16 + kg * 4 + e;
        stile[ml * (kPN + 8) + nl] = from_f32<bf16_t>(acc[i][j][e] + bj);
      }
  }
  __syncthreads();
  // + spatial pos (rounded), + temporal pos, 8 channels per thread-vector
  const int hw = p.gh * p.gw;
  const int per_b = p.tt * hw;
  const bf16_t* spos = static_cast<const bf16_t*>(p.spos);
  const bf16_t* tpos = static_cast<const bf16_t*>(p.tpos);
  bf16_t* out = static_cast<bf16_t*>(p.out);
  // the positional loads of all 6 chunks first, then the adds and stores: one L2 round
  // trip per tile instead of one per chunk (each store would otherwise order the next loads)
  constexpr int kEpi = kPT * (kPN / 8) / 256;
  uint4 svs[kEpi], tvs[kEpi];
  long long orow[kEpi];
  int soff[kEpi];
#pragma unroll
  for (int it = 0; it < kEpi; ++it) {
    const int idx = tid + it * 256;
    const int ml = idx / (kPN / 8);
    const int c8 = (idx - ml * (kPN / 8)) * 8;
    const int m = mt0 + ml;
    const bool ok = m < p.M;
    const int b = ok ? m / per_b : 0;
    const int rem = ok ? m - b * per_b : 0;
    const int t = rem / hw;
    const int sp = rem - t * hw;
    const int n = blockIdx.y * kPN + c8;
    svs[it] = *reinterpret_cast<const uint4*>(spos + (long long)sp * p.embed + n);
    tvs[it] = *reinterpret_cast<const uint4*>(tpos + (long long)t * p.embed + n);
    orow[it] = ok ? b * p.out_sb + (long long)(p.row0 + rem) * p.embed + n : -1;
    soff[it] = ml * (kPN + 8) + c8;
  }
#pragma unroll
  for (int it = 0; it < kEpi; ++it) {
    if (orow[it] < 0) continue;
    const uint4 cv = *reinterpret_cast<const uint4*>(&stile[soff[it]]);
    const uint32_t cw[4] = {cv.x, cv.y, cv.z, cv.w},
                   sw[4] = {svs[it].x, svs[it].y, svs[it].z, svs[it].w},
                   tw[4] = {tvs[it].x, tvs[it].y, tvs[it].z, tvs[it].w};
    uint32_t ow[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float o[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float c = __uint_as_float(h ? (cw[q] & 0xffff0000u) : (cw[q] << 16));
        const float sp_ = __uint_as_float(h ? (sw[q] & 0xffff0000u) : (sw[q] << 16));
        const float tp = __uint_as_float(h ? (tw[q] & 0xffff0000u) : (tw[q] << 16));
        o[h] = round_to<bf16_t>(c + sp_) + tp;
      }
      ow[q] = static_cast<uint32_t>(from_f32<bf16_t>(o[0])) |
              (static_cast<uint32_t>(from_f32<bf16_t>(o[1])) << 16);
    }
    *reinterpret_cast<uint4*>(out + orow[it]) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
  }
  patch_frame_rows<bf16_t>(p, blockIdx.x, gridDim.x, blockIdx.y);  // after the tile: the head / padding rows never delay it
}

// 16x16 patches, bf16, embed % 192 == 0, an LDS-staged GEMM: workgroup tile 128 tokens x
// 192 channels, 4 waves of 64 x 96 (24 accumulators), K in steps of 32 with the im2col A
// tile (8 KB) and the weight tile (12 KB) staged through two LDS buffers by register
// prefetch (the next step's loads are in flight during this step's 24 MFMAs per wave).
// The epilogue re-uses the staging area for the same vectorised bias / pos adds as
// patch_mfma16_kernel.  Same k order and rounding points as the 64x64 kernel.
constexpr int kGT = 128, kGN = 192, kGP = 40;  // tile tokens, channels; LDS row pitch (bf16)
__global__ __launch_bounds__(256) void patch_gemm_kernel(const PatchParams p) {
  // staging: 2 buffers x (A 128 x 40 + B 192 x 40) bf16 = 40 KB; epilogue: 128 x 200 bf16
  __shared__ __attribute__((aligned(16))) bf16_t smem[kGT * (kGN + 8)];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  // XCD-grouped tile order (one linear grid): ids g * 8 * nn + ni * 8 + x hold token tile
  // g * 8 + x, channel tile ni, so the nn channel tiles of one token tile share the id's
  // residue mod 8 — the same XCD — and read their video patches through one L2.
  const int nn = p.embed / kGN, nm = (p.M + kGT - 1) / kGT;
  const int grp = blockIdx.x / (8 * nn), rg = blockIdx.x - grp * 8 * nn;
  const int mti = grp * 8 + (rg & 7), nti = rg >> 3;
  if (mti >= nm) return;  // the last group's missing token tiles (before any barrier)
  const int mt0 = mti * kGT;
  const int nt0 = nti * kGN;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * 96;
  const int r16 = lane & 15, kg = lane >> 4;
  const bf16_t* vid = static_cast<const bf16_t*>(p.video);
  const bf16_t* wt = static_cast<const bf16_t*>(p.w);
  const long long plane = (long long)p.frames * p.height * p.width;
  constexpr int kA = kGT * kGP, kB = kGN * kGP, kBuf = kA + kB;

  // staging roles: A: 512 16-byte chunks (row = idx >> 2, c = idx & 3) -> 2 per thread;
  //                B: 768 chunks -> 3 per thread
  long long abase[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int idx = tid + q * 256;
    const int row = idx >> 2, c = idx & 3;
    const int m = mt0 + row;
    abase[q] = token_base(p, m < p.M ? m : 0) + (long long)(c >> 1) * p.width + (c & 1) * 8;
  }
  auto koff_of = [&](int kk) {
    const int step = kk >> 5;
    const int steps_per_c = 8 * p.kt;
    const int ci = step / steps_per_c;
    const int sr = step - ci * steps_per_c;
    return ci * plane + (long long)(sr >> 3) * p.height * p.width +
           (long long)(2 * (sr & 7)) * p.width;
  };
  // the staged chunks in named registers: as arrays the compiler kept the weight chunks in
  // scratch, and each k-step waited for their loads before its MFMAs
  uint4 ra0, ra1, rb0, rb1, rb2;
  const int brow = tid >> 2, bc = (tid & 3) * 8;  // B chunk q: row brow + 64 q, column bc
  auto fetch = [&](int kk) {
    const long long ko = koff_of(kk);
    // rows past the last token read token 0's pixels (abase): their outputs are never
    // stored, and no branch here lets the loads stay in flight across the MFMAs
    ra0 = *reinterpret_cast<const uint4*>(vid + abase[0] + ko);
    ra1 = *reinterpret_cast<const uint4*>(vid + abase[1] + ko);
    const bf16_t* wb = wt + (long long)(nt0 + brow) * p.K + kk + bc;
    rb0 = *reinterpret_cast<const uint4*>(wb);
    rb1 = *reinterpret_cast<const uint4*>(wb + 64LL * p.K);
    rb2 = *reinterpret_cast<const uint4*>(wb + 128LL * p.K);
  };
  auto put = [&](int buf) {
    bf16_t* sa = smem + buf * kBuf + brow * kGP + bc;  // A chunk q: row brow + 64 q
    bf16_t* sb = smem + buf * kBuf + kA + brow * kGP + bc;
    *reinterpret_cast<uint4*>(sa) = ra0;
    *reinterpret_cast<uint4*>(sa + 64 * kGP) = ra1;
    *reinterpret_cast<uint4*>(sb) = rb0;
    *reinterpret_cast<uint4*>(sb + 64 * kGP) = rb1;
    *reinterpret_cast<uint4*>(sb + 128 * kGP) = rb2;
  };

  f32x4 acc[4][6];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  fetch(0);
  put(0);
  __syncthreads();
  const int nk = p.K / 32;
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) fetch((ks + 1) * 32);  // lands while this step's MFMAs run
    const bf16_t* sa = smem + buf * kBuf;
    const bf16_t* sb = sa + kA;
    bf16x8 a[4], b[6];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(sa + (wm + i * 16 + r16) * kGP + kg * 8);
#pragma unroll
    for (int j = 0; j < 6; ++j)
      b[j] = *reinterpret_cast<const bf16x8*>(sb + (wn + j * 16 + r16) * kGP + kg * 8);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    if (ks + 1 < nk) put(buf ^ 1);  // the other buffer's readers finished before the last barrier
    __syncthreads();
  }
  // epilogue staging: round(acc + bias) as bf16 [token][channel]
  bf16_t* stile = smem;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int nl = wn + j * 16 + r16;
    const float bj = p.bias[nt0 + nl];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        stile[(wm + i * 16 + kg * 4 + e) * (kGN + 8) + nl] = from_f32<bf16_t>(acc[i][j][e] + bj);
  }
  __syncthreads();
  const int hw = p.gh * p.gw;
  const int per_b = p.tt * hw;
  const bf16_t* spos = static_cast<const bf16_t*>(p.spos);
  const bf16_t* tpos = static_cast<const bf16_t*>(p.tpos);
  bf16_t* out = static_cast<bf16_t*>(p.out);
  // the positional loads of 6 chunks first, then their adds and stores: one L2 round trip
  // per half tile instead of one per chunk (each store would otherwise order the next loads)
  constexpr int kEpi = kGT * (kGN / 8) / 256, kEpiH = kEpi / 2;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    uint4 svs[kEpiH], tvs[kEpiH];
    long long orow[kEpiH];
    int soff[kEpiH];
#pragma unroll
    for (int it = 0; it < kEpiH; ++it) {
      const int idx = tid + (half * kEpiH + it) * 256;
      const int ml = idx / (kGN / 8);
      const int c8 = (idx - ml * (kGN / 8)) * 8;
      const int m = mt0 + ml;
      const bool ok = m < p.M;
      const int b = ok ? m / per_b : 0;
      const int rem = ok ? m - b * per_b : 0;
      const int t = rem / hw;
      const int sp = rem - t * hw;
      const int n = nt0 + c8;
      svs[it] = *reinterpret_cast<const uint4*>(spos + (long long)sp * p.embed + n);
      tvs[it] = *reinterpret_cast<const uint4*>(tpos + (long long)t * p.embed + n);
      orow[it] = ok ? b * p.out_sb + (long long)(p.row0 + rem) * p.embed + n : -1;
      soff[it] = ml * (kGN + 8) + c8;
    }
#pragma unroll
    for (int it = 0; it < kEpiH; ++it) {
      if (orow[it] < 0) continue;
      const uint4 cv = *reinterpret_cast<const uint4*>(&stile[soff[it]]);
      const uint32_t cw[4] = {cv.x, cv.y, cv.z, cv.w},
                     sw[4] = {svs[it].x, svs[it].y, svs[it].z, svs[it].w},
                     tw[4] = {tvs[it].x, tvs[it].y, tvs[it].z, tvs[it].w};
      uint32_t ow[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float o[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float c = __uint_as_float(h ? (cw[q] & 0xffff0000u) : (cw[q] << 16));
          const float sp_ = __uint_as_float(h ? (sw[q] & 0xffff0000u) : (sw[q] << 16));
          const float tp = __uint_as_float(h ? (tw[q] & 0xffff0000u) : (tw[q] << 16));
          o[h] = round_to<bf16_t>(c + sp_) + tp;
        }
        ow[q] = static_cast<uint32_t>(from_f32<bf16_t>(o[0])) |
                (static_cast<uint32_t>(from_f32<bf16_t>(o[1])) << 16);
      }
      *reinterpret_cast<uint4*>(out + orow[it]) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    }
  }
  patch_frame_rows<bf16_t>(p, mti, nm, nti);  // after the tile: the head / padding rows never delay it
}

template <typename T>
__global__ __launch_bounds__(256) void patch_generic_kernel(const PatchParams p) {
  patch_frame_rows<T>(p, blockIdx.x, gridDim.x, blockIdx.y);
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)p.M * p.embed) return;
  const int m = static_cast<int>(gid / p.embed);
  const int n = static_cast<int>(gid - (long long)m * p.embed);
  const T* vid = static_cast<const T*>(p.video);
  const T* wt = static_cast<const T*>(p.w) + (long long)n * p.K;
  const long long base = token_base(p, m);
  float acc = 0.0f;
  for (int k = 0; k < p.K; ++k) acc = fmaf(to_f32(vid[base + k_offset(p, k)]), to_f32(wt[k]), acc);
  patch_store<T>(p, m, n, acc);
}

}  // namespace vm

using namespace vm;

extern "C" int vm_patch_embed_fwd(const void* video, const void* weight, const float* bias,
                                  const void* spos, const void* tpos, void* out, long long out_sb,
                                  int row0, int batch, int cin, int frames, int height, int width,
                                  int kt, int patch_h, int patch_w, int embed, int dtype,
                                  const void* cls, const void* cls_pos, int pad_rows,
                                  vm_stream_t stream) {
  if (!video || !weight || !bias || !spos || !tpos || !out) {
    vmhost::set_error("vm_patch_embed_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (batch < 0 || cin < 1 || kt < 1 || patch_h < 1 || patch_w < 1 || embed < 1 ||
      frames % kt != 0 || height < patch_h || width < patch_w || !vmhost::dtype_ok(dtype) ||
      row0 < 0 || pad_rows < 0 || (cls == nullptr) != (cls_pos == nullptr) ||
      1LL * batch * (pad_rows + (cls ? row0 : 0)) * embed > 0x7fffffffLL) {
    vmhost::set_error("vm_patch_embed_fwd: bad shape/dtype");
    return VM_E_INVALID;
  }
  PatchParams p{};
  p.video = video; p.w = weight; p.bias = bias; p.spos = spos; p.tpos = tpos; p.out = out;
  p.cls = cls; p.cls_pos = cls_pos; p.pad_rows = pad_rows;
  p.out_sb = out_sb; p.row0 = row0; p.batch = batch; p.cin = cin; p.frames = frames;
  p.height = height; p.width = width; p.kt = kt; p.ph = patch_h; p.pw = patch_w; p.embed = embed;
  p.tt = frames / kt; p.gh = height / patch_h; p.gw = width / patch_w;
  p.K = cin * kt * patch_h * patch_w;
  const long long M = 1LL * batch * p.tt * p.gh * p.gw;
  if (M == 0) return VM_OK;
  if (M > 0x7fffffffLL) {
    vmhost::set_error("vm_patch_embed_fwd: too many tokens");
    return VM_E_INVALID;
  }
  p.M = static_cast<int>(M);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool mfma_ok = dtype == VM_DTYPE_BF16 && patch_w % 8 == 0 && width % 8 == 0 &&
                       p.K % 8 == 0 && vmhost::aligned16(video) && vmhost::aligned16(weight);
  const bool wide_ok = mfma_ok && patch_h == 16 && patch_w == 16 && embed % kPN == 0 && p.K % 64 == 0 &&
                       out_sb % 8 == 0 && vmhost::aligned16(out) && vmhost::aligned16(spos) &&
                       vmhost::aligned16(tpos);
  // the 128-token LDS-staged tiles pay off on chip-filling batches; small ones keep more,
  // smaller workgroups (B = 1: 147 of 64 x 192 against 75 of 128 x 192).  All three MFMA
  // kernels accumulate in the same k order and round at the same points (bit-identical).
  if (wide_ok && p.M >= 32768) {
    dim3 grid(static_cast<unsigned>((p.M + 8 * kGT - 1) / (8 * kGT) * 8 * (embed / kGN)));
    hipLaunchKernelGGL(patch_gemm_kernel, grid, dim3(256), 0, s, p);
  } else if (wide_ok) {  // the 64x192 register-fragment kernel
    dim3 grid((p.M + kPT - 1) / kPT, embed / kPN);
    hipLaunchKernelGGL(patch_mfma16_kernel, grid, dim3(256), 0, s, p);
  } else if (mfma_ok) {
    dim3 grid((p.M + 63) / 64, (embed + 63) / 64);
    hipLaunchKernelGGL(patch_mfma_kernel, grid, dim3(256), 0, s, p);
  } else {
    const long long total = M * embed;
    dim3 grid(static_cast<unsigned>((total + 255) / 256));
    if (dtype == VM_DTYPE_BF16) hipLaunchKernelGGL(patch_generic_kernel<bf16_t>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(patch_generic_kernel<float>, grid, dim3(256), 0, s, p);
  }
  return vmhost::launch_status("vm_patch_embed_fwd");
}
