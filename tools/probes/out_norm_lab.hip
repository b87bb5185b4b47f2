// out_proj GEMM fused with the next block's residual add + RMSNorm / LayerNorm.
//
// Between two blocks the reference runs (models/videomamba/mamba_simple.py:445-446, then
// videomamba.py:141-166 with fused_add_norm — mamba-ssm rms_norm_fn / layer_norm_fn):
//     hidden = y @ W_out^T                       (bf16 out, fp32 accumulation)
//     s      = float(hidden) + residual          (fp32, residual_in_fp32)
//     hn     = norm(s) * w (+ b)                 (statistics in fp32, rounded once)
// Done as two launches the hidden (rows x N bf16) makes an HBM round trip and the library
// GEMM pads N = 576 to 3 x 256-column tiles.  Here one workgroup owns 128 whole rows
// (every output column), so the row statistics close inside the workgroup:
//   main loop : 8 waves = 2 row halves x 4 column groups (CB blocks of 16 columns each),
//               v_mfma_f32_16x16x32_bf16 from LDS; each 32-wide K slice of the A tile
//               (128 y rows) and of W_out (all N rows; 1.3 MB at M, L2-resident) is
//               staged global -> registers -> LDS one slice ahead, double-buffered;
//   epilogue  : hidden rounded to bf16 (the reference's rounding point), + residual,
//               residual_out written, row sums reduced across the 16 lanes of a row
//               group (shuffles) and the 4 waves (LDS), normalised output written.
// HBM per row: y (K bf16) in, residual in and out (N fp32), hn out (N bf16).

#include <stdlib.h>

#include "vm_common.h"

namespace vm {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_on;
typedef __attribute__((ext_vector_type(4))) float f32x4_on;

struct OutNormParams {
  const bf16_t* y; const bf16_t* w_out; const float* res; const float* nw; const float* nb;
  bf16_t* out; float* res_out;
  long long rows, y_sl;
  int n, k, is_rms;
  float eps;
};

constexpr int kONRows = 128;  // rows per workgroup
constexpr int kONWaves = 8;   // 2 row halves x 4 column groups
constexpr int kONPitch = 40;  // LDS row pitch (bf16) of the 32-wide K slices: 80 B rows

__device__ __forceinline__ float sum16(float v) {  // over the 16 lanes sharing lane >> 4
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
}

// LDS: double-buffered K slices (32 wide) of the A tile (128 y rows) and of all of W_out
// (N rows), staged through registers one slice ahead; one barrier per slice.
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// EPI 0: epilogue straight from the MFMA layout (64-byte row pieces);
//     1: hidden staged through LDS in 32-row passes, then one wave per row as
//        vm_add_norm_fwd does it (16-byte lane accesses, full rows: coalesced);
//     2: GEMM only (timing probe, writes nothing useful).
template <int CB, bool RMS, int EPI = 1>  // column blocks of 16 per wave: N = 64 * CB
__global__ __launch_bounds__(512) void out_norm_kernel(const OutNormParams p) {
  constexpr int N = 64 * CB;
  static_assert(kONRows * 4 == 512, "one A chunk per thread");
  constexpr int kBChunks = N * 4;                 // 16-byte chunks per W_out slice
  constexpr int kCh = 1 + (kBChunks + 511) / 512; // chunk 0: A, then W_out
  __shared__ __attribute__((aligned(16))) bf16_t sA[2][kONRows * kONPitch];
  __shared__ __attribute__((aligned(16))) bf16_t sB[2][N * kONPitch];
  __shared__ float red[4][kONRows];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int rh = wave >> 2, cg = wave & 3;  // row half, column group
  const long long row0 = static_cast<long long>(blockIdx.x) * kONRows;
  const int K = p.k;

  // staging role: thread = (row tid/4, K quarter tid%4) of the A slice and of W_out rows
  // tid/4 + 128 (q - 1), q = 1 .. kCh-1 (the last one partial when N % 128 != 0)
  const int srow = tid >> 2;
  const int sq8 = (tid & 3) * 8;
  long long ar = row0 + srow;
  ar = ar < p.rows ? ar : p.rows - 1;
  const bf16_t* asrc = p.y + ar * p.y_sl + sq8;
  const bf16_t* bsrc = p.w_out + static_cast<long long>(srow) * K + sq8;
  const long long bq = 128ll * K;
  const int ldst = srow * kONPitch + sq8;
  // (plain macros, not lambdas over the staging array: a captured array is not split into
  // registers and the compiler parks it in LDS)
  uint4 stg0, stg1, stg2, stg3, stg4, stg5, stg6;
  static_assert(kCh <= 7, "N <= 768");
#define VM_ON_LIVE(q) ((q) < kCh && ((q) == 0 || ((q) - 1) * 128 + srow < N))
#define VM_ON_GL(q, k0)                                                                   \
  if (VM_ON_LIVE(q))                                                                      \
    stg##q = *reinterpret_cast<const uint4*>((q) == 0 ? asrc + (k0)                       \
                                                      : bsrc + ((q) - 1) * bq + (k0));
#define VM_ON_LS(q, buf)                                                                  \
  if (VM_ON_LIVE(q))                                                                      \
    *reinterpret_cast<uint4*>((q) == 0 ? sA[buf] + ldst                                   \
                                       : sB[buf] + ((q) - 1) * 128 * kONPitch + ldst) = stg##q;
#define VM_ON_GLOAD(k0) \
  { VM_ON_GL(0, k0) VM_ON_GL(1, k0) VM_ON_GL(2, k0) VM_ON_GL(3, k0) VM_ON_GL(4, k0) VM_ON_GL(5, k0) VM_ON_GL(6, k0) }
#define VM_ON_LSTORE(buf) \
  { VM_ON_LS(0, buf) VM_ON_LS(1, buf) VM_ON_LS(2, buf) VM_ON_LS(3, buf) VM_ON_LS(4, buf) VM_ON_LS(5, buf) VM_ON_LS(6, buf) }

  f32x4_on acc[4][CB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[i][j] = f32x4_on{0.f, 0.f, 0.f, 0.f};

  const int ka = (lane >> 4) * 8;
  const int arow = (rh * 64 + (lane & 15)) * kONPitch + ka;
  const int brow = (cg * CB * 16 + (lane & 15)) * kONPitch + ka;
  VM_ON_GLOAD(0)
  VM_ON_LSTORE(0)
  __syncthreads();
  const int steps = K / 32;
  for (int s = 0; s < steps; ++s) {
    const int buf = s & 1;
    if (s + 1 < steps) VM_ON_GLOAD((s + 1) * 32)
    bf16x8_on a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = *reinterpret_cast<const bf16x8_on*>(&sA[buf][arow + i * 16 * kONPitch]);
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const bf16x8_on b = *reinterpret_cast<const bf16x8_on*>(&sB[buf][brow + j * 16 * kONPitch]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc[i][j], 0, 0, 0);
    }
    if (s + 1 < steps) VM_ON_LSTORE(buf ^ 1)
    __syncthreads();
  }

#undef VM_ON_LIVE
#undef VM_ON_GL
#undef VM_ON_LS
#undef VM_ON_GLOAD
#undef VM_ON_LSTORE
  if constexpr (EPI == 2) {
    float t = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < CB; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1.2345e30f) p.out[tid] = from_f32<bf16_t>(t);
    return;
  }
  if constexpr (EPI == 1) {
    constexpr int HP = N + 16;  // fp32 pitch: 4 row groups x 16 columns hit 64 banks
    static_assert(32 * HP * 4 <= 2 * N * kONPitch * 2, "hidden pass fits in sB");
    float* hid = reinterpret_cast<float*>(&sB[0][0]);
    constexpr int CPL = (N + 255) / 256;  // 4-column chunks per lane
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      if (rh == (pass >> 1)) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const int i = 2 * (pass & 1) + ii;
#pragma unroll
          for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              hid[(ii * 16 + (lane >> 4) * 4 + e) * HP + cg * CB * 16 + j * 16 + (lane & 15)] =
                  to_f32(from_f32<bf16_t>(acc[i][j][e]));  // hidden in bf16
        }
      }
      __syncthreads();
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int lr = wave * 4 + rr;
        const long long row = row0 + pass * 32 + lr;
        if (row < p.rows) {
          float v[CPL][4];
          float sm = 0.0f;
#pragma unroll
          for (int m = 0; m < CPL; ++m) {
            const int c = lane * 4 + 256 * m;
            if (c < N) {
              const float4 hv = *reinterpret_cast<const float4*>(&hid[lr * HP + c]);
              v[m][0] = hv.x; v[m][1] = hv.y; v[m][2] = hv.z; v[m][3] = hv.w;
              if (p.res) {
                const float4 r = *reinterpret_cast<const float4*>(p.res + row * N + c);
                v[m][0] += r.x; v[m][1] += r.y; v[m][2] += r.z; v[m][3] += r.w;
              }
            } else {
              v[m][0] = v[m][1] = v[m][2] = v[m][3] = 0.0f;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) sm += v[m][q];
          }
          float mean = 0.0f, sq = 0.0f;
          if constexpr (RMS) {
#pragma unroll
            for (int m = 0; m < CPL; ++m)
#pragma unroll
              for (int q = 0; q < 4; ++q) sq = fmaf(v[m][q], v[m][q], sq);
          } else {
            mean = wsum(sm) / N;
#pragma unroll
            for (int m = 0; m < CPL; ++m) {
              const bool in = lane * 4 + 256 * m < N;
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const float dv = in ? v[m][q] - mean : 0.0f;
                sq = fmaf(dv, dv, sq);
              }
            }
          }
          const float rs = rsqrtf(wsum(sq) / N + p.eps);
#pragma unroll
          for (int m = 0; m < CPL; ++m) {
            const int c = lane * 4 + 256 * m;
            if (c < N) {
              const float4 wv = *reinterpret_cast<const float4*>(p.nw + c);
              const float w4[4] = {wv.x, wv.y, wv.z, wv.w};
              float o[4];
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                o[q] = (v[m][q] - mean) * rs * w4[q];
                if (p.nb) o[q] += p.nb[c + q];
              }
              uint2 packed;
              packed.x = static_cast<uint32_t>(from_f32<bf16_t>(o[0])) |
                         (static_cast<uint32_t>(from_f32<bf16_t>(o[1])) << 16);
              packed.y = static_cast<uint32_t>(from_f32<bf16_t>(o[2])) |
                         (static_cast<uint32_t>(from_f32<bf16_t>(o[3])) << 16);
              *reinterpret_cast<uint2*>(p.out + row * N + c) = packed;
              if (p.res_out)
                *reinterpret_cast<float4*>(p.res_out + row * N + c) =
                    make_float4(v[m][0], v[m][1], v[m][2], v[m][3]);
            }
          }
        }
      }
      __syncthreads();
    }
    return;
  }

  // ---- epilogue: acc[i][j][e] is (row rh*64 + i*16 + (lane>>4)*4 + e,
  //                                 col (cg*CB + j)*16 + lane&15)
  const int c0 = cg * CB * 16 + (lane & 15);
  const int lrow0 = rh * 64 + (lane >> 4) * 4;
  float rsum[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long row = row0 + lrow0 + i * 16 + e;
      const bool live = row < p.rows;
      const long long base = (live ? row : 0) * N + c0;
      float sm = 0.0f;
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        float v = to_f32(from_f32<bf16_t>(acc[i][j][e]));  // hidden in bf16
        if (p.res) v += live ? p.res[base + j * 16] : 0.0f;
        acc[i][j][e] = v;
        sm += v;
      }
      rsum[i][e] = sm;
    }
  // residual_out (in place over residual is fine: each element is read above by this lane)
  if (p.res_out) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long long row = row0 + lrow0 + i * 16 + e;
        if (row < p.rows) {
#pragma unroll
          for (int j = 0; j < CB; ++j) p.res_out[row * N + c0 + j * 16] = acc[i][j][e];
        }
      }
  }
  auto row_total = [&](float (&part)[4][4], float (&tot)[4][4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) part[i][e] = sum16(part[i][e]);
    __syncthreads();
    if ((lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[cg][lrow0 + i * 16 + e] = part[i][e];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = lrow0 + i * 16 + e;
        tot[i][e] = (red[0][r] + red[1][r]) + (red[2][r] + red[3][r]);
      }
  };
  float mean[4][4], sq[4][4];
  if constexpr (RMS) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float q = 0.0f;
#pragma unroll
        for (int j = 0; j < CB; ++j) q = fmaf(acc[i][j][e], acc[i][j][e], q);
        sq[i][e] = q;
        mean[i][e] = 0.0f;
      }
  } else {
    row_total(rsum, mean);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float m = mean[i][e] / N;
        mean[i][e] = m;
        float q = 0.0f;
#pragma unroll
        for (int j = 0; j < CB; ++j) {
          const float dv = acc[i][j][e] - m;
          q = fmaf(dv, dv, q);
        }
        sq[i][e] = q;
      }
  }
  row_total(sq, sq);  // sums of squares -> in place
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) sq[i][e] = rsqrtf(sq[i][e] / N + p.eps);
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    const float wv = p.nw[c0 + j * 16];
    const float bv = p.nb ? p.nb[c0 + j * 16] : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long long row = row0 + lrow0 + i * 16 + e;
        if (row < p.rows) {
          float o = (acc[i][j][e] - mean[i][e]) * sq[i][e] * wv;
          if (p.nb) o += bv;
          p.out[row * N + c0 + j * 16] = from_f32<bf16_t>(o);
        }
      }
  }
}

}  // namespace vm

using namespace vm;

extern "C" int vm_out_proj_add_norm_fwd(const void* y, long long y_sl, const void* w_out,
                                        const float* residual, const float* norm_weight,
                                        const float* norm_bias, void* out, float* residual_out,
                                        long long rows, int n, int k, float eps, int is_rms,
                                        vm_stream_t stream) {
  if (!y || !w_out || !norm_weight || !out) {
    vmhost::set_error("vm_out_proj_add_norm_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (rows < 0 || k < 32 || k % 32 != 0 || n < 64 || n % 64 != 0 || n > 64 * 12 ||
      y_sl < k || y_sl % 8 != 0 || !vmhost::aligned16(y) || !vmhost::aligned16(w_out)) {
    vmhost::set_error("vm_out_proj_add_norm_fwd: unsupported shape (k %% 32 == 0, n %% 64 == 0, "
                      "n <= 768, 16-byte aligned y rows and W_out)");
    return VM_E_INVALID;
  }
  if (rows == 0) return VM_OK;
  OutNormParams p{};
  p.y = static_cast<const bf16_t*>(y); p.w_out = static_cast<const bf16_t*>(w_out);
  p.res = residual; p.nw = norm_weight; p.nb = norm_bias;
  p.out = static_cast<bf16_t*>(out); p.res_out = residual_out;
  p.rows = rows; p.y_sl = y_sl; p.n = n; p.k = k; p.is_rms = is_rms; p.eps = eps;
  dim3 grid(static_cast<unsigned>((rows + kONRows - 1) / kONRows));
  hipStream_t st = static_cast<hipStream_t>(stream);
  // VM_OUT_NORM_EPI (per call): 1 LDS-staged row epilogue (default), 0 direct, 2 GEMM-only
  // timing probe
  const char* ev = getenv("VM_OUT_NORM_EPI");
  const int epi = ev ? atoi(ev) : 1;
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(512), 0, st, p); };
  switch (n / 64) {
#define VM_ON_CASE(C)                                                                   \
    case C:                                                                             \
      if (epi == 0 && is_rms) go(out_norm_kernel<C, true, 0>);                         \
      else if (epi == 0) go(out_norm_kernel<C, false, 0>);                             \
      else if (epi == 2) go(out_norm_kernel<C, true, 2>);                              \
      else if (is_rms) go(out_norm_kernel<C, true, 1>);                                \
      else go(out_norm_kernel<C, false, 1>);                                           \
      break;
    VM_ON_CASE(1) VM_ON_CASE(2) VM_ON_CASE(3) VM_ON_CASE(4) VM_ON_CASE(5) VM_ON_CASE(6)
    VM_ON_CASE(7) VM_ON_CASE(8) VM_ON_CASE(9) VM_ON_CASE(10) VM_ON_CASE(11) VM_ON_CASE(12)
#undef VM_ON_CASE
  }
  return vmhost::launch_status("vm_out_proj_add_norm_fwd");
}
