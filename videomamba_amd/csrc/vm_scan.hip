// Channel-major selective scan (forward) and the one-token state update for gfx950.
//
// Replaces mamba-ssm's selective_scan_fn / selective_state_update as called by the
// reference at models/videomamba/mamba_simple.py:122-172 and :483-494; the math is
// _selective_scan_ref (mamba_simple.py:30-106): fp32 internally, softplus threshold 20,
// output rounded to the input dtype, state carried in fp32.
//
// This file holds the time-parallel kernel for channel-major operands (unit step stride;
// the small-batch mixer layout) and the ABI entry points, which route token-major operands
// (unit channel stride) to vm_scan_seq.hip.  Measured-loser variants of round 1 (v1-v4, the
// time-split form) live in tools/probes/scan_variants_r01.hip and are not built.
//
// scan_v5_kernel: one wave per channel row; lane l covers K consecutive steps of a
// 64*K-step block.  Per state n: a lane-local fold of its K steps into (a, b), a DPP
// Hillis-Steele scan over the 64 lanes (row_shr 1/2/4/8, row_bcast 15/31) whose range
// products are exp2 of delta prefix sums (state-independent, off the serial chain), the
// block carry entering at lane 0, and a re-sweep emitting y.  B_t / C_t rows are staged
// per block in LDS as fp32.

#include <stdlib.h>

#include "vm_scan.h"

namespace vm {

template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ float dppz(float v) {  // invalid source lanes read 0
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWMASK, 0xf, true));
}

// Scalar-math successor of v4 (measured on gfx950: v_pk_fma_f32 costs ~2x v_fma_f32 per
// wave instruction, so packing buys nothing; v_exp_f32 ~3x).  One state per pass, K
// steps per lane with any even K (K=10 covers L=3137 in 5 blocks of 640 at 98% lane
// use), B/C staged as fp32 in a [state][K/2][lane][2] layout (ds_read_b64, 512
// contiguous bytes per wave), u/delta/z read with 4-byte (bf16 pair) or 16-byte loads.
template <typename T, int K>
__device__ __forceinline__ void load_even(const T* row, int t0, int L, bool vec, float (&v)[K]) {
  if (vec && t0 + K <= L) {
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int j = 0; j < K; j += 2) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(row + t0 + j);
        v[j] = __uint_as_float(w << 16);
        v[j + 1] = __uint_as_float(w & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int j = 0; j < K; j += 2) {
        const float2 w = *reinterpret_cast<const float2*>(row + t0 + j);
        v[j] = w.x;
        v[j + 1] = w.y;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = (t0 + k < L) ? to_f32(row[t0 + k]) : 0.0f;
  }
}

// bf16 pairs as raw words (the pipelined v5 keeps the next block's inputs packed)
template <int K>
__device__ __forceinline__ void load_even_raw(const bf16_t* row, int t0, int L, bool vec,
                                              uint32_t (&w)[K / 2]) {
  if (vec && t0 + K <= L) {
#pragma unroll
    for (int j = 0; j < K / 2; ++j) w[j] = *reinterpret_cast<const uint32_t*>(row + t0 + 2 * j);
  } else {
#pragma unroll
    for (int j = 0; j < K / 2; ++j) {
      const uint32_t lo = t0 + 2 * j < L ? static_cast<uint32_t>(row[t0 + 2 * j]) : 0u;
      const uint32_t hi = t0 + 2 * j + 1 < L ? static_cast<uint32_t>(row[t0 + 2 * j + 1]) : 0u;
      w[j] = lo | (hi << 16);
    }
  }
}
template <int K>
__device__ __forceinline__ void unpack_even(const uint32_t (&w)[K / 2], float (&v)[K]) {
#pragma unroll
  for (int j = 0; j < K / 2; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}

template <typename T, int K>
__device__ __forceinline__ void store_even(T* row, int t0, int LO, bool vec, const float (&v)[K]) {
  if (vec && t0 + K <= LO) {
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int j = 0; j < K; j += 2)
        *reinterpret_cast<uint32_t*>(row + t0 + j) =
            static_cast<uint32_t>(from_f32<bf16_t>(v[j])) |
            (static_cast<uint32_t>(from_f32<bf16_t>(v[j + 1])) << 16);
    } else {
#pragma unroll
      for (int j = 0; j < K; j += 2)
        *reinterpret_cast<float2*>(row + t0 + j) = make_float2(v[j], v[j + 1]);
    }
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (t0 + k < LO) row[t0 + k] = from_f32<T>(v[k]);
  }
}

// PIPE (bf16, small grids: one workgroup per CU): the next time block's B/C rows and
// u / delta / z are loaded into registers while the current block computes, so a block
// no longer waits on its own global loads (three round trips per block otherwise).
// S > 1 (small grids): the 16 states of a channel are split over S waves (16/S each); the
// waves' partial y sums meet in LDS and the first wave of the channel gates and stores.
// A B = 1 chunk then runs S times as many waves, each with 1/S of the state chains.
template <typename T, int K, int NW, bool PIPE = false, int S = 1>
__global__ __launch_bounds__(64 * NW) void scan_v5_kernel(const ScanParams p) {
  static_assert(K % 2 == 0, "K must be even");
  static_assert(!PIPE || sizeof(T) == 2, "the pipelined form keeps bf16 words");
  static_assert(NW % S == 0 && kMaxN % S == 0, "whole channels per workgroup");
  constexpr int TB = 64 * K;
  constexpr int K2 = K / 2;
  constexpr int NS = kMaxN / S;  // states per wave
  constexpr int NCH = NW / S;    // channels per workgroup
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sB = smem;                 // [N][K2][64][2]
  float* sC = smem + kMaxN * TB;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sg = S > 1 ? wave % S : 0;  // state group
  const int b = blockIdx.y;
  const int d_raw = blockIdx.x * NCH + wave / S;
  const bool active = d_raw < p.dim;
  const int d = active ? d_raw : p.dim - 1;
  const int N = p.dstate;
  const int L = p.seqlen;
  const int LO = p.out_len;
  const bool vx = p.vec_x != 0;

  const T* urow = static_cast<const T*>(p.u) + b * p.u_sb + d * p.u_sd;
  const T* drow = static_cast<const T*>(p.delta) + b * p.dl_sb + d * p.dl_sd;
  const T* zrow = p.z ? static_cast<const T*>(p.z) + b * p.z_sb + d * p.z_sd : nullptr;
  T* orow = static_cast<T*>(p.out) + b * p.o_sb + d * p.o_sd;
  const T* Bb = static_cast<const T*>(p.B) + b * p.b_sb;
  const T* Cb = static_cast<const T*>(p.C) + b * p.c_sb;

  float A2[NS], carry[NS];  // wave-uniform (SGPRs): this wave's states sg*NS ..
#pragma unroll
  for (int nn = 0; nn < NS; ++nn) {
    const int n = sg * NS + nn;
    A2[nn] = (n < N) ? p.A[d * N + n] * kLog2e : 0.0f;
    carry[nn] = (n < N && p.h0) ? load_dyn(p.h0, b * p.h0_sb + d * p.h0_sd + n, p.h0_dtype) : 0.0f;
  }
  const float Dv = p.D ? p.D[d] : 0.0f;
  const float bias = p.dbias ? p.dbias[d] : 0.0f;

  // B/C staging role: chunk idx = (B|C row, 8-step chunk); PIPE keeps kSt chunks per thread
  const int chunks = 2 * N * (TB / 8);
  constexpr int kSt = (2 * kMaxN * (TB / 8) + 64 * NW - 1) / (64 * NW);
  auto stage_src = [&](int idx, int t_blk, const T*& src, int& t, int& n, bool& isC) {
    const int row = idx / (TB / 8);
    const int c8 = idx - row * (TB / 8);
    isC = row >= N;
    n = isC ? row - N : row;
    src = (isC ? Cb + n * p.c_sn : Bb + n * p.b_sn);
    t = t_blk + c8 * 8;
  };
  auto stage_put = [&](int idx, const float (&w)[8]) {
    const int row = idx / (TB / 8);
    const int c8 = idx - row * (TB / 8);
    const bool isC = row >= N;
    const int n = isC ? row - N : row;
    float* base = (isC ? sC : sB) + n * TB;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const int r = c8 * 8 + j;       // block-relative step (even)
      const int ln = r / K, k = r - ln * K;
      *reinterpret_cast<float2*>(base + ((k >> 1) * 64 + ln) * 2) = make_float2(w[j], w[j + 1]);
    }
  };
  uint4 stq[PIPE ? kSt : 1];
  auto stage_fetch = [&](int t_blk) {  // PIPE: raw bf16 chunks into registers
#pragma unroll
    for (int c = 0; c < kSt; ++c) {
      const int idx = tid + c * 64 * NW;
      uint4 q = make_uint4(0, 0, 0, 0);
      if (idx < chunks) {
        const T* src; int t, n; bool isC;
        stage_src(idx, t_blk, src, t, n, isC);
        if (p.vec_bc && t + 8 <= L) {
          q = *reinterpret_cast<const uint4*>(src + t);
        } else {
          uint32_t h8[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t lo = t + 2 * j < L ? static_cast<uint32_t>(src[t + 2 * j]) : 0u;
            const uint32_t hi = t + 2 * j + 1 < L ? static_cast<uint32_t>(src[t + 2 * j + 1]) : 0u;
            h8[j] = lo | (hi << 16);
          }
          q = make_uint4(h8[0], h8[1], h8[2], h8[3]);
        }
      }
      if constexpr (PIPE) stq[c] = q;
    }
  };
  const int t0_first = lane * K;
  uint32_t nu[PIPE ? K / 2 : 1], nd[PIPE ? K / 2 : 1], nz[PIPE ? K / 2 : 1];
  auto row_fetch = [&](int t_blk) {
    if constexpr (PIPE) {
      const int t0n = t_blk + t0_first;
      load_even_raw<K>(reinterpret_cast<const bf16_t*>(urow), t0n, L, vx, nu);
      load_even_raw<K>(reinterpret_cast<const bf16_t*>(drow), t0n, L, vx, nd);
      if (zrow) load_even_raw<K>(reinterpret_cast<const bf16_t*>(zrow), t0n, L, vx, nz);
    }
  };
  if constexpr (PIPE) {
    if (LO > 0) {
      stage_fetch(0);
      row_fetch(0);
    }
  }

  for (int t_blk = 0; t_blk < LO; t_blk += TB) {
    // ---- stage B/C: thread = (B|C, state, 8-step chunk) -> four float2 writes ----
    __syncthreads();
    if constexpr (PIPE) {
#pragma unroll
      for (int c = 0; c < kSt; ++c) {
        const int idx = tid + c * 64 * NW;
        if (idx < chunks) {
          const uint32_t q4[4] = {stq[c].x, stq[c].y, stq[c].z, stq[c].w};
          float w[8];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            w[2 * j] = __uint_as_float(q4[j] << 16);
            w[2 * j + 1] = __uint_as_float(q4[j] & 0xffff0000u);
          }
          stage_put(idx, w);
        }
      }
    } else {
      for (int idx = tid; idx < chunks; idx += 64 * NW) {
        const T* src; int t, n; bool isC;
        stage_src(idx, t_blk, src, t, n, isC);
        float w[8];
        if (p.vec_bc && t + 8 <= L) {
          load8(src + t, w);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) w[j] = (t + j < L) ? to_f32(src[t + j]) : 0.0f;
        }
        stage_put(idx, w);
      }
    }
    __syncthreads();

    // ---- per-lane prologue ----
    const int t0 = t_blk + lane * K;
    float dl[K], du[K], y[K];
    uint32_t cz[PIPE ? K / 2 : 1];
    {
      float uv[K], dv[K];
      if constexpr (PIPE) {
        unpack_even<K>(nu, uv);
        unpack_even<K>(nd, dv);
#pragma unroll
        for (int j = 0; j < K / 2; ++j) cz[j] = nz[j];
        if (t_blk + TB < LO) {  // the next block's inputs land while this one computes
          stage_fetch(t_blk + TB);
          row_fetch(t_blk + TB);
        }
      } else {
        load_even<T, K>(urow, t0, L, vx, uv);
        load_even<T, K>(drow, t0, L, vx, dv);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        float dd = dv[k] + bias;
        if (p.softplus) dd = softplus_fast(dd);
        dd = (t0 + k < L) ? dd : 0.0f;
        dl[k] = dd;
        du[k] = dd * uv[k];
        y[k] = sg == 0 ? Dv * uv[k] : 0.0f;
      }
    }
    float sd = 0.0f;
#pragma unroll
    for (int k = 0; k < K; ++k) sd += dl[k];
    float srow = sd;
    srow += dppz<0x111>(srow);
    srow += dppz<0x112>(srow);
    srow += dppz<0x114>(srow);
    srow += dppz<0x118>(srow);
    const float shalf = srow + dppz<0x142, 0xa>(srow);

    // ---- states ----
#pragma unroll
    for (int nn = 0; nn < NS; ++nn) {
      const int n = sg * NS + nn;
      if (n < N) {
        const float* bs = sB + n * TB + lane * 2;
        float a[K], bb[K];
        float fold = 0.0f;
#pragma unroll
        for (int k2 = 0; k2 < K2; ++k2) {
          const float2 v = *reinterpret_cast<const float2*>(bs + k2 * 128);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int k = 2 * k2 + i;
            a[k] = __builtin_amdgcn_exp2f(dl[k] * A2[nn]);
            bb[k] = du[k] * (i ? v.y : v.x);
            fold = fmaf(a[k], fold, bb[k]);
          }
        }
        const float e1 = __builtin_amdgcn_exp2f(sd * A2[nn]);
        if (lane == 0) fold = fmaf(e1, carry[nn], fold);
        const float e2 = e1 * dppz<0x111>(e1);
        const float e4 = e2 * dppz<0x112>(e2);
        const float e8 = e4 * dppz<0x114>(e4);
        fold = fmaf(e1, dppz<0x111>(fold), fold);
        fold = fmaf(e2, dppz<0x112>(fold), fold);
        fold = fmaf(e4, dppz<0x114>(fold), fold);
        fold = fmaf(e8, dppz<0x118>(fold), fold);
        fold = fmaf(__builtin_amdgcn_exp2f(srow * A2[nn]), dppz<0x142, 0xa>(fold), fold);
        fold = fmaf(__builtin_amdgcn_exp2f(shalf * A2[nn]), dppz<0x143, 0xc>(fold), fold);
        float h = dppz<0x138>(fold);
        if (lane == 0) h = carry[nn];
        carry[nn] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fold), 63));
        const float* cs = sC + n * TB + lane * 2;
#pragma unroll
        for (int k2 = 0; k2 < K2; ++k2) {
          const float2 v = *reinterpret_cast<const float2*>(cs + k2 * 128);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int k = 2 * k2 + i;
            h = fmaf(a[k], h, bb[k]);
            y[k] = fmaf(h, i ? v.y : v.x, y[k]);
          }
        }
      }
    }

    if constexpr (S > 1) {  // partial y of the other state groups -> the channel's first wave
      float* red = smem + 2 * kMaxN * TB;  // [NW][K][64]
      if (sg != 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) red[(wave * K + k) * 64 + lane] = y[k];
      }
      __syncthreads();
      if (sg == 0) {
#pragma unroll
        for (int g = 1; g < S; ++g)
#pragma unroll
          for (int k = 0; k < K; ++k) y[k] += red[((wave + g) * K + k) * 64 + lane];
      }
    }
    if (zrow && sg == 0) {
      float zv[K];
      if constexpr (PIPE) unpack_even<K>(cz, zv);
      else load_even<T, K>(zrow, t0, L, vx, zv);
#pragma unroll
      for (int k = 0; k < K; ++k) y[k] *= silu_fast(zv[k]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) y[k] = (t0 + k < L) ? y[k] : 0.0f;
    if (active && sg == 0 && t0 < LO) store_even<T, K>(orow, t0, LO, vx, y);
  }

  if (p.hl && active && lane == 0) {
#pragma unroll
    for (int nn = 0; nn < NS; ++nn) {
      const int n = sg * NS + nn;
      if (n < N) store_dyn(p.hl, b * p.hl_sb + d * p.hl_sd + n, p.hl_dtype, carry[nn]);
    }
  }
}

// State-split form (S waves per channel, NW waves per workgroup), pipelined for bf16.
template <typename T, int K, int NW, int S>
static void launch_v5_split(const ScanParams& p, hipStream_t s) {
  const size_t lds = (2 * kMaxN * 64 * K + NW * K * 64) * sizeof(float);
  constexpr int NCH = NW / S;
  dim3 grid((p.dim + NCH - 1) / NCH, p.batch);
  hipLaunchKernelGGL((scan_v5_kernel<T, K, NW, sizeof(T) == 2, S>), grid, dim3(64 * NW), lds, s, p);
}

// pipe: -1 auto (bf16 grids of at most one workgroup per CU), 0 off, 1 on (bf16 only)
template <typename T, int K, int NW>
static void launch_v5(const ScanParams& p, hipStream_t s, int pipe = -1) {
  const size_t lds = 2 * kMaxN * 64 * K * sizeof(float);
  dim3 grid((p.dim + NW - 1) / NW, p.batch);
  const bool use_pipe = sizeof(T) == 2 && (pipe == 1 || (pipe < 0 && grid.x * grid.y <= 256));
  if constexpr (sizeof(T) == 2) {
    if (use_pipe) {
      hipLaunchKernelGGL((scan_v5_kernel<T, K, NW, true>), grid, dim3(64 * NW), lds, s, p);
      return;
    }
  }
  hipLaunchKernelGGL((scan_v5_kernel<T, K, NW>), grid, dim3(64 * NW), lds, s, p);
}

// Pick the steps-per-lane K that covers out_len with the least padded work; per block
// the scan costs about as much as 8/K of a step, so ties go to the larger K.  The LDS
// staging is 2*16*64*K fp32 (80 KB at K=10): with 8-wave workgroups two fit per CU
// (4 waves/SIMD), which caps K at 10.
template <typename T>
static void launch_v5_auto(const ScanParams& p, hipStream_t s) {
  auto cost = [&](int k) {
    const double tb = 64.0 * k;
    return ((p.out_len + tb - 1) / tb) * tb * (1.0 + 4.0 / k);
  };
  // Grids of at most one workgroup per CU (e.g. the B = 1 streaming chunk): the states
  // split over two waves per channel (variant 30).  Measured at M (D = 1152, L = 3137,
  // profiles/r01f_v5_state_split.txt): B = 1 58.0 -> 48.5 us, B = 2 equal, B >= 4 slower.
  const long long wgs = static_cast<long long>((p.dim + 7) / 8) * p.batch;
  if (sizeof(T) == 2 && wgs <= 256 && cost(10) <= cost(8)) launch_v5_split<T, 10, 10, 2>(p, s);
  else if (cost(10) <= cost(8)) launch_v5<T, 10, 8>(p, s);
  else launch_v5<T, 8, 8>(p, s);
}

// --------------------------------------------------------------------- one-token step
struct StepParams {
  void* state; const void* x; const void* dt; const float* A; const void* B; const void* C;
  const float* D; const void* z; const float* dbias; void* out;
  long long s_sb, s_sd, x_sb, dt_sb, b_sb, c_sb, z_sb, o_sb;
  int batch, dim, dstate, softplus, state_dtype;
};

template <typename T>
__global__ __launch_bounds__(256) void state_update_kernel(const StepParams p) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= p.batch * p.dim) return;
  const int b = gid / p.dim;
  const int d = gid - b * p.dim;
  const float x = to_f32(static_cast<const T*>(p.x)[b * p.x_sb + d]);
  float dt = to_f32(static_cast<const T*>(p.dt)[b * p.dt_sb + d]);
  if (p.dbias) dt += p.dbias[d];
  if (p.softplus) dt = softplus(dt);
  const T* Bp = static_cast<const T*>(p.B) + b * p.b_sb;
  const T* Cp = static_cast<const T*>(p.C) + b * p.c_sb;
  const long long sbase = b * p.s_sb + d * p.s_sd;
  float y = 0.0f;
  for (int n = 0; n < p.dstate; ++n) {
    const float s = load_dyn(p.state, sbase + n, p.state_dtype);
    const float ns = s * __expf(dt * p.A[d * p.dstate + n]) + dt * x * to_f32(Bp[n]);
    store_dyn(p.state, sbase + n, p.state_dtype, ns);
    y = fmaf(ns, to_f32(Cp[n]), y);
  }
  if (p.D) y += x * p.D[d];
  if (p.z) y *= silu(to_f32(static_cast<const T*>(p.z)[b * p.z_sb + d]));
  static_cast<T*>(p.out)[b * p.o_sb + d] = from_f32<T>(y);
}


template <typename T>
static void dispatch_scan(const ScanParams& p, hipStream_t s) {
  launch_v5_auto<T>(p, s);
}

}  // namespace vm

using namespace vm;

namespace {
// Second parameter set of a paired (bidirectional) scan; nullptr for a plain scan.
struct PairArgs {
  int split; const float* A; const float* D; const float* dbias; const void* h0; void* hl;
  int frame_len;
};
}  // namespace

static int scan_entry(
    const char* name,
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
    int batch, int dim, int seqlen, int dstate, int dtype, const PairArgs* pair,
    int segments, void* workspace, long long workspace_bytes, void* sync, long long sync_bytes,
    vm_stream_t stream) {
  if (!u || !delta || !A || !B || !C || !out) {
    vmhost::set_error("%s: null required pointer", name);
    return VM_E_INVALID;
  }
  if (batch < 0 || dim < 0 || seqlen < 0 || out_len < seqlen || dstate < 1 || dstate > kMaxN) {
    vmhost::set_error("%s: bad shape batch=%d dim=%d seqlen=%d dstate=%d "
                      "(dstate must be in [1, %d])", name, batch, dim, seqlen, dstate, kMaxN);
    return VM_E_INVALID;
  }
  if (!vmhost::dtype_ok(dtype) || (h0 && !vmhost::dtype_ok(h0_dtype)) ||
      (h_last && !vmhost::dtype_ok(hl_dtype))) {
    vmhost::set_error("%s: unsupported dtype", name);
    return VM_E_INVALID;
  }
  if (batch == 0 || dim == 0) return VM_OK;
  ScanParams p{};
  p.u = u; p.delta = delta; p.A = A; p.B = B; p.C = C; p.D = D; p.z = z; p.dbias = delta_bias;
  p.h0 = h0; p.hl = h_last; p.out = out;
  p.u_sb = u_sb; p.u_sd = u_sd; p.dl_sb = dl_sb; p.dl_sd = dl_sd;
  p.b_sb = b_sb; p.b_sn = b_sn; p.c_sb = c_sb; p.c_sn = c_sn;
  p.z_sb = z_sb; p.z_sd = z_sd; p.o_sb = o_sb; p.o_sd = o_sd;
  p.u_sl = u_sl; p.dl_sl = dl_sl; p.b_sl = b_sl; p.c_sl = c_sl; p.z_sl = z_sl; p.o_sl = o_sl;
  p.h0_sb = h0_sb; p.h0_sd = h0_sd; p.hl_sb = hl_sb; p.hl_sd = hl_sd;
  p.batch = batch; p.dim = dim; p.seqlen = seqlen; p.out_len = out_len; p.dstate = dstate;
  p.softplus = delta_softplus; p.h0_dtype = h0_dtype; p.hl_dtype = hl_dtype;
  p.split = batch;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t ws_bytes = workspace_bytes > 0 ? static_cast<size_t>(workspace_bytes) : 0;
  if (pair) {
    const int F = pair->frame_len;
    if (!pair->A || pair->split * 2 != batch || F < 1 || seqlen % F ||
        static_cast<long long>(seqlen) * F >= (1ll << 31)) {
      vmhost::set_error("%s: need batch == 2*split, A_bwd, and frame_len dividing seqlen", name);
      return VM_E_INVALID;
    }
    if (!seq_supported(p, dtype) || !seq_pair_supported(p, dtype, segments, workspace ? ws_bytes : 0)) {
      vmhost::set_error("%s: paired scans take token-major operands with 16 unit-stride states "
                        "and, when segmented, the vm_selective_scan_workspace_bytes workspace",
                        name);
      return VM_E_INVALID;
    }
    p.split = pair->split; p.A_hi = pair->A; p.D_hi = pair->D; p.dbias_hi = pair->dbias;
    p.h0_hi = pair->h0; p.hl_hi = pair->hl;
    // output row of step t: t + (L - F) - 2F floor(t / F) (reversed frame order, tokens
    // within a frame in order); floor by a reciprocal multiply, exact for L*F < 2^32
    if (F == 1) {
      p.ro_c0 = seqlen - 1; p.ro_s = -1; p.ro_c1 = 0; p.ro_m = 0u;
    } else {
      p.ro_c0 = seqlen - F; p.ro_s = 1; p.ro_c1 = 2 * F;
      p.ro_m = static_cast<unsigned>(0xffffffffu / static_cast<unsigned>(F)) + 1u;
    }
  }
  // Token-major operands (channel stride 1): channel-per-lane sequential kernels.
  if (seq_supported(p, dtype)) {
    seq_launch(p, dtype, segments, workspace, ws_bytes, sync,
               sync_bytes > 0 ? static_cast<size_t>(sync_bytes) : 0, s);
    return vmhost::launch_status(name);
  }
  // Channel-major operands (step stride 1): time-parallel kernels.
  if (u_sl != 1 || dl_sl != 1 || b_sl != 1 || c_sl != 1 || o_sl != 1 || (z && z_sl != 1)) {
    vmhost::set_error("%s: operands must have a unit channel stride "
                      "(u/delta/z/out) or a unit step stride (all operands)", name);
    return VM_E_INVALID;
  }
  const long long m = dtype == VM_DTYPE_BF16 ? 8 : 4;  // elements per 16 bytes
  auto rows_ok = [&](const void* ptr, long long s1, long long s2) {
    return ptr == nullptr || (vmhost::aligned16(ptr) && s1 % m == 0 && s2 % m == 0);
  };
  p.vec_x = rows_ok(u, u_sb, u_sd) && rows_ok(delta, dl_sb, dl_sd) && rows_ok(z, z_sb, z_sd) &&
            rows_ok(out, o_sb, o_sd);
  p.vec_bc = rows_ok(B, b_sb, b_sn) && rows_ok(C, c_sb, c_sn);
  // seqlen == 0 still launches: the block loop is empty and h_last receives h0 (or 0).
  if (dtype == VM_DTYPE_BF16) dispatch_scan<bf16_t>(p, s);
  else dispatch_scan<float>(p, s);
  return vmhost::launch_status(name);
}

#define VM_SCAN_ARGS                                                                  \
  const void *u, long long u_sb, long long u_sd, long long u_sl, const void *delta,   \
      long long dl_sb, long long dl_sd, long long dl_sl, const float *A, const void *B, \
      long long b_sb, long long b_sn, long long b_sl, const void *C, long long c_sb,     \
      long long c_sn, long long c_sl, const float *D, const void *z, long long z_sb,     \
      long long z_sd, long long z_sl, const float *delta_bias, int delta_softplus,       \
      const void *h0, int h0_dtype, long long h0_sb, long long h0_sd, void *h_last,      \
      int hl_dtype, long long hl_sb, long long hl_sd, void *out, long long o_sb,         \
      long long o_sd, long long o_sl, int out_len, int batch, int dim, int seqlen,       \
      int dstate, int dtype
#define VM_SCAN_PASS                                                                  \
  u, u_sb, u_sd, u_sl, delta, dl_sb, dl_sd, dl_sl, A, B, b_sb, b_sn, b_sl, C, c_sb, c_sn, \
      c_sl, D, z, z_sb, z_sd, z_sl, delta_bias, delta_softplus, h0, h0_dtype, h0_sb,      \
      h0_sd, h_last, hl_dtype, hl_sb, hl_sd, out, o_sb, o_sd, o_sl, out_len, batch, dim,  \
      seqlen, dstate, dtype

extern "C" int vm_selective_scan_fwd(VM_SCAN_ARGS, int segments, void* workspace,
                                     long long workspace_bytes, void* sync,
                                     long long sync_bytes, vm_stream_t stream) {
  return scan_entry("vm_selective_scan_fwd", VM_SCAN_PASS, nullptr, segments, workspace,
                    workspace_bytes, sync, sync_bytes, stream);
}

extern "C" int vm_selective_scan_bidir_fwd(VM_SCAN_ARGS, int split, const float* A_bwd,
                                           const float* D_bwd, const float* delta_bias_bwd,
                                           const void* h0_bwd, void* h_last_bwd, int frame_len,
                                           int segments, void* workspace,
                                           long long workspace_bytes, void* sync,
                                           long long sync_bytes, vm_stream_t stream) {
  const PairArgs pair{split, A_bwd, D_bwd, delta_bias_bwd, h0_bwd, h_last_bwd, frame_len};
  return scan_entry("vm_selective_scan_bidir_fwd", VM_SCAN_PASS, &pair, segments, workspace,
                    workspace_bytes, sync, sync_bytes, stream);
}
#undef VM_SCAN_ARGS
#undef VM_SCAN_PASS

extern "C" int vm_selective_scan_dtproj_fwd(
    const void* u, long long u_sb, long long u_sd, long long u_sl, const void* dt_low,
    long long dtl_sb, long long dtl_sl, int dt_rank, const void* w_dt, int w_dt_ld,
    const float* A, const void* B, long long b_sb, long long b_sn, long long b_sl,
    const void* C, long long c_sb, long long c_sn, long long c_sl, const float* D,
    const void* z, long long z_sb, long long z_sd, long long z_sl, const float* delta_bias,
    int delta_softplus, const void* h0, int h0_dtype, long long h0_sb, long long h0_sd,
    void* h_last, int hl_dtype, long long hl_sb, long long hl_sd, void* out, long long o_sb,
    long long o_sd, long long o_sl, int out_len, int batch, int dim, int seqlen, int dstate,
    int dtype, int segments, void* workspace, long long workspace_bytes, void* sync,
    long long sync_bytes, vm_stream_t stream) {
  const char* name = "vm_selective_scan_dtproj_fwd";
  if (!u || !dt_low || !w_dt || !A || !B || !C || !z || !out) {
    vmhost::set_error("%s: null required pointer", name);
    return VM_E_INVALID;
  }
  if (batch < 0 || dim < 0 || seqlen < 0 || out_len < seqlen || dstate != kMaxN ||
      (h0 && !vmhost::dtype_ok(h0_dtype)) || (h_last && !vmhost::dtype_ok(hl_dtype))) {
    vmhost::set_error("%s: bad shape or state dtype (dstate must be %d)", name, kMaxN);
    return VM_E_INVALID;
  }
  if (batch == 0 || dim == 0) return VM_OK;
  ScanParams p{};
  p.u = u; p.delta = nullptr; p.A = A; p.B = B; p.C = C; p.D = D; p.z = z; p.dbias = delta_bias;
  p.h0 = h0; p.hl = h_last; p.out = out;
  p.u_sb = u_sb; p.u_sd = u_sd; p.dl_sb = 0; p.dl_sd = 1;
  p.b_sb = b_sb; p.b_sn = b_sn; p.c_sb = c_sb; p.c_sn = c_sn;
  p.z_sb = z_sb; p.z_sd = z_sd; p.o_sb = o_sb; p.o_sd = o_sd;
  p.u_sl = u_sl; p.dl_sl = 0; p.b_sl = b_sl; p.c_sl = c_sl; p.z_sl = z_sl; p.o_sl = o_sl;
  p.h0_sb = h0_sb; p.h0_sd = h0_sd; p.hl_sb = hl_sb; p.hl_sd = hl_sd;
  p.batch = batch; p.dim = dim; p.seqlen = seqlen; p.out_len = out_len; p.dstate = dstate;
  p.softplus = delta_softplus; p.h0_dtype = h0_dtype; p.hl_dtype = hl_dtype;
  p.split = batch;
  DtpArgs q{};
  q.dtl = static_cast<const bf16_t*>(dt_low); q.dtl_sb = dtl_sb; q.dtl_sl = dtl_sl;
  q.wdt = static_cast<const bf16_t*>(w_dt); q.wdt_ld = w_dt_ld; q.dt_rank = dt_rank;
  if (segments < 0 || workspace_bytes < 0 || sync_bytes < 0) {
    vmhost::set_error("%s: negative segments / workspace / sync size", name);
    return VM_E_INVALID;
  }
  // the segmented form when the cost model (or `segments`) asks for one: dt_proj inside the
  // chunked scan, in conv_proj's arithmetic (ABI v11)
  if (seq_chunk_steps(batch, dim, seqlen, segments) > 0) {
    if (!seq_dtp_chunk_supported(p, q, dtype, segments, static_cast<size_t>(workspace_bytes)) ||
        !workspace) {
      vmhost::set_error("%s: the segmented form needs bf16 token-major operands with z, "
                        "softplus, 16 states, C directly after B in the x_dbl rows, segments of "
                        "at most 64 steps (vm_selective_scan_chunk_steps), a (dim, 32 | 64) W_dt "
                        "with dt_rank <= its width and a multiple of 4, and the workspace of "
                        "vm_selective_scan_workspace_bytes", name);
      return VM_E_INVALID;
    }
    seq_dtp_chunk_launch(p, q, segments, workspace, static_cast<size_t>(workspace_bytes), sync,
                         static_cast<size_t>(sync_bytes), static_cast<hipStream_t>(stream));
    return vmhost::launch_status(name);
  }
  if (!seq_dtp_supported(p, q, dtype, dt_rank)) {
    vmhost::set_error("%s: needs bf16 token-major operands with z, softplus, 16 states, C "
                      "directly after B in the x_dbl rows, dim %% 128 == 0, dt_rank <= 64 and a multiple of 4, "
                      "8-byte aligned dt_low rows and a (dim, >= 16*ceil(r/16)) W_dt", name);
    return VM_E_INVALID;
  }
  seq_dtp_launch(p, q, dt_rank, static_cast<hipStream_t>(stream));
  return vmhost::launch_status(name);
}

extern "C" int vm_selective_scan_chunk_steps(int batch, int dim, int seqlen, int dstate,
                                             int segments) {
  if (batch <= 0 || dim <= 0 || seqlen < 0 || dstate < 1 || dstate > kMaxN || segments < 0)
    return 0;
  return seq_chunk_steps(batch, dim, seqlen, segments);
}

extern "C" long long vm_selective_scan_workspace_bytes(int batch, int dim, int seqlen,
                                                       int dstate, int segments) {
  if (batch <= 0 || dim <= 0 || seqlen < 0 || dstate < 1 || dstate > kMaxN) return 0;
  return static_cast<long long>(seq_workspace_bytes(batch, dim, seqlen, segments, nullptr));
}

extern "C" long long vm_selective_scan_sync_bytes(int batch, int dim, int seqlen, int dstate,
                                                  int segments) {
  if (batch <= 0 || dim <= 0 || seqlen < 0 || dstate < 1 || dstate > kMaxN) return 0;
  return static_cast<long long>(seq_sync_bytes(batch, dim, seqlen, segments));
}

// Host-side read of a sync buffer's sticky error word (a host copy of at least its first
// kSyncHeaderWords words): 0 = every one-launch scan that used the buffer handed its block
// aggregates on in time, 1 = some block's bounded wait ran out (its outputs are NaN).
extern "C" int vm_selective_scan_sync_status(const void* sync_host, long long bytes) {
  if (!sync_host || bytes < static_cast<long long>(kSyncHeaderWords * sizeof(unsigned))) {
    vmhost::set_error("vm_selective_scan_sync_status: need a host copy of the sync header "
                      "(%d bytes)", static_cast<int>(kSyncHeaderWords * sizeof(unsigned)));
    return VM_E_INVALID;
  }
  return static_cast<const unsigned*>(sync_host)[0] != 0u ? 1 : 0;
}

extern "C" int vm_selective_state_update(void* state, int state_dtype, long long s_sb, long long s_sd,
                                         const void* x, long long x_sb, const void* dt, long long dt_sb,
                                         const float* A, const void* B, long long b_sb,
                                         const void* C, long long c_sb, const float* D,
                                         const void* z, long long z_sb, const float* dt_bias,
                                         int dt_softplus, void* out, long long o_sb,
                                         int batch, int dim, int dstate, int dtype,
                                         vm_stream_t stream) {
  if (!state || !x || !dt || !A || !B || !C || !out) {
    vmhost::set_error("vm_selective_state_update: null required pointer");
    return VM_E_INVALID;
  }
  if (batch < 0 || dim < 0 || dstate < 1 || !vmhost::dtype_ok(dtype) ||
      !vmhost::dtype_ok(state_dtype)) {
    vmhost::set_error("vm_selective_state_update: bad shape or dtype");
    return VM_E_INVALID;
  }
  if (batch == 0 || dim == 0) return VM_OK;
  StepParams p{};
  p.state = state; p.x = x; p.dt = dt; p.A = A; p.B = B; p.C = C; p.D = D; p.z = z;
  p.dbias = dt_bias; p.out = out;
  p.s_sb = s_sb; p.s_sd = s_sd; p.x_sb = x_sb; p.dt_sb = dt_sb; p.b_sb = b_sb; p.c_sb = c_sb;
  p.z_sb = z_sb; p.o_sb = o_sb;
  p.batch = batch; p.dim = dim; p.dstate = dstate; p.softplus = dt_softplus;
  p.state_dtype = state_dtype;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int n = batch * dim;
  dim3 grid((n + 255) / 256);
  if (dtype == VM_DTYPE_BF16)
    hipLaunchKernelGGL(state_update_kernel<bf16_t>, grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(state_update_kernel<float>, grid, dim3(256), 0, s, p);
  return vmhost::launch_status("vm_selective_state_update");
}
