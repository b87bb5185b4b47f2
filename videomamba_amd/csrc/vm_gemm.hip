// Small-M projection GEMM for the streaming-chunk latency path: out = x @ w^T (+ bias),
// bf16 operands, fp32 accumulation on v_mfma_f32_16x16x32_bf16, bf16 out.  Replaces the
// mixer's in_proj / out_proj nn.Linear calls (mamba_simple.py:333-339, :445-446) when the
// token count is one clip's (B = 1: M = 3144 rows).  There the library's 256x128 tiles give
// ~1 workgroup per CU and each walks the whole K serially (14-15 us per projection);
// 128x128 / 64x128 tiles put 2-4 workgroups on every CU.
//
// Layout: x (m, k) and w (n, k) both K-contiguous (the nn.Linear layouts), out (m, n).
// A workgroup (4 waves, 2 x 2) owns a BM x 128 output tile and walks K in 64-wide steps:
// A / W pieces are fetched two steps ahead into two register slots while the current
// step's MFMAs run from LDS (double-buffered, one barrier per step).  The tile leaves
// through LDS as 16-byte row stores.  Each output row's dot products run in the same order
// whatever m is, so a row's bits do not depend on the sequence length (chunked == full).

#include "vm_common.h"

namespace vm {

typedef __attribute__((__vector_size__(8 * sizeof(short)))) short bf16x8_t;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4_t;

struct LinParams {
  const bf16_t* x; long long ldx;
  const bf16_t* w; long long ldw;
  const float* bias;
  bf16_t* out; long long ldo;
  int m, n, k;
};

// Fused residual add + RMSNorm of the NEXT block (videomamba.py:141-166 with
// fused_add_norm / rms_norm / residual_in_fp32): after the GEMM, out (= h, the block's
// output rounded to bf16) is complete for a 16-row granule once every column tile of the
// grid has stored its part; the workgroup whose counter add comes last normalises the
// granule:  res += h (fp32, in place);  hn = bf16(res * rsqrt(mean(res^2) + eps) * w).
// Hand-off (MI355X_MICROARCH.md cross-workgroup table, row 1): every h store is sc1, each
// storing wave waits vmcnt(0), a workgroup barrier, then ONE lane per granule adds to the
// granule's counter (agent-scope atomic); the last adder's waves read h with sc1 loads after
// a barrier.  The last adder also resets the counter, so the buffer is zero after a launch.
struct NormTail {
  float* res;         // (m, n) fp32, row stride ldr: read and updated in place
  long long ldr;
  const float* w;     // (n) fp32 norm weight
  bf16_t* hn;         // (m, n) bf16 normalised output, row stride ldh
  long long ldh;
  float eps;
  unsigned* cnt;      // ceil(m / 16) zeroed counters
};
constexpr int kNormGran = 16;  // rows per hand-off granule
constexpr int kSC1 = 16;       // buffer cache-policy bit: sc1 (agent-coherent)

__device__ __forceinline__ float lin_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int kLinBN = 128;
constexpr int kLinBK = 64;
constexpr int kLinPitch = 72;  // bf16 per staged row: 64 + 8 pad (144 B)

template <int BM, int NK, bool NORM = false>  // NK = k / 64 K-steps, fully unrolled
__global__ __launch_bounds__(256) void linear_kernel(const LinParams p, const NormTail q) {
  constexpr int BN = kLinBN, BK = kLinBK, PITCH = kLinPitch;
  constexpr int WM = BM / 2, WN = BN / 2;  // wave tile
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int KQ = BK / 8;                                      // 16-B pieces per row
  constexpr int AP = BM * KQ / 256, BP = BN * KQ / 256;           // pieces per thread
  constexpr int kStage = (BM + BN) * PITCH;                       // bf16 per LDS stage
  constexpr int kOutPitch = BN + 8;
  static_assert(BM * kOutPitch <= 2 * kStage, "output tile must fit the staging buffers");
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];   // [2][kStage]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  constexpr int nk = NK;

  // Operands come in through buffer loads: rows past m (or n) fall outside the buffer's
  // byte range and read as 0 with no branch, so every load of a step is issued back to back
  // and waited for only where its registers go to LDS.  Two register slots: the loads for
  // step s are issued at the top of step s - 2 and land in LDS at the end of step s - 1.
  const auto xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p.x), 0, static_cast<int>((long long)p.m * p.ldx * 2), 0x00020000);
  const auto wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p.w), 0, static_cast<int>((long long)p.n * p.ldw * 2), 0x00020000);
  typedef __attribute__((__vector_size__(4 * sizeof(int)))) int i32x4_t;
  i32x4_t ra0[AP], rb0[BP], ra1[AP], rb1[BP];
  auto gload = [&](int kt, i32x4_t (&a)[AP], i32x4_t (&b)[BP]) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int pc = tid + 256 * i, row = pc / KQ, kq = pc % KQ;
      const int off = ((m0 + row) * static_cast<int>(p.ldx) + k0 + kq * 8) * 2;
      a[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int pc = tid + 256 * i, row = pc / KQ, kq = pc % KQ;
      const int off = ((n0 + row) * static_cast<int>(p.ldw) + k0 + kq * 8) * 2;
      b[i] = __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0);
    }
  };
  auto lstore = [&](int buf, const i32x4_t (&a)[AP], const i32x4_t (&b)[BP]) {
    bf16_t* sA = smem + buf * kStage;
    bf16_t* sB = sA + BM * PITCH;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int pc = tid + 256 * i;
      *reinterpret_cast<i32x4_t*>(&sA[(pc / KQ) * PITCH + (pc % KQ) * 8]) = a[i];
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int pc = tid + 256 * i;
      *reinterpret_cast<i32x4_t*>(&sB[(pc / KQ) * PITCH + (pc % KQ) * 8]) = b[i];
    }
  };
  // workgroup barrier that waits only for this wave's LDS traffic: __syncthreads() also
  // drains vmcnt, which would collapse the two-step prefetch to zero
  auto lds_barrier = [&]() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const bf16_t* sA = smem + buf * kStage;
    const bf16_t* sB = sA + BM * PITCH;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8_t af[TM], bw[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(
            &sA[(wm * WM + i * 16 + (lane & 15)) * PITCH + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bw[j] = *reinterpret_cast<const bf16x8_t*>(
            &sB[(wn * WN + j * 16 + (lane & 15)) * PITCH + ks * 32 + (lane >> 4) * 8]);
      __builtin_amdgcn_sched_barrier(0);  // all fragment reads in flight before the MFMAs
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bw[j], acc[i][j], 0, 0, 0);
    }
  };

  gload(0, ra0, rb0);
  if (nk > 1) gload(1, ra1, rb1);
  lstore(0, ra0, rb0);
  lds_barrier();
#pragma unroll
  for (int kt = 0; kt < nk; ++kt) {  // fully unrolled: slots and waits are static
    // (sched_barrier: keep the step's loads at its top — the scheduler otherwise sinks
    // them to the end of the step, which leaves one step of prefetch instead of two)
    if (kt & 1) {
      if (kt + 2 < nk) gload(kt + 2, ra1, rb1);  // slot 1 held step kt, already in LDS
      __builtin_amdgcn_sched_barrier(0);
      compute(1);
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nk) lstore(0, ra0, rb0);
    } else {
      if (kt + 2 < nk) gload(kt + 2, ra0, rb0);
      __builtin_amdgcn_sched_barrier(0);
      compute(0);
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nk) lstore(1, ra1, rb1);
    }
    lds_barrier();
  }

  // epilogue: D[4(lane/16) + r][lane % 16] of every 16x16 tile -> LDS -> 16-B row stores
  // (the loop's last barrier has every wave past its final LDS reads)
  bf16_t* sO = smem;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WN + j * 16 + (lane & 15);
      const float b = p.bias && n0 + col < p.n ? p.bias[n0 + col] : 0.0f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * WM + i * 16 + (lane >> 4) * 4 + r;
        sO[row * kOutPitch + col] = from_f32<bf16_t>(acc[i][j][r] + b);
      }
    }
  __syncthreads();
  constexpr int kPieces = BM * BN / 8;
  const auto hr = __builtin_amdgcn_make_buffer_rsrc(
      p.out, 0, static_cast<int>((long long)p.m * p.ldo * 2), 0x00020000);
#pragma unroll
  for (int i = 0; i < kPieces / 256; ++i) {
    const int pc = tid + 256 * i, row = pc / (BN / 8), cq = pc % (BN / 8);
    const int gm = m0 + row, gn = n0 + cq * 8;
    if (gm < p.m && gn < p.n) {
      const uint4 v = *reinterpret_cast<const uint4*>(&sO[row * kOutPitch + cq * 8]);
      if constexpr (NORM) {  // agent-coherent: another workgroup normalises these rows
        typedef __attribute__((__vector_size__(4 * sizeof(int)))) int v4i;
        __builtin_amdgcn_raw_buffer_store_b128(v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w}, hr,
                                               (gm * static_cast<int>(p.ldo) + gn) * 2, 0, kSC1);
      } else {
        *reinterpret_cast<uint4*>(p.out + (long long)gm * p.ldo + gn) = v;
      }
    }
  }
  if constexpr (NORM) {
    // ---- hand-off: the last column tile of a 16-row granule normalises it ----
    __shared__ int s_last[BM / kNormGran];
    __builtin_amdgcn_s_waitcnt(0);  // this wave's h stores are acknowledged
    __syncthreads();
    const int ntn = (p.n + BN - 1) / BN;
    if (tid < BM / kNormGran) {
      const int g = m0 / kNormGran + tid;
      int last = 0;
      if (g * kNormGran < p.m) {
        const unsigned old =
            __hip_atomic_fetch_add(&q.cnt[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = old == static_cast<unsigned>(ntn - 1);
        if (last) __hip_atomic_store(&q.cnt[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      s_last[tid] = last;
    }
    __syncthreads();
    // per row: vm_add_norm_fwd's RMS arithmetic and lane -> chunk map (lane*4 + 256*j), so
    // the fused result is bit-identical to out_proj followed by vm_add_norm_fwd
    constexpr int CPL = 4;  // n <= 1024
#pragma unroll 1
    for (int gi = 0; gi < BM / kNormGran; ++gi) {
      if (!s_last[gi]) continue;
#pragma unroll 1
      for (int rr = 0; rr < kNormGran / 4; ++rr) {
        const int gm = m0 + gi * kNormGran + wave * (kNormGran / 4) + rr;
        if (gm >= p.m) break;
        float v[CPL][4];
        float* rrow = q.res + (long long)gm * q.ldr;
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
          const int c = lane * 4 + 256 * j;
          if (c < p.n) {
            const auto hv = __builtin_amdgcn_raw_buffer_load_b64(
                hr, (gm * static_cast<int>(p.ldo) + c) * 2, 0, kSC1);
            const float4 r = *reinterpret_cast<const float4*>(rrow + c);
            v[j][0] = __uint_as_float(hv[0] << 16) + r.x;
            v[j][1] = __uint_as_float(hv[0] & 0xffff0000u) + r.y;
            v[j][2] = __uint_as_float(hv[1] << 16) + r.z;
            v[j][3] = __uint_as_float(hv[1] & 0xffff0000u) + r.w;
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[j][i] = 0.0f;
          }
        }
        float sq = 0.0f;
#pragma unroll
        for (int j = 0; j < CPL; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) sq = fmaf(v[j][i], v[j][i], sq);
        const float rstd = rsqrtf(lin_wave_sum(sq) / p.n + q.eps);
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
          const int c = lane * 4 + 256 * j;
          if (c < p.n) {
            const float4 w = *reinterpret_cast<const float4*>(q.w + c);
            const float y0 = (v[j][0] - 0.0f) * rstd * w.x, y1 = (v[j][1] - 0.0f) * rstd * w.y;
            const float y2 = (v[j][2] - 0.0f) * rstd * w.z, y3 = (v[j][3] - 0.0f) * rstd * w.w;
            *reinterpret_cast<uint2*>(q.hn + (long long)gm * q.ldh + c) = uint2{
                static_cast<uint32_t>(from_f32<bf16_t>(y0)) |
                    (static_cast<uint32_t>(from_f32<bf16_t>(y1)) << 16),
                static_cast<uint32_t>(from_f32<bf16_t>(y2)) |
                    (static_cast<uint32_t>(from_f32<bf16_t>(y3)) << 16)};
            *reinterpret_cast<float4*>(rrow + c) = make_float4(v[j][0], v[j][1], v[j][2], v[j][3]);
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------- LDS-DMA pipelined form
// The same GEMM (same per-row K order: 64-wide steps, two 16x16x32 MFMAs per step in k
// order, so every output row is bit-identical to linear_kernel's whatever the tile shape)
// with the operand tiles staged global -> LDS by buffer_load ... lds (no VGPR round trip,
// no ds_write pass) into NBUF stage buffers, NBUF - 1 steps in flight across the raw
// s_barrier (counted vmcnt, never 0 in the loop; cdna_hip_programming.md §5 "Pipelining
// across barriers").  linear_kernel's register ring keeps one step in flight and its
// barrier drains vmcnt, so at B = 1 (M = 3144) each of its K steps waited out an L2 round
// trip: in_proj (N = 2304, K = 576) ran 24.7 us against ~4 us of MFMA work.
// LDS image per stage: [BM rows | BN rows] x 128 B (64 bf16 of K), 16-byte chunks
// XOR-swizzled by (row / 2) & 7 so a 16-row fragment read touches every 16-byte slot of
// the 256-byte bank row once; the swizzle is applied to the per-lane SOURCE address (the
// DMA writes lane-linear).  Rows past m / n read as zero (buffer range) and are never
// stored.  Workgroups are renumbered so each XCD owns a contiguous run of M tiles (their x
// rows enter one L2 once; W is read by every XCD).
constexpr int kDmaRow = 128;  // bytes per staged row

__device__ __forceinline__ int dma_slot(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
// s_waitcnt vmcnt(N) lgkmcnt(0) (expcnt left at its maximum)
template <int N>
__device__ __forceinline__ void dma_wait_vm_lgkm0() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0070);
}

// NWM = wave rows (2: 4 waves in 2 x 2; 4: 8 waves in 4 x 2, two per SIMD at one workgroup
// per CU — a wave's MFMA / LDS-read latency then has a partner to hide behind)
template <int BM, int BN, int NK, int NBUF, int NWM = 2>
__global__ __launch_bounds__(128 * NWM) void linear_dma_kernel(const LinParams p) {
  constexpr int R = kDmaRow;
  constexpr int NW = 2 * NWM;     // waves
  constexpr int NT = 64 * NW;     // threads
  constexpr int STAGE = (BM + BN) * R;
  constexpr int WM = BM / NWM, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int GA = BM * R / (1024 * NW), GB = BN * R / (1024 * NW);  // DMA instr. per wave per stage
  constexpr int G = GA + GB;
  static_assert(NBUF >= 2 && NBUF <= 4, "one to three stages in flight");
  static_assert(TM * 16 == WM && TN * 16 == WN, "wave tiles of whole 16 x 16 blocks");
  static_assert(GA * 1024 * NW == BM * R && GB * 1024 * NW == BN * R,
                "tile rows must fill whole DMA rounds");
  constexpr int kOutPitch = BN + 8;
  static_assert(BM * kOutPitch * 2 <= NBUF * STAGE, "output tile must fit the stage buffers");
  extern __shared__ __attribute__((aligned(16))) char dsm[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // bijective XCD-contiguous renumbering of the linear workgroup id (N tiles fastest)
  const int ntn = gridDim.y;
  const int nwg = gridDim.x * gridDim.y;
  const int h = blockIdx.x + gridDim.x * blockIdx.y;
  const int xcd = h & 7, qq = nwg >> 3, rr = nwg & 7;
  const int l = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (h >> 3);
  const int m0 = (l / ntn) * BM, n0 = (l % ntn) * BN;

  const auto xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p.x), 0, static_cast<int>((long long)p.m * p.ldx * 2), 0x00020000);
  const auto wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p.w), 0, static_cast<int>((long long)p.n * p.ldw * 2), 0x00020000);
  // per-lane source byte offsets (at k = 0) of this wave's DMA instructions
  int aoff[GA], boff[GB];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int o = (wave * GA + i) * 1024 + lane * 16;
    const int row = o / R, chunk = dma_slot(row, (o % R) >> 4);
    aoff[i] = ((m0 + row) * static_cast<int>(p.ldx)) * 2 + chunk * 16;
  }
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int o = (wave * GB + i) * 1024 + lane * 16;
    const int row = o / R, chunk = dma_slot(row, (o % R) >> 4);
    boff[i] = ((n0 + row) * static_cast<int>(p.ldw)) * 2 + chunk * 16;
  }
  auto issue = [&](int kt, int buf) {
    char* sa = dsm + buf * STAGE;
#pragma unroll
    for (int i = 0; i < GA; ++i)
      dma16(xr, sa + (wave * GA + i) * 1024, aoff[i] + kt * R);
    char* sb = sa + BM * R;
#pragma unroll
    for (int i = 0; i < GB; ++i)
      dma16(wr, sb + (wave * GB + i) * 1024, boff[i] + kt * R);
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const char* sA = dsm + buf * STAGE;
    const char* sB = sA + BM * R;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[TM], bw[TN];
      const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8_t*>(sA + row * R + dma_slot(row, chunk) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + (lane & 15);
        bw[j] = *reinterpret_cast<const bf16x8_t*>(sB + row * R + dma_slot(row, chunk) * 16);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bw[j], acc[i][j], 0, 0, 0);
    }
  };

#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s)
    if (s < NK) issue(s, s);
#pragma unroll
  for (int kt = 0; kt < NK; ++kt) {
    // stage kt's DMA (this wave's share) has landed once at most the stages issued after
    // it are outstanding; the barrier then covers every wave's share, and every wave is
    // past its reads of the buffer the next issue overwrites (stage kt - 1's)
    constexpr int kMaxAfter = NBUF - 2;
    const int after = (kt + kMaxAfter < NK ? kMaxAfter : NK - 1 - kt);
    // (lgkmcnt(0) too: this wave's fragment reads of the buffer the issue below refills
    // have completed before it arrives; the signal fences keep the compiler from moving
    // LDS accesses across the barrier)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (after >= 2) dma_wait_vm_lgkm0<2 * G>();
    else if (after == 1) dma_wait_vm_lgkm0<G>();
    else dma_wait_vm_lgkm0<0>();
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (kt + NBUF - 1 < NK) issue(kt + NBUF - 1, (kt + NBUF - 1) % NBUF);
    compute(kt % NBUF);
  }

  // epilogue: D[4(lane/16) + r][lane % 16] of every 16x16 tile -> LDS -> 16-B row stores
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();  // every wave is past its last fragment reads
  bf16_t* sO = reinterpret_cast<bf16_t*>(dsm);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WN + j * 16 + (lane & 15);
      const float b = p.bias && n0 + col < p.n ? p.bias[n0 + col] : 0.0f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * WM + i * 16 + (lane >> 4) * 4 + r;
        sO[row * kOutPitch + col] = from_f32<bf16_t>(acc[i][j][r] + b);
      }
    }
  __syncthreads();
  constexpr int kPieces = BM * BN / 8;
#pragma unroll
  for (int i = 0; i < (kPieces + NT - 1) / NT; ++i) {
    const int pc = tid + NT * i;
    if (kPieces % NT != 0 && pc >= kPieces) break;
    const int row = pc / (BN / 8), cq = pc % (BN / 8);
    const int gm = m0 + row, gn = n0 + cq * 8;
    if (gm < p.m && gn < p.n)
      *reinterpret_cast<uint4*>(p.out + (long long)gm * p.ldo + gn) =
          *reinterpret_cast<const uint4*>(&sO[row * kOutPitch + cq * 8]);
  }
}

// Tile choice for the pipelined form (row bits do not depend on it), measured at the B = 1
// chunk shapes (scripts/diag/variant_linear.py): wide outputs (in_proj, N = 2 * d_inner)
// on 128 x 128 tiles with two stage buffers (64 KB: two workgroups per CU; 14.1 us against
// 17.6 for linear_kernel, three buffers 16.3), eight waves each since round 4 (four per
// SIMD with the second workgroup: 13.2 against 14.3-14.7 us, B = 2 21.9 against 22.9;
// 256 x 128 / 128 x 256 tiles at one workgroup per CU, 8 or 16 waves, 14.2-14.3 us;
// profiles/r04x_linear_waves.jsonl); narrow ones (out_proj, N = d_model) on 128 x 64
// tiles with three buffers (72 KB; 9.1 against 11.3 us), eight waves since round 4 (B = 1
// the same 9.4 us, B = 2 12.5-13.0 against 13.2-13.4; profiles/r04z_out_proj_waves.jsonl).
#define VM_LDMA_TILE(BMV, BNV, NBV, NWMV)                                                     \
  {                                                                                           \
    const dim3 grid((p.m + BMV - 1) / BMV, (p.n + BNV - 1) / BNV);                            \
    const size_t lds = static_cast<size_t>(NBV) * (BMV + BNV) * kDmaRow;                      \
    switch (p.k / kLinBK) {                                                                   \
      VM_LDMA_K(BMV, BNV, NBV, NWMV, 3) VM_LDMA_K(BMV, BNV, NBV, NWMV, 6)                     \
      VM_LDMA_K(BMV, BNV, NBV, NWMV, 9) VM_LDMA_K(BMV, BNV, NBV, NWMV, 12)                    \
      VM_LDMA_K(BMV, BNV, NBV, NWMV, 18) VM_LDMA_K(BMV, BNV, NBV, NWMV, 24)                   \
      default: break;                                                                         \
    }                                                                                         \
  }
#define VM_LDMA_K(BMV, BNV, NBV, NWMV, NKV)                                                    \
  case NKV:                                                                                    \
    hipLaunchKernelGGL((linear_dma_kernel<BMV, BNV, NKV, NBV, NWMV>), grid, dim3(128 * NWMV), \
                       lds, s, p);                                                             \
    break;
static void linear_dma_launch(const LinParams& p, hipStream_t s) {
  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)
  else VM_LDMA_TILE(128, 64, 3, 4)
}
#undef VM_LDMA_K
#undef VM_LDMA_TILE

// The persistent 256-row tile kernel (vm_gemm_tile.hip): bit-identical rows, used once the
// tile count fills every CU several times over.
int gemm_tile_bn(int m, int n, int k, long long ldx, long long ldw, long long ldo);
long long gemm_tile_count(int m, int n, int bn);
void gemm_tile_launch(const bf16_t* x, long long ldx, const bf16_t* w, long long ldw,
                      bf16_t* out, long long ldo, int m, int n, int k, int bn, int workgroups,
                      hipStream_t s);
// the persistent kernel runs from 1.5 tiles per CU (twice the tile count >= 3 x CUs): C5's
// in_proj (12,544 rows, 441 tiles) 41.9 -> ~35 us, the C5 chunk 8.55 -> 8.26 ms
constexpr int kTileMinPerCU2 = 3;

// CUs of the device that owns `stream` (the current device for the null stream), cached per
// device id; 0 when it cannot be queried
static int device_cus(hipStream_t stream) {
  static int cus[64] = {0};
  int dev = 0;
  if (stream) {
    if (hipStreamGetDevice(stream, &dev) != hipSuccess) return 0;
  } else if (hipGetDevice(&dev) != hipSuccess) {
    return 0;
  }
  if (dev < 0 || dev >= 64) return 0;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cus[dev] = n;
  }
  return cus[dev];
}

}  // namespace vm

using namespace vm;

extern "C" int vm_linear_fwd(const void* x, long long ldx, const void* w, long long ldw,
                             const float* bias, void* out, long long ldo, int m, int n, int k,
                             int dtype, vm_stream_t stream) {
  return vm_linear_fwd_form(x, ldx, w, ldw, bias, out, ldo, m, n, k, dtype, 0, stream);
}

extern "C" int vm_linear_fwd_form(const void* x, long long ldx, const void* w, long long ldw,
                                  const float* bias, void* out, long long ldo, int m, int n,
                                  int k, int dtype, int form, vm_stream_t stream) {
  if (!x || !w || !out) {
    vmhost::set_error("vm_linear_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (form < 0 || form > 2) {
    vmhost::set_error("vm_linear_fwd_form: form %d (0 auto, 1 LDS-DMA tiles, 2 persistent)", form);
    return VM_E_INVALID;
  }
  if (dtype != VM_DTYPE_BF16 || m < 0 || n < 1 || k < kLinBK || n % 8 || k % kLinBK ||
      ldx < k || ldw < k || ldo < n || ldx % 8 || ldw % 8 || ldo % 8 || !vmhost::aligned16(x) ||
      !vmhost::aligned16(w) || !vmhost::aligned16(out) || (long long)n * ldw * 2 >= (1ll << 31)) {
    vmhost::set_error("vm_linear_fwd: bf16 only; k a multiple of 64; n and the leading "
                      "dimensions multiples of 8; 16-byte aligned operands, w under 2 GB");
    return VM_E_INVALID;
  }
  switch (k / kLinBK) {  // the unrolled K-step counts both kernel forms are built for
    case 3: case 6: case 9: case 12: case 18: case 24: break;
    default:
      vmhost::set_error("vm_linear_fwd: k = %d (supported: 192, 384, 576, 768, 1152, 1536)", k);
      return VM_E_INVALID;
  }
  if (m == 0) return VM_OK;
  LinParams p{};
  p.x = static_cast<const bf16_t*>(x); p.ldx = ldx;
  p.w = static_cast<const bf16_t*>(w); p.ldw = ldw;
  p.bias = bias; p.out = static_cast<bf16_t*>(out); p.ldo = ldo;
  p.m = m; p.n = n; p.k = k;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int bn = bias ? 0 : gemm_tile_bn(m, n, k, ldx, ldw, ldo);
  if (form == 2 && !bn) {
    vmhost::set_error("vm_linear_fwd_form: the persistent form needs no bias, n a multiple of "
                      "192 or 256 and 256-row ranges under 2 GB");
    return VM_E_INVALID;
  }
  if (form != 1 && bn) {
    const int wgs = device_cus(s) / 8 * 8;  // persistent workgroups: whole XCD runs
    if (form == 2 && wgs < 8) {
      vmhost::set_error("vm_linear_fwd_form: the persistent form needs the launch device's CU "
                        "count (query failed or < 8 CUs)");
      return VM_E_INVALID;
    }
    if (wgs >= 8 && (form == 2 || 2 * gemm_tile_count(m, n, bn) >=
                                      static_cast<long long>(kTileMinPerCU2) * wgs)) {
      gemm_tile_launch(p.x, ldx, p.w, ldw, p.out, ldo, m, n, k, bn, wgs, s);
      return vmhost::launch_status("vm_linear_fwd");
    }
  }
  // the LDS-DMA and register-ring forms address x through one buffer (31-bit offsets)
  if ((long long)m * ldx * 2 >= (1ll << 31)) {
    vmhost::set_error("vm_linear_fwd: x past 2 GB needs the persistent form (no bias, n a "
                      "multiple of 192 or 256)");
    return VM_E_INVALID;
  }
  linear_dma_launch(p, s);
  return vmhost::launch_status("vm_linear_fwd");
}

extern "C" long long vm_linear_add_norm_counter_bytes(int m) {
  return m <= 0 ? 0 : static_cast<long long>((m + kNormGran - 1) / kNormGran) * sizeof(unsigned);
}

extern "C" int vm_linear_add_norm_fwd(const void* x, long long ldx, const void* w, long long ldw,
                                      void* h, long long ldo, float* residual, long long ldr,
                                      const float* norm_weight, float eps, void* hn, long long ldh,
                                      int m, int n, int k, void* counters,
                                      long long counter_bytes, vm_stream_t stream) {
  if (!x || !w || !h || !residual || !norm_weight || !hn || !counters) {
    vmhost::set_error("vm_linear_add_norm_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (m < 0 || n < 4 || n > 1024 || n % 8 || k < kLinBK || k % kLinBK || ldx < k || ldw < k ||
      ldo < n || ldr < n || ldh < n || ldx % 8 || ldw % 8 || ldo % 8 || ldr % 4 || ldh % 4 ||
      !vmhost::aligned16(x) || !vmhost::aligned16(w) || !vmhost::aligned16(h) ||
      !vmhost::aligned16(residual) || !vmhost::aligned16(norm_weight) || !vmhost::aligned16(hn) ||
      (long long)m * ldx * 2 >= (1ll << 31) || (long long)n * ldw * 2 >= (1ll << 31) ||
      (long long)m * ldo * 2 >= (1ll << 31) ||
      counter_bytes < vm_linear_add_norm_counter_bytes(m)) {
    vmhost::set_error("vm_linear_add_norm_fwd: bf16 x / w / h / hn, fp32 residual and weight; "
                      "k a multiple of 64, n a multiple of 8 and <= 1024, 16-byte aligned "
                      "rows under 2 GB, vm_linear_add_norm_counter_bytes(m) zeroed counters");
    return VM_E_INVALID;
  }
  if (m == 0) return VM_OK;
  LinParams p{};
  p.x = static_cast<const bf16_t*>(x); p.ldx = ldx;
  p.w = static_cast<const bf16_t*>(w); p.ldw = ldw;
  p.bias = nullptr; p.out = static_cast<bf16_t*>(h); p.ldo = ldo;
  p.m = m; p.n = n; p.k = k;
  NormTail q{};
  q.res = residual; q.ldr = ldr; q.w = norm_weight; q.hn = static_cast<bf16_t*>(hn); q.ldh = ldh;
  q.eps = eps; q.cnt = static_cast<unsigned*>(counters);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid((m + 63) / 64, (n + kLinBN - 1) / kLinBN);
  const size_t lds = 2 * (64 + kLinBN) * kLinPitch * sizeof(bf16_t);
  switch (k / kLinBK) {
#define VM_LIN(NKV)                                                                   \
  case NKV:                                                                           \
    hipLaunchKernelGGL((linear_kernel<64, NKV, true>), grid, dim3(256), lds, s, p, q); \
    break;
    VM_LIN(3) VM_LIN(6) VM_LIN(9) VM_LIN(12) VM_LIN(18) VM_LIN(24)
#undef VM_LIN
    default:
      vmhost::set_error("vm_linear_add_norm_fwd: k = %d (supported: 192, 384, 576, 768, 1152, "
                        "1536)", k);
      return VM_E_INVALID;
  }
  return vmhost::launch_status("vm_linear_add_norm_fwd");
}
