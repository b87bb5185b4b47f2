// Small-M projection GEMM for the streaming-chunk latency path: out = x @ w^T (+ bias),
// bf16 operands, fp32 accumulation on v_mfma_f32_16x16x32_bf16, bf16 out.  Replaces the
// mixer's in_proj / out_proj nn.Linear calls (mamba_simple.py:333-339, :445-446) below the
// chip-filling row counts of the persistent kernel (vm_gemm_tile.hip); at B = 1 (M = 3144
// rows) the library's 256x128 tiles give ~1 workgroup per CU and each walks the whole K
// serially (14-15 us per projection), 128x128 / 128x64 tiles put 1-2 on every CU.
//
// Layout: x (m, k) and w (n, k) both K-contiguous (the nn.Linear layouts), out (m, n).
// Each output row's dot products run in the same order whatever m is, so a row's bits do
// not depend on the sequence length (chunked == full).  vm_linear_add_norm_fwd runs the same
// kernel with the next block's residual add + RMSNorm as a second phase (NORM).

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
// fused_add_norm / rms_norm / residual_in_fp32), phase B of linear_dma_kernel<..., NORM>:
// res += h (fp32, in place);  hn = bf16(res * rsqrt(mean(res^2) + eps) * w), h being the
// block's output rounded to bf16.
struct NormTail {
  float* res;         // (m, n) fp32, row stride ldr: read and updated in place
  long long ldr;
  const float* w;     // (n) fp32 norm weight
  bf16_t* hn;         // (m, n) bf16 normalised output, row stride ldh
  long long ldh;
  float eps;
  unsigned* cnt;      // vm_linear_add_norm_counter_bytes(m) zeroed bytes, left zeroed
};
constexpr int kSC1 = 16;  // buffer cache-policy bit: sc1 (agent-coherent)

__device__ __forceinline__ float lin_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int kLinBK = 64;  // K step

// ---------------------------------------------------------------- LDS-DMA pipelined form
// Per-row K order: 64-wide steps, two 16x16x32 MFMAs per step in k order (the persistent
// kernel's too, so every output row is bit-identical whatever the tile shape), with the
// operand tiles staged global -> LDS by buffer_load ... lds (no VGPR round trip, no
// ds_write pass) into NBUF stage buffers, NBUF - 1 steps in flight across the raw s_barrier
// (counted vmcnt, never 0 in the loop; cdna_hip_programming.md §5 "Pipelining across
// barriers").  The round-2 register ring (removed in round 5) kept one step in flight and
// its barrier drained vmcnt, so at B = 1 (M = 3144) each of its K steps waited out an L2
// round trip: in_proj (N = 2304, K = 576) ran 24.7 us against ~4 us of MFMA work.
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
// NORM (vm_linear_add_norm_fwd, round 5): after its tile the workgroup also runs the next
// block's residual add + RMSNorm for a share of the rows (see the phase-B comment below);
// the host launches it only when the whole grid is co-resident (grid <= CUs).
template <int BM, int BN, int NK, int NBUF, int NWM = 2, bool NORM = false>
__global__ __launch_bounds__(128 * NWM) void linear_dma_kernel(const LinParams p, const NormTail q) {
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

  // NORM phase-B operands that no workgroup of this launch writes — the residual rows this
  // wave normalises and the norm weight — are loaded now and held across the GEMM
  constexpr int kNR = NORM ? 2 : 1;  // rows per wave in phase B
  constexpr int kNC = 4;             // 4-column chunks per lane (n <= 1024)
  typedef __attribute__((__vector_size__(4 * sizeof(float)))) float nv4f;
  nv4f nres[kNR][kNC], nw[kNC];
  const int rpw = NORM ? (p.m + nwg - 1) / nwg : 0;  // rows per workgroup in phase B
  const int nrow0 = l * rpw + wave * kNR;            // this wave's first row (group 0)
  auto ncol = [&](int j, int es) {  // byte offset of chunk j of a row (out of range past n)
    int o = lane * 4 + 256 * j < p.n ? (lane * 4 + 256 * j) * es : 0x7ffffff0;
    asm volatile("" : "+v"(o));
    return o;
  };
  if constexpr (NORM) {
    const auto wq = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(q.w), 0, p.n * 4, 0x00020000);
#pragma unroll
    for (int j = 0; j < kNC; ++j)
      nw[j] = __builtin_bit_cast(nv4f, __builtin_amdgcn_raw_buffer_load_b128(wq, ncol(j, 4), 0, 0));
#pragma unroll
    for (int r = 0; r < kNR; ++r) {
      const int row = nrow0 + r;
      const bool live = wave * kNR + r < rpw && row < p.m;  // group 0
      const auto rq = __builtin_amdgcn_make_buffer_rsrc(
          q.res + (long long)(live ? row : 0) * q.ldr, 0, live ? p.n * 4 : 0, 0x00020000);
#pragma unroll
      for (int j = 0; j < kNC; ++j)
        nres[r][j] = __builtin_bit_cast(nv4f, __builtin_amdgcn_raw_buffer_load_b128(rq, ncol(j, 4), 0, 0));
    }
  }

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
  const auto hr = __builtin_amdgcn_make_buffer_rsrc(
      p.out, 0, static_cast<int>((long long)p.m * p.ldo * 2), 0x00020000);
  // this tile's rows (BM * ldo * 2 bytes at most: no 31-bit offset limit on the whole output)
  const auto tr = __builtin_amdgcn_make_buffer_rsrc(
      p.out + (long long)m0 * p.ldo, 0,
      static_cast<int>(min(static_cast<long long>(p.m - m0), static_cast<long long>(BM)) * p.ldo * 2),
      0x00020000);
#pragma unroll
  for (int i = 0; i < (kPieces + NT - 1) / NT; ++i) {
    const int pc = tid + NT * i;
    if (kPieces % NT != 0 && pc >= kPieces) break;
    const int row = pc / (BN / 8), cq = pc % (BN / 8);
    const int gm = m0 + row, gn = n0 + cq * 8;
    if (gm < p.m && gn < p.n) {
      const uint4 v = *reinterpret_cast<const uint4*>(&sO[row * kOutPitch + cq * 8]);
      if constexpr (NORM) {  // agent-coherent: other workgroups read these rows in phase B
        typedef __attribute__((__vector_size__(4 * sizeof(int)))) int v4i;
        __builtin_amdgcn_raw_buffer_store_b128(v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w}, hr,
                                               (gm * static_cast<int>(p.ldo) + gn) * 2, 0, kSC1);
      } else {  // write-through (sc1): see kSmallStoreWT
        typedef __attribute__((__vector_size__(4 * sizeof(int)))) int v4i;
        __builtin_amdgcn_raw_buffer_store_b128(v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w}, tr,
                                               (row * static_cast<int>(p.ldo) + gn) * 2, 0, kSmallStoreWT);
      }
    }
  }
  if constexpr (NORM) {
    // ---- phase B: the next block's add + RMSNorm, spread over every workgroup ----
    // Workgroup l normalises rows [l * rpw, (l + 1) * rpw) (one wave per row, kNR rows per
    // wave), which the ntn column tiles of at most two BM-row tiles produced.  Hand-off
    // (MI355X_MICROARCH.md cross-workgroup table, row 1): every h store above is sc1; each
    // storing wave waits vmcnt(0), a workgroup barrier, then ONE lane adds to the row tile's
    // counter (agent-scope atomic); a consumer's lane 0 polls the counters of the row tiles
    // it needs with sc1 loads until each reaches ntn, a workgroup barrier, then every h load
    // is an sc1 load.  The consumers of a row tile count themselves in a second counter; the
    // last one resets both, so the buffer is zero again after the launch (graph replays).
    // The whole grid is co-resident (host check), so a poll never waits on an undispatched
    // producer; it is bounded anyway: a timeout sets the error word and makes the rows NaN.
    unsigned* err = q.cnt;
    unsigned* tcnt = q.cnt + 16;
    const int nmt = (p.m + BM - 1) / BM;
    unsigned* ccnt = tcnt + nmt;
    // (the flag lives in the dynamic LDS, free after the stores: a second __shared__ object
    // beside the DMA stage buffers can make hipcc drain vmcnt before every K-step's reads)
    int& s_ok = *reinterpret_cast<int*>(dsm);
    __builtin_amdgcn_s_waitcnt(0);  // this wave's h stores are acknowledged
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(&tcnt[m0 / BM], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int r_lo = l * rpw, r_hi = min(p.m, r_lo + rpw);
    if (r_lo >= r_hi) return;  // uniform: no rows for this workgroup
    if (tid == 0) {
      int ok = 1;
      for (int mt = r_lo / BM; mt <= (r_hi - 1) / BM; ++mt) {
        unsigned spins = 0;
        while (__hip_atomic_load(&tcnt[mt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
               static_cast<unsigned>(ntn)) {
          if (++spins >= (1u << 20)) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      s_ok = ok;
    }
    __syncthreads();
    const bool ok = s_ok != 0;
    // per row: vm_add_norm_fwd's add_rms_bf16_kernel arithmetic and lane -> chunk map
    // (lane * 4 + 256 j; chunks past n read 0 and add nothing), so the fused result is
    // bit-identical to out_proj followed by vm_add_norm_fwd.  Rows go in groups of
    // NW * kNR (one row per wave and r); the first group's residual rows came in at the
    // kernel start, later groups' (small grids only) are loaded here.
#pragma unroll 1
    for (int g0 = 0; g0 < rpw; g0 += NW * kNR) {
      if (g0 > 0) {
#pragma unroll
        for (int r = 0; r < kNR; ++r) {
          const int row = nrow0 + g0 + r;
          const bool live = g0 + wave * kNR + r < rpw && row < p.m;
          const auto rq = __builtin_amdgcn_make_buffer_rsrc(
              q.res + (long long)(live ? row : 0) * q.ldr, 0, live ? p.n * 4 : 0, 0x00020000);
#pragma unroll
          for (int j = 0; j < kNC; ++j)
            nres[r][j] = __builtin_bit_cast(nv4f, __builtin_amdgcn_raw_buffer_load_b128(rq, ncol(j, 4), 0, 0));
        }
      }
      uint32_t hq[kNR][kNC][2];
#pragma unroll
      for (int r = 0; r < kNR; ++r) {
        const int row = nrow0 + g0 + r;
        const bool live = g0 + wave * kNR + r < rpw && row < p.m;
        const auto hq_r = __builtin_amdgcn_make_buffer_rsrc(
            p.out + (long long)(live ? row : 0) * p.ldo, 0, live ? p.n * 2 : 0, 0x00020000);
#pragma unroll
        for (int j = 0; j < kNC; ++j) {
          const auto v = __builtin_amdgcn_raw_buffer_load_b64(hq_r, ncol(j, 2), 0, kSC1);
          hq[r][j][0] = v[0];
          hq[r][j][1] = v[1];
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // every h load of the wave's rows in flight first
#pragma unroll
      for (int r = 0; r < kNR; ++r) {
        const int row = nrow0 + g0 + r;
        const bool live = g0 + wave * kNR + r < rpw && row < p.m;
        float v[kNC][4];
#pragma unroll
        for (int j = 0; j < kNC; ++j) {
          v[j][0] = __uint_as_float(hq[r][j][0] << 16) + nres[r][j][0];
          v[j][1] = __uint_as_float(hq[r][j][0] & 0xffff0000u) + nres[r][j][1];
          v[j][2] = __uint_as_float(hq[r][j][1] << 16) + nres[r][j][2];
          v[j][3] = __uint_as_float(hq[r][j][1] & 0xffff0000u) + nres[r][j][3];
        }
        float sq = 0.0f;
#pragma unroll
        for (int j = 0; j < kNC; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) sq = fmaf(v[j][i], v[j][i], sq);
        float rstd = rsqrtf(lin_wave_sum(sq) / p.n + q.eps);
        if (!ok) rstd = __builtin_nanf("");
        const auto hn_r = __builtin_amdgcn_make_buffer_rsrc(
            q.hn + (long long)(live ? row : 0) * q.ldh, 0, live ? p.n * 2 : 0, 0x00020000);
        const auto ro_r = __builtin_amdgcn_make_buffer_rsrc(
            q.res + (long long)(live ? row : 0) * q.ldr, 0, live ? p.n * 4 : 0, 0x00020000);
#pragma unroll
        for (int j = 0; j < kNC; ++j) {
          float y[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) y[i] = (v[j][i] - 0.0f) * rstd * nw[j][i];
          typedef __attribute__((__vector_size__(2 * sizeof(int)))) int v2i;
          const v2i o2 = {static_cast<int>(static_cast<uint32_t>(from_f32<bf16_t>(y[0])) |
                                           (static_cast<uint32_t>(from_f32<bf16_t>(y[1])) << 16)),
                          static_cast<int>(static_cast<uint32_t>(from_f32<bf16_t>(y[2])) |
                                           (static_cast<uint32_t>(from_f32<bf16_t>(y[3])) << 16))};
          __builtin_amdgcn_raw_buffer_store_b64(o2, hn_r, ncol(j, 2), 0, 0);
          typedef __attribute__((__vector_size__(4 * sizeof(int)))) int v4i;
          const v4i r4 = {static_cast<int>(__float_as_uint(v[j][0])), static_cast<int>(__float_as_uint(v[j][1])),
                          static_cast<int>(__float_as_uint(v[j][2])), static_cast<int>(__float_as_uint(v[j][3]))};
          __builtin_amdgcn_raw_buffer_store_b128(r4, ro_r, ncol(j, 4), 0, 0);
        }
      }
    }
    // count this workgroup out of the row tiles it read; the last consumer of a tile resets
    // both of its counters (every producer has added: the poll saw ntn)
    if (tid == 0) {
      for (int mt = r_lo / BM; mt <= (r_hi - 1) / BM; ++mt) {
        const int first = (mt * BM) / rpw;
        const int last = min((min(mt * BM + BM, p.m) - 1) / rpw, nwg - 1);
        const unsigned old =
            __hip_atomic_fetch_add(&ccnt[mt], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == static_cast<unsigned>(last - first)) {
          __hip_atomic_store(&tcnt[mt], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ccnt[mt], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
}

// Tile choice for the pipelined form (row bits do not depend on it), measured at the B = 1
// chunk shapes (scripts/diag/variant_linear.py): wide outputs (in_proj, N = 2 * d_inner)
// on 128 x 128 tiles with two stage buffers (64 KB: two workgroups per CU; 14.1 us against
// 17.6 for the register ring, three buffers 16.3), eight waves each since round 4 (four per
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
                       lds, s, p, NormTail{});                                                 \
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
bool gemm_tile_norm_ok(int n, int k, int bn);
void gemm_tile_norm_launch(const bf16_t* x, long long ldx, const bf16_t* w, long long ldw,
                           bf16_t* out, long long ldo, float* res, long long ldr, const float* nw,
                           float eps, bf16_t* hn, long long ldh, unsigned* cnt, int m, int n,
                           int k, int workgroups, hipStream_t s);
// the persistent kernel runs from 1.5 tiles per CU (twice the tile count >= 3 x CUs): C5's
// in_proj (12,544 rows, 441 tiles) 41.9 -> ~35 us, the C5 chunk 8.55 -> 8.26 ms
constexpr int kTileMinPerCU2 = 3;

using vmhost::device_cus;

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

// Counter buffer of vm_linear_add_norm_fwd: an error word (+ pad) and two counters per
// 128-row tile (producers, consumers).
extern "C" long long vm_linear_add_norm_counter_bytes(int m) {
  return m <= 0 ? 0 : static_cast<long long>(16 + 2 * ((m + 127) / 128)) * sizeof(unsigned);
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
      (long long)n * ldw * 2 >= (1ll << 31) || counter_bytes < vm_linear_add_norm_counter_bytes(m)) {
    vmhost::set_error("vm_linear_add_norm_fwd: bf16 x / w / h / hn, fp32 residual and weight; "
                      "k a multiple of 64, n a multiple of 8 and <= 1024, 16-byte aligned "
                      "rows, w under 2 GB, vm_linear_add_norm_counter_bytes(m) zeroed counters");
    return VM_E_INVALID;
  }
  switch (k / kLinBK) {
    case 3: case 6: case 9: case 12: case 18: case 24: break;
    default:
      vmhost::set_error("vm_linear_add_norm_fwd: k = %d (supported: 192, 384, 576, 768, 1152, "
                        "1536)", k);
      return VM_E_INVALID;
  }
  if (m == 0) return VM_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // one launch when the whole 128 x 64-tile grid is co-resident at one workgroup per CU
  constexpr int BM = 128, BN = 64;
  const long long nwg = static_cast<long long>((m + BM - 1) / BM) * ((n + BN - 1) / BN);
  const int cus = device_cus(s);
  if (cus > 0 && nwg <= cus) {
    LinParams p{};
    p.x = static_cast<const bf16_t*>(x); p.ldx = ldx;
    p.w = static_cast<const bf16_t*>(w); p.ldw = ldw;
    p.bias = nullptr; p.out = static_cast<bf16_t*>(h); p.ldo = ldo;
    p.m = m; p.n = n; p.k = k;
    NormTail q{};
    q.res = residual; q.ldr = ldr; q.w = norm_weight; q.hn = static_cast<bf16_t*>(hn); q.ldh = ldh;
    q.eps = eps; q.cnt = static_cast<unsigned*>(counters);
    const dim3 grid((m + BM - 1) / BM, (n + BN - 1) / BN);
    // 3 stage buffers = 72 KB; 96 KB requested so a CU holds one workgroup (the validated
    // one-per-CU form of the hand-off)
    const size_t lds = 96 * 1024;
    switch (k / kLinBK) {
#define VM_LN(NKV)                                                                               \
  case NKV:                                                                                      \
    hipLaunchKernelGGL((linear_dma_kernel<BM, BN, NKV, 3, 4, true>), grid, dim3(512), lds, s, p, q); \
    break;
      VM_LN(3) VM_LN(6) VM_LN(9) VM_LN(12) VM_LN(18) VM_LN(24)
#undef VM_LN
      default: break;
    }
    return vmhost::launch_status("vm_linear_add_norm_fwd");
  }
  // chip-filling row counts: the persistent tile GEMM with the norm pass per 256-row block
  // (vm_gemm_tile.hip, NORM), where vm_linear_fwd_form would pick the persistent form
  {
    const int bn = gemm_tile_bn(m, n, k, ldx, ldw, ldo);
    const int wgs = cus / 8 * 8;
    if (bn && gemm_tile_norm_ok(n, k, bn) && wgs >= 8 &&
        2 * gemm_tile_count(m, n, bn) >= static_cast<long long>(kTileMinPerCU2) * wgs) {
      gemm_tile_norm_launch(static_cast<const bf16_t*>(x), ldx, static_cast<const bf16_t*>(w), ldw,
                            static_cast<bf16_t*>(h), ldo, residual, ldr, norm_weight, eps,
                            static_cast<bf16_t*>(hn), ldh, static_cast<unsigned*>(counters), m, n,
                            k, wgs, s);
      return vmhost::launch_status("vm_linear_add_norm_fwd");
    }
  }
  // otherwise the two launches it replaces (the same kernels: bit-identical either way)
  if (ldo != n || ldr != n || ldh != n) {
    vmhost::set_error("vm_linear_add_norm_fwd: a grid past the CU count runs the separate "
                      "kernels, which need contiguous h / residual / hn rows");
    return VM_E_INVALID;
  }
  int rc = vm_linear_fwd_form(x, ldx, w, ldw, nullptr, h, ldo, m, n, k, VM_DTYPE_BF16, 0, stream);
  if (rc != VM_OK) return rc;
  return vm_add_norm_fwd(h, VM_DTYPE_BF16, residual, VM_DTYPE_F32, norm_weight, nullptr, hn,
                         VM_DTYPE_BF16, residual, VM_DTYPE_F32, m, n, eps, 1, stream);
}
