// Persistent 256-row tile GEMM for the mixer's projections at chip-filling batches:
// out = x @ w^T, bf16 operands, fp32 accumulation on v_mfma_f32_16x16x32_bf16, bf16 out.
// Replaces the library GEMM that in_proj / out_proj (mamba_simple.py:333-339, :445-446)
// ran on above 8 clips, whose M-dependent kernel choice made a chunked stream differ from the
// one-pass forward (C4 at 72 clips: 1.4e-4).  Every output element here is the same chain
// of MFMAs as in linear_dma_kernel (vm_gemm.hip): K in 64-wide steps, two 32-deep MFMAs per
// step in k order, one accumulator per element — so a row's bits depend on neither the row
// count nor the tile shape, and the two kernels agree bit for bit.
//
// Structure (cdna_hip_programming.md §5 "256² 8-phase template", rebuilt for short K):
//   * one 512-thread workgroup per CU, persistent: it walks a run of output tiles, and the
//     K-tile stream continues across tile boundaries (the next tile's first K-tiles are
//     loaded during the current tile's last ones), so K = 576 / 1152 pays no per-tile
//     pipeline fill;
//   * tile BM x BN (256 x 256 for in_proj-like N, 256 x 192 for out_proj-like N), BK = 64;
//     LDS = two stage buffers of (BM + BN) rows x 128 B, each split in four half-tiles
//     (A top / bottom rows, B left / right rows) staged by LDS-DMA (buffer_load ... lds,
//     16 B per lane, 16-B chunks XOR-swizzled by (row / 2) & 7 on the source address);
//   * a wave owns TMH m-tiles in each A half and TNH n-tiles in each B half; each K-tile is
//     4 phases, one output quadrant each: (top, left), (top, right), (bottom, right),
//     (bottom, left).  Each half-tile is read in exactly one phase (the fragments stay in
//     registers for the quadrants that reuse them), one half-tile is issued per phase, and
//     each is issued 4-5 phases before its read: counted vmcnt waits (8, never 0), raw
//     s_barrier, two barriers per phase;
//   * vmcnt counts the output stores too, and a store may complete before an older
//     LDS-DMA load (LLVM treats mixed VMEM reads / writes on vmcnt as out of order): a wait
//     that allowed the S stores of the previous tile as "younger ops" let a wave read a
//     half-tile that had not landed (1 launch in 30 differed at B = 72,
//     scripts/diag/determinism_b72.py).  No wait counts a store (see the wait rule below);
//   * waves 4-7 (the SIMD partners of waves 0-3) run one barrier behind (stagger), so a
//     SIMD's two waves alternate MFMA and LDS / issue segments;
//   * the MFMA computes out^T tiles (A operand = W rows, B operand = x rows): a lane holds 4
//     consecutive output columns of one row; one v_permlane16_swap per pair of n-tiles
//     gives each lane 8, stored as 16-byte buffer stores straight from registers.
// Hazard rules (cdna_hip_programming.md §5 template notes, derived for this stagger): a
// half-tile is read only in a phase after the one whose wait retired it; a region is
// re-staged only 2+ phases after its last read, and every read completes (lgkmcnt(0))
// before the reading phase's first barrier.

#include <utility>

#include "vm_common.h"

namespace vm {

namespace {

typedef __attribute__((__vector_size__(8 * sizeof(short)))) short tg_bf16x8;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float tg_f32x4;
typedef __attribute__((__vector_size__(4 * sizeof(int)))) int tg_i32x4;
typedef __bf16 tg_b2 __attribute__((ext_vector_type(2)));
typedef float tg_f2 __attribute__((ext_vector_type(2)));

template <int... Is, class F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, Is...>, F&& f) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

__device__ __forceinline__ uint32_t tg_pack(float a, float b) {  // lo = a, hi = b (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(tg_f2{a, b}, tg_b2));
}

__device__ __forceinline__ int tg_slot(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// s_waitcnt vmcnt(N) (expcnt, lgkmcnt left at their maxima)
template <int N>
__device__ __forceinline__ void tg_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0070 | 0x0F00);
}
__device__ __forceinline__ void tg_wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

// raw s_barrier with compiler fences: no LDS access moves across it
__device__ __forceinline__ void tg_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__device__ __forceinline__ void tg_dma(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           voff, soff, 0, 0);
}

struct TileGemmParams {
  const bf16_t* x; long long ldx;  // (m, k), row stride ldx elements
  const bf16_t* w; long long ldw;  // (n, k)
  bf16_t* out; long long ldo;      // (m, n)
  int m, n, k;
  int ntn;    // n / BN
  int tiles;  // ceil(m / BM) * ntn
  int tpx;    // ceil(tiles / 8) (NORM: rounded up to whole row blocks of ntn tiles): the
              // contiguous tile range of one XCD's workgroups
  // NORM (vm_linear_add_norm_fwd at chip-filling row counts): the next block's residual
  // add + RMSNorm, res += out (fp32, in place), hn = bf16(res * rsqrt(mean(res^2) + eps) * nw)
  float* res; long long ldr;
  const float* nw;
  bf16_t* hn; long long ldh;
  float eps;
  unsigned* cnt;  // [0] error word, [16 + row block] producer counts; left zeroed
};
constexpr int kTileSC1 = 16;  // buffer cache-policy bit sc1: agent-coherent (cross-workgroup)
// rows of the NORM pass each wave has in flight at once (18 VGPRs per row at n = 576)
constexpr int kTileNormRows = 8;

struct TileRes {  // one output tile: its x rows' buffer, its w rows' offset, its index
  __amdgpu_buffer_rsrc_t x;
  int wsoff;  // n0 * ldw * 2
  int t;      // tile index, -1 past the workgroup's run
};

// The wait rule: every wait is vmcnt(8) and never counts a tile's output stores as
// "younger" ops: the first wait after the stores (the next tile's first phase) also waits
// for them to complete.  A phase waits for its own fragment reads after its first barrier,
// just before its MFMAs (the reads overlap the barrier wait; cdna_hip_programming.md's 8-phase
// template order).  (Reading phase 1's B-right fragments right after phase 0's first barrier,
// to overlap phase 0's MFMAs, reads an unlanded half-tile: waves 4-7 pass their phase-0 wait
// only after that barrier — the stagger needs the read one phase after the wait; measured
// wrong in every launch.)  The store placements, wave priorities and wait forms measured
// against this one live in git history, not in the product source.

}  // namespace

template <int WGM, int TMH, int TNH, int NK, bool NORM = false, int NC = 1>
__global__ __launch_bounds__(512) void gemm_tile_kernel(const TileGemmParams p) {
  constexpr int WGN = 8 / WGM;
  constexpr int BM = 2 * WGM * TMH * 16, BN = 2 * WGN * TNH * 16;
  constexpr int HA = BM / 2, HB = BN / 2;
  constexpr int RB = 128;  // bytes per staged row: 64 bf16 of K
  constexpr int A_BYTES = BM * RB, STAGE = (BM + BN) * RB;
  constexpr int TPI = (NK & 1) ? 2 : 1;  // tiles per loop iteration: stage parity stays static
  constexpr int QI = TPI * NK;           // K-tiles per iteration (even)
  constexpr int S = 2 * TMH * TNH;       // 16-byte stores per wave per tile
  constexpr int VM = 8;                  // loads younger than an awaited half-tile: 4 x 2
  static_assert(WGM * WGN == 8 && HA == 128 && (HB == 128 || HB == 96), "tile geometry");
  static_assert(NK >= 3, "the prefetch reaches two K-tiles ahead inside one tile");
  static_assert(S <= 16, "output stores per wave per tile");
  static_assert(!NORM || (TPI == 1 && NC >= 1 && NC <= 4), "NORM: even NK, n <= 1024");
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WGN, wc = wave % WGN;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- tiles: XCD-contiguous runs (workgroup b on XCD b % 8 under round-robin dispatch;
  // placement is a speed choice only), consecutive tiles share an x panel in that L2
  const int b = blockIdx.x;
  const int wpx = gridDim.x >> 3;
  const int t_begin = (b & 7) * p.tpx + (b >> 3);
  const int t_end = min(((b & 7) + 1) * p.tpx, p.tiles);
  const int ntiles = t_end > t_begin ? (t_end - t_begin + wpx - 1) / wpx : 0;
  const int iters = (ntiles + TPI - 1) / TPI;
  if (iters == 0) return;  // uniform across the workgroup

  const int xbytes = static_cast<int>(p.ldx * 2), wbytes = static_cast<int>(p.ldw * 2);
  // w: one buffer over all n rows (n % BN == 0: every staged row exists)
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.w), 0,
                                                     static_cast<int>(p.n * p.ldw * 2), 0x00020000);
  auto tile_res = [&](int k) __attribute__((always_inline)) -> TileRes {  // this workgroup's k-th tile
    TileRes r;
    if (k >= ntiles) {  // past the run: x loads out of range (0), nothing stored
      r.x = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.x), 0, 0, 0x00020000);
      r.wsoff = 0;
      r.t = -1;
      return r;
    }
    const int t = t_begin + k * wpx;
    const int mt = t / p.ntn, nt = t - mt * p.ntn;
    const long long m0 = static_cast<long long>(mt) * BM;
    const long long rows = min(static_cast<long long>(p.m) - m0, static_cast<long long>(BM));
    r.x = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.x + m0 * p.ldx), 0,
                                            static_cast<int>(rows * p.ldx * 2), 0x00020000);
    r.wsoff = nt * BN * wbytes;
    r.t = t;
    return r;
  };
  // the output rows [r0, r0 + 16) of tile t, rebased so a row past m (or a tile past the
  // run) falls out of the buffer's range; the store offsets then stay per-lane constants
  auto out_res = [&](int t, int r0) __attribute__((always_inline)) {
    long long m0 = 0, rows = 0;
    int n0 = 0;
    if (t >= 0) {
      const int mt = t / p.ntn;
      n0 = (t - mt * p.ntn) * BN;
      m0 = static_cast<long long>(mt) * BM + r0;
      rows = min(static_cast<long long>(p.m) - m0, 16LL);
    }
    const long long nrec = rows > 0 ? rows * p.ldo * 2 - n0 * 2 : 0;
    return __builtin_amdgcn_make_buffer_rsrc(p.out + m0 * p.ldo + n0, 0, static_cast<int>(nrec),
                                             0x00020000);
  };

  // ---- per-lane DMA source offsets: instruction j of a half covers rows 64 j + 8 wave +
  // lane / 8 (128-row halves) or, for 96-row B halves, rows 64 + 4 wave + lane / 8 with
  // lanes 0-31 for j = 1; LDS is lane-linear, the chunk swizzle sits on the source
  int aoff[2][2], boff[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ra = 64 * j + 8 * wave + (lane >> 3);
    const int rb = (j == 0 || HB == 128) ? 64 * j + 8 * wave + (lane >> 3)
                                         : 64 + 4 * wave + (lane >> 3);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      aoff[h][j] = (h * HA + ra) * xbytes + tg_slot(ra, lane & 7) * 16;
      boff[h][j] = (h * HB + rb) * wbytes + tg_slot(rb, lane & 7) * 16;
    }
  }
  // which: 0 A top, 1 A bottom, 2 B left, 3 B right
  auto issue = [&](const TileRes& r, int which, int buf, int kt) __attribute__((always_inline)) {
    char* base = lds + buf * STAGE;
    const int soff = kt * RB;
    if (which < 2) {
      char* d = base + which * HA * RB;
      tg_dma(r.x, d + wave * 1024, aoff[which][0], soff);
      tg_dma(r.x, d + 8192 + wave * 1024, aoff[which][1], soff);
    } else {
      const int g = which - 2;
      char* d = base + A_BYTES + g * HB * RB;
      tg_dma(wrs, d + wave * 1024, boff[g][0], r.wsoff + soff);
      if (HB == 128) {
        tg_dma(wrs, d + 8192 + wave * 1024, boff[g][1], r.wsoff + soff);
      } else if (lane < 32) {
        tg_dma(wrs, d + 8192 + wave * 512, boff[g][1], r.wsoff + soff);
      }
    }
  };

  // ---- fragments: per lane 16 bytes at (row = tile row + lane % 16, chunk 4 ks + lane / 16)
  int la[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) la[ks] = fr * RB + tg_slot(fr, ks * 4 + fq) * 16;
  const int arow0 = wr * TMH * 16, bcol0 = wc * TNH * 16;
  tg_bf16x8 xf[TMH][2], wf[2][TNH][2];
  auto read_a = [&](int buf, int h) __attribute__((always_inline)) {
    const char* base = lds + buf * STAGE + (h * HA + arow0) * RB;
#pragma unroll
    for (int i = 0; i < TMH; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        xf[i][ks] = *reinterpret_cast<const tg_bf16x8*>(base + i * 16 * RB + la[ks]);
  };
  auto read_b = [&](int buf, int g) __attribute__((always_inline)) {
    const char* base = lds + buf * STAGE + A_BYTES + (g * HB + bcol0) * RB;
#pragma unroll
    for (int j = 0; j < TNH; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        wf[g][j][ks] = *reinterpret_cast<const tg_bf16x8*>(base + j * 16 * RB + la[ks]);
  };

  tg_f32x4 acc[2][TMH][2][TNH];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < TMH; ++i)
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int j = 0; j < TNH; ++j) acc[h][i][g][j] = tg_f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&](int h, int g) __attribute__((always_inline)) {  // quadrant (A half h, B half g) over the K-tile
#pragma unroll
    for (int i = 0; i < TMH; ++i)
#pragma unroll
      for (int j = 0; j < TNH; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[h][i][g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[g][j][ks], xf[i][ks],
                                                                    acc[h][i][g][j], 0, 0, 0);
  };

  // ---- epilogue: D[n = 4 (lane/16) + r][m = lane % 16] per 16x16 tile; n-tiles paired
  // (index g * TNH + j, pairs (2c, 2c+1)) and v_permlane16_swap-ed so a lane holds 8
  // consecutive columns: lane row r16 = lane / 16 takes tile 2c + (r16 & 1), columns
  // 8 (r16 >> 1) .. +7
  const int st_lane = fr * static_cast<int>(p.ldo) * 2 + (8 * (fq >> 1)) * 2;
  auto store_tile = [&](const TileRes& tr, int h0 = 0, int h1 = 2) __attribute__((always_inline)) {
#pragma unroll
    for (int h = h0; h < h1; ++h)
#pragma unroll
      for (int i = 0; i < TMH; ++i) {
        const auto o = out_res(tr.t, h * HA + arow0 + i * 16);
#pragma unroll
        for (int c = 0; c < TNH; ++c) {
          const int ia = 2 * c, ib = 2 * c + 1;
          const tg_f32x4& A = acc[h][i][ia / TNH][ia % TNH];
          const tg_f32x4& B = acc[h][i][ib / TNH][ib % TNH];
          const int col_a = (ia / TNH) * HB + bcol0 + (ia % TNH) * 16;
          const int col_b = (ib / TNH) * HB + bcol0 + (ib % TNH) * 16;
          const uint32_t a0 = tg_pack(A[0], A[1]), a1 = tg_pack(A[2], A[3]);
          const uint32_t b0 = tg_pack(B[0], B[1]), b1 = tg_pack(B[2], B[3]);
          const auto s0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
          const tg_i32x4 v{static_cast<int>(s0[0]), static_cast<int>(s1[0]),
                           static_cast<int>(s0[1]), static_cast<int>(s1[1])};
          const int col = (fq & 1) ? col_b : col_a;
          // NORM: sc1, so the row block's norm pass on another workgroup reads them
          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 0);
        }
      }
  };

  // ---- NORM: the next block's add + RMSNorm of a finished 256-row block (NORM only).
  // The ntn tiles of a row block are consecutive tile indices in one XCD's range (tpx is a
  // whole number of row blocks), run by neighbouring workgroups at the same or an earlier
  // step.  A producer (column tile < ntn - 1) makes its sc1 stores complete (vmcnt(0)) and,
  // once every wave has (the barrier after), adds 1 to the block's counter; the last column
  // tile's workgroup (the poller) completes its own stores, lines up its waves, polls the
  // counter to ntn - 1 (sc1 / agent-scope, bounded: a timeout sets the error word and
  // poisons the rows with NaN), then normalises the block: one wave per row, each lane the
  // 4-column chunks lane * 4 + 256 j — add_rms_bf16_kernel's arithmetic and order
  // (vm_norm.hip), so the result is bit-identical to out_proj then vm_add_norm_fwd — and
  // resets the counter.  (MI355X_MICROARCH.md cross-workgroup hand-off; the grid is one
  // workgroup per CU, every producer runs.)
  typedef __attribute__((__vector_size__(4 * sizeof(float)))) float nv4f;
  auto ncol = [&](int j, int es) __attribute__((always_inline)) {  // chunk j (out of range past n)
    uint32_t o = lane * 4 + 256 * j < p.n ? (lane * 4 + 256 * j) * es : 0x7ffffff0u;
    asm volatile("" : "+v"(o));
    return o;
  };
  auto norm_pass = [&](int mt) __attribute__((always_inline)) {
    const long long r0 = static_cast<long long>(mt) * BM;
    const int rows = static_cast<int>(min(static_cast<long long>(p.m) - r0, static_cast<long long>(BM)));
    int ok = 1;
    if (lane == 0) {
      unsigned spins = 0;
      while (__hip_atomic_load(&p.cnt[16 + mt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
             static_cast<unsigned>(p.ntn - 1)) {
        if (++spins >= (1u << 20)) {
          __hip_atomic_store(p.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    ok = __builtin_amdgcn_readfirstlane(ok);
    nv4f nwv[NC];
    {
      const auto wq = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.nw), 0, p.n * 4, 0x00020000);
#pragma unroll
      for (int j = 0; j < NC; ++j)
        nwv[j] = __builtin_bit_cast(nv4f, __builtin_amdgcn_raw_buffer_load_b128(wq, ncol(j, 4), 0, 0));
    }
    constexpr int RPW = BM / 8;  // rows per wave
    // one buffer per operand over the block's rows (range: the live rows; a dead row's or a
    // column past n's offset falls outside), row offsets in the lane offset
    const auto hr = __builtin_amdgcn_make_buffer_rsrc(p.out + r0 * p.ldo, 0, static_cast<int>(rows * p.ldo * 2), 0x00020000);
    const auto rr = __builtin_amdgcn_make_buffer_rsrc(p.res + r0 * p.ldr, 0, static_cast<int>(rows * p.ldr * 4), 0x00020000);
    const auto hnr = __builtin_amdgcn_make_buffer_rsrc(p.hn + r0 * p.ldh, 0, static_cast<int>(rows * p.ldh * 2), 0x00020000);
    uint32_t c2[NC], c4[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      c2[j] = ncol(j, 2);
      c4[j] = ncol(j, 4);
    }
#pragma unroll 1
    for (int g = 0; g < RPW; g += kTileNormRows) {
      uint32_t hq[kTileNormRows][NC][2];
      nv4f rq[kTileNormRows][NC];
#pragma unroll
      for (int r = 0; r < kTileNormRows; ++r) {
        const uint32_t lr = wave * RPW + g + r;
        const uint32_t oh = lr * static_cast<uint32_t>(p.ldo) * 2, orr = lr * static_cast<uint32_t>(p.ldr) * 4;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          const auto v = __builtin_amdgcn_raw_buffer_load_b64(hr, c2[j] + oh, 0, kTileSC1);
          hq[r][j][0] = v[0];
          hq[r][j][1] = v[1];
          rq[r][j] = __builtin_bit_cast(nv4f, __builtin_amdgcn_raw_buffer_load_b128(rr, c4[j] + orr, 0, 0));
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // every load of the group in flight first
#pragma unroll
      for (int r = 0; r < kTileNormRows; ++r) {
        const uint32_t lr = wave * RPW + g + r;
        const uint32_t ohn = lr * static_cast<uint32_t>(p.ldh) * 2, orr = lr * static_cast<uint32_t>(p.ldr) * 4;
        float v[NC][4];
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          v[j][0] = __uint_as_float(hq[r][j][0] << 16) + rq[r][j][0];
          v[j][1] = __uint_as_float(hq[r][j][0] & 0xffff0000u) + rq[r][j][1];
          v[j][2] = __uint_as_float(hq[r][j][1] << 16) + rq[r][j][2];
          v[j][3] = __uint_as_float(hq[r][j][1] & 0xffff0000u) + rq[r][j][3];
        }
        float sq = 0.0f;
#pragma unroll
        for (int j = 0; j < NC; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) sq = fmaf(v[j][i], v[j][i], sq);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
        float rstd = rsqrtf(sq / p.n + p.eps);
        if (!ok) rstd = __builtin_nanf("");
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          float y[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) y[i] = (v[j][i] - 0.0f) * rstd * nwv[j][i];
          typedef __attribute__((__vector_size__(2 * sizeof(int)))) int v2i;
          const v2i o2 = {static_cast<int>(static_cast<uint32_t>(from_f32<bf16_t>(y[0])) |
                                           (static_cast<uint32_t>(from_f32<bf16_t>(y[1])) << 16)),
                          static_cast<int>(static_cast<uint32_t>(from_f32<bf16_t>(y[2])) |
                                           (static_cast<uint32_t>(from_f32<bf16_t>(y[3])) << 16))};
          __builtin_amdgcn_raw_buffer_store_b64(o2, hnr, c2[j] + ohn, 0, 0);
          const tg_i32x4 r4 = {static_cast<int>(__float_as_uint(v[j][0])), static_cast<int>(__float_as_uint(v[j][1])),
                               static_cast<int>(__float_as_uint(v[j][2])), static_cast<int>(__float_as_uint(v[j][3]))};
          __builtin_amdgcn_raw_buffer_store_b128(r4, rr, c4[j] + orr, 0, 0);
        }
      }
    }
  };
  int sig_mt = -1;   // NORM: the producer row block wave 4 counts in after its next barrier
  int pend_mt = -1;  // NORM: the polled row block normalised at the end of the next tile

  // the iteration's tiles and the next iteration's first (scalars, not an array: an array
  // of descriptors captured by the lambdas below stays in memory and loses uniformity)
  TileRes cur0 = tile_res(0), cur1 = tile_res(TPI == 2 ? 1 : ntiles), nxt = tile_res(TPI);

  // ---- prologue: K-tiles 0 (all four halves) and 1 (A top, B left) of the first tile;
  // the wait retires what the first phases read before their own waits run (A top / B left
  // of K-tile 0)
  issue(cur0, 0, 0, 0);
  issue(cur0, 2, 0, 0);
  issue(cur0, 3, 0, 0);
  issue(cur0, 1, 0, 0);
  issue(cur0, 0, 1, 1);
  issue(cur0, 2, 1, 1);
  tg_wait_vm<VM>();
  tg_barrier();
  if (wave >= 4) tg_barrier();  // stagger: waves 4-7 run one barrier behind

#pragma unroll 1
  for (int it = 0; it < iters; ++it) {
    static_for<QI * 4>([&](auto ic) __attribute__((always_inline)) {
      constexpr int q = decltype(ic)::value / 4, P = decltype(ic)::value % 4;
      constexpr int kt = q % NK, tp = q / NK, buf = q & 1;
      // 1. this phase's half-tile: p0 B right (q+1), p1 A bottom (q+1), p2 A top (q+2),
      //    p3 B left (q+2); past the iteration it belongs to the next one's first tile
      constexpr int qt = q + (P < 2 ? 1 : 2);
      constexpr int which = P == 0 ? 3 : P == 1 ? 1 : P == 2 ? 0 : 2;
      if constexpr (qt >= QI) issue(nxt, which, qt & 1, qt - QI);
      else if constexpr (qt / NK == 0) issue(cur0, which, qt & 1, qt % NK);
      else issue(cur1, which, qt & 1, qt % NK);
      // 2. fragment reads of this phase's quadrant
      if constexpr (P == 0) { read_a(buf, 0); read_b(buf, 0); }
      if constexpr (P == 1) read_b(buf, 1);
      if constexpr (P == 2) read_a(buf, 1);
      __builtin_amdgcn_sched_barrier(0);
      // 3. retire the half-tile(s) the next phase reads (never counting output stores)
      if constexpr (P != 2) tg_wait_vm<VM>();
      tg_barrier();
      if constexpr (NORM && P == 0 && kt == 0) {
        // every wave's stores of the previous tile completed before this barrier (waves 0-3
        // run one barrier ahead of wave 4): count the producer tile in
        if (sig_mt >= 0 && wave == 4 && lane == 0)
          __hip_atomic_fetch_add(&p.cnt[16 + sig_mt], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sig_mt = -1;
      }
      tg_wait_lgkm0();
      __builtin_amdgcn_sched_barrier(0);
      // 4. the quadrant's MFMAs
      if constexpr (P == 0) mfma(0, 0);
      if constexpr (P == 1) mfma(0, 1);
      if constexpr (P == 2) mfma(1, 1);
      if constexpr (P == 3) mfma(1, 0);
      tg_barrier();
      // 5. the tile is done after its last quadrant: store it, restart the accumulators
      if constexpr (P == 3 && kt == NK - 1) {
        if constexpr (tp == 0) store_tile(cur0, 0, 2);
        else store_tile(cur1, 0, 2);
        if constexpr (NORM) {
          __builtin_amdgcn_s_waitcnt(0);  // this wave's sc1 stores are acknowledged
          const int mt = cur0.t / p.ntn;
          const bool poller = cur0.t - mt * p.ntn == p.ntn - 1;  // uniform
          if (pend_mt >= 0) {
            // the row block this workgroup polled for one tile ago: line the waves up (waves
            // 0-3 skip the stagger's barrier; every wave's stores are then acknowledged),
            // count this tile in, normalise, re-stagger
            if (wave < 4) tg_barrier();
            tg_barrier();
            if (!poller && wave == 0 && lane == 0)
              __hip_atomic_fetch_add(&p.cnt[16 + mt], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            norm_pass(pend_mt);
            if (wave >= 4) {
              tg_barrier();  // waves 0-3 have finished their polls and rows
              if (wave == 4 && lane == 0)
                __hip_atomic_store(&p.cnt[16 + pend_mt], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            pend_mt = -1;
          } else if (!poller) {
            sig_mt = mt;  // wave 4 counts it in after its next barrier
          }
          // the poller normalises its block after its NEXT tile: its producers (the
          // neighbouring workgroups' same-step tiles) have then long finished, so a norm pass
          // never waits on another workgroup's norm pass (no chain across the XCD's runs)
          if (poller) pend_mt = mt;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < TMH; ++i)
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
              for (int j = 0; j < TNH; ++j) acc[h][i][g][j] = tg_f32x4{0.f, 0.f, 0.f, 0.f};
      }
    });
    cur0 = nxt;
    if (TPI == 2) cur1 = tile_res(TPI * it + TPI + 1);
    nxt = tile_res(TPI * it + 2 * TPI);
  }
  // the last prefetches (out of range) still write LDS: drain before the workgroup ends
  __builtin_amdgcn_s_waitcnt(0);
  if (wave < 4) tg_barrier();  // balance the stagger's extra barrier
  if constexpr (NORM) {
    tg_barrier();  // every wave's stores of the last tile are acknowledged
    if (sig_mt >= 0 && wave == 0 && lane == 0)
      __hip_atomic_fetch_add(&p.cnt[16 + sig_mt], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (pend_mt >= 0) {
      norm_pass(pend_mt);
      tg_barrier();
      if (wave == 0 && lane == 0)
        __hip_atomic_store(&p.cnt[16 + pend_mt], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Configurations: (WGM, TMH, TNH) -> BM x BN
//   wide  (2, 4, 2): 256 x 256, waves 2 (M) x 4 (N), 128 x 64 per wave
//   narrow (4, 2, 3): 256 x 192, waves 4 x 2, 64 x 96 per wave (out_proj: N = 576 = 3 x 192)
constexpr int kTileBM = 256;
constexpr size_t kTileLdsWide = 2 * (256 + 256) * 128;
constexpr size_t kTileLdsNarrow = 2 * (256 + 192) * 128;

// 0: not supported; 256 or 192: the BN this shape runs with
int gemm_tile_bn(int m, int n, int k, long long ldx, long long ldw, long long ldo) {
  if (k % 64 != 0) return 0;
  switch (k / 64) {
    case 3: case 6: case 9: case 12: case 18: case 24: break;
    default: return 0;
  }
  const int bn = (n >= 1024 && n % 256 == 0) ? 256 : (n % 192 == 0 ? 192 : (n % 256 == 0 ? 256 : 0));
  if (!bn) return 0;
  // per-tile buffer ranges: 256 rows of x / out, bn rows of w
  if (256LL * ldx * 2 >= (1LL << 31) || 256LL * ldo * 2 >= (1LL << 31) ||
      static_cast<long long>(bn) * ldw * 2 >= (1LL << 31))
    return 0;
  (void)m;
  return bn;
}

long long gemm_tile_count(int m, int n, int bn) {
  return static_cast<long long>((m + kTileBM - 1) / kTileBM) * (n / bn);
}

#define VM_TG_K(WGM, TMH, TNH, NKV, LDS)                                                \
  case NKV:                                                                             \
    hipLaunchKernelGGL((gemm_tile_kernel<WGM, TMH, TNH, NKV>), grid, dim3(512), LDS, s, p); \
    break;
#define VM_TG_CFG(WGM, TMH, TNH, LDS)                                                      \
  switch (p.k / 64) {                                                                      \
    VM_TG_K(WGM, TMH, TNH, 3, LDS) VM_TG_K(WGM, TMH, TNH, 6, LDS)                          \
    VM_TG_K(WGM, TMH, TNH, 9, LDS) VM_TG_K(WGM, TMH, TNH, 12, LDS)                         \
    VM_TG_K(WGM, TMH, TNH, 18, LDS) VM_TG_K(WGM, TMH, TNH, 24, LDS)                        \
    default: break;                                                                        \
  }

// Launch on `workgroups` persistent workgroups (a multiple of 8, one per CU); the shape was
// accepted by gemm_tile_bn.
void gemm_tile_launch(const bf16_t* x, long long ldx, const bf16_t* w, long long ldw,
                      bf16_t* out, long long ldo, int m, int n, int k, int bn, int workgroups,
                      hipStream_t s) {
  TileGemmParams p{};
  p.x = x; p.ldx = ldx; p.w = w; p.ldw = ldw; p.out = out; p.ldo = ldo;
  p.m = m; p.n = n; p.k = k;
  p.ntn = n / bn;
  p.tiles = static_cast<int>(gemm_tile_count(m, n, bn));
  p.tpx = (p.tiles + 7) / 8;
  const dim3 grid(workgroups);
  if (bn == 256) {
    VM_TG_CFG(2, 4, 2, kTileLdsWide)
  } else {
    VM_TG_CFG(4, 2, 3, kTileLdsNarrow)
  }
}
#undef VM_TG_CFG
#undef VM_TG_K

// The NORM form (out_proj + the next block's residual add + RMSNorm): 256 x 192 tiles,
// K = 384 / 768 / 1152 with n = 192 / 384 / 576 (VideoMamba Ti / S / M out_proj).
bool gemm_tile_norm_ok(int n, int k, int bn) {
  return bn == 192 && ((n == 192 && k == 384) || (n == 384 && k == 768) || (n == 576 && k == 1152));
}

void gemm_tile_norm_launch(const bf16_t* x, long long ldx, const bf16_t* w, long long ldw,
                           bf16_t* out, long long ldo, float* res, long long ldr, const float* nw,
                           float eps, bf16_t* hn, long long ldh, unsigned* cnt, int m, int n,
                           int k, int workgroups, hipStream_t s) {
  TileGemmParams p{};
  p.x = x; p.ldx = ldx; p.w = w; p.ldw = ldw; p.out = out; p.ldo = ldo;
  p.m = m; p.n = n; p.k = k;
  p.ntn = n / 192;
  p.tiles = static_cast<int>(gemm_tile_count(m, n, 192));
  p.tpx = ((p.tiles + 7) / 8 + p.ntn - 1) / p.ntn * p.ntn;  // whole row blocks per XCD range
  p.res = res; p.ldr = ldr; p.nw = nw; p.hn = hn; p.ldh = ldh; p.eps = eps; p.cnt = cnt;
  const dim3 grid(workgroups);
  switch (k / 64) {
    case 6:
      hipLaunchKernelGGL((gemm_tile_kernel<4, 2, 3, 6, true, 1>), grid, dim3(512), kTileLdsNarrow, s, p);
      break;
    case 12:
      hipLaunchKernelGGL((gemm_tile_kernel<4, 2, 3, 12, true, 2>), grid, dim3(512), kTileLdsNarrow, s, p);
      break;
    case 18:
      hipLaunchKernelGGL((gemm_tile_kernel<4, 2, 3, 18, true, 3>), grid, dim3(512), kTileLdsNarrow, s, p);
      break;
    default: break;
  }
}

}  // namespace vm
