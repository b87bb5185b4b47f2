// in_proj with the depthwise causal conv1d + SiLU and the x_proj partials in its epilogue,
// for the streaming-chunk latency path (small batches, token-major).  Replaces, in one
// launch, the mixer's in_proj GEMM (mamba_simple.py:333-339) and the first kernel of the
// split-K conv_proj (causal_conv1d_fn + x_proj, :381-416); the second split-K kernel
// (xdbl_dt_tm_kernel, vm_conv_proj_sk.hip) then sums the partials and runs dt_proj.
//
// Why: at B = 1 the layer is a chain of latency-bound kernels.  in_proj
// wrote x (3144 x 1152 bf16) only for conv_proj to read it back with a 3-row halo and
// stream all of W_x per 16-token tile (14.7 us per layer at B = 1).  Here the x half of
// in_proj runs on tiles of 112 output rows that also compute the 16 rows above them (the
// conv halo: one more MFMA row block), so the workgroup that produced a 112 x 128 x tile —
// exactly one 128-channel split of the split-K x_proj — convolves it in LDS, writes u,
// and runs that split's x_proj partial on the matrix cores against a 20 KB W_x slice.
// x never reaches HBM; the raw x rows a sequence's new conv state needs are written from
// the same LDS tile.
//
// Bits.  Every x value is the in_proj GEMM's own MFMA chain (linear_dma_kernel's K order:
// 64-wide steps, two 16x16x32 MFMAs each), rounded to bf16 as in_proj stores it; the conv,
// SiLU, u rounding, x_proj MFMA operand layout and partial rows are conv_xproj_tm_kernel's
// (vm_conv_proj_sk.hip) instruction for instruction, and the reduction is that form's
// second kernel — so u / x_dbl / dt / the conv state are bit-identical to in_proj +
// vm_conv_proj_fwd's small-batch forms (the fused one is bit-identical to split-K), and
// chunked == full stays exact (tests/test_gpu_parity.py::test_in_proj_conv_proj_*).
//
// Layout: one 1-D grid of nx x-tiles (row tiles of 112 x splits) then nz z-tiles (the z
// half, 128 x 128 tiles written into z), XCD-contiguous; 8 waves (4 x 2 of 32 x 64), two
// workgroups per CU (64 KB LDS), the grid co-resident at B = 1 (261 + 225 of 512 slots).

#include "vm_conv_proj.h"

namespace vm {

typedef __attribute__((__vector_size__(8 * sizeof(short)))) short ic_bf16x8;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float ic_f32x4;
typedef __attribute__((__vector_size__(4 * sizeof(int)))) int ic_i32x4;

struct InConvParams {
  const bf16_t* x; long long ldx;  // hn (ntok, k)
  const bf16_t* w; long long ldw;  // in_proj weight (2 dim, k)
  bf16_t* z; long long ldz;        // z half of xz: (ntok, dim)
  ConvProjTmArgs a;                // conv / x_proj operands (a.x unused)
  float* part;                     // [nsplit][ntok][ep] fp32 x_proj partials
  int ntok, nsplit, ep, k;
  int nxr, nzr;                    // x row tiles (112 rows), z row tiles (128 rows)
};

constexpr int kIcRow = 128;                  // bytes per staged K row (64 bf16)
constexpr int kIcOut = 112;                  // x output rows per tile
constexpr int kIcHalo = 16;                  // rows above them computed for the conv
constexpr int kIcPitch = 136;                // bf16 pitch of the LDS x / u tile
constexpr int kIcCsSeq = 3;                  // sequences starting in a tile (out_len >= 56)
constexpr int kIcStage = (128 + 128) * kIcRow;  // one K-step stage: A and B rows
constexpr int kIcOBytes = 128 * kIcPitch * 2;   // x tile [128][kIcPitch] bf16
constexpr int kIcWBytes = 80 * kIcPitch * 2;    // W_x slice [e_pad <= 80][kIcPitch]
constexpr int kIcCBytes = kIcCsSeq * 3 * 128 * 4;
constexpr int kIcLds = (2 * kIcStage > kIcOBytes + kIcWBytes + kIcCBytes)
                           ? 2 * kIcStage : kIcOBytes + kIcWBytes + kIcCBytes;

__device__ __forceinline__ int ic_slot(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Workgroup barrier over LDS traffic only: __syncthreads() also waits vmcnt(0), which would
// make every barrier of the epilogue wait for the u / partial stores issued before it.
__device__ __forceinline__ void ic_lds_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt / expcnt at their maximum
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

template <int NK, int NB>
__global__ __launch_bounds__(512) void inproj_conv_kernel(const InConvParams q) {
  constexpr int R = kIcRow;
  constexpr int NW = 8, NT = 512;
  constexpr int WM = 32, WN = 64, TM = 2, TN = 4;
  constexpr int GA = 128 * R / (1024 * NW), GB = GA;  // 2 + 2 DMA instructions per wave
  const ConvProjTmArgs& p = q.a;
  extern __shared__ __attribute__((aligned(16))) char dsm[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // The x tiles come first in dispatch order, so the hardware spreads them one per CU
  // before any CU takes a second workgroup (x and z tiles then pair up on a CU instead of
  // whole XCDs holding only x tiles); within each part an XCD-contiguous renumbering
  // (linear_dma_kernel's) lets a row tile's splits share one L2.
  const int nx = q.nxr * q.nsplit;
  const bool xt = static_cast<int>(blockIdx.x) < nx;  // uniform
  const int h = xt ? blockIdx.x : blockIdx.x - nx;
  const int nwg = xt ? nx : gridDim.x - nx;
  const int xcd = h & 7, qq = nwg >> 3, rr = nwg & 7;
  const int lt = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (h >> 3);
  const int rt = lt / q.nsplit, sp = lt - rt * q.nsplit;
  // A rows: x tiles rt * 112 - 16 .. + 127 (rows < 0 read as zero), z tiles rt * 128 ..
  const int m0 = xt ? rt * kIcOut - kIcHalo : rt * 128;
  const int n0 = (xt ? 0 : p.dim) + sp * 128;  // W rows (output channels)

  const auto xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(q.x), 0, static_cast<int>((long long)q.ntok * q.ldx * 2), 0x00020000);
  const auto wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(q.w), 0, static_cast<int>((long long)2 * p.dim * q.ldw * 2), 0x00020000);
  int aoff[GA], boff[GB];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int o = (wave * GA + i) * 1024 + lane * 16;
    const int row = o / R, chunk = ic_slot(row, (o % R) >> 4);
    // a row above the batch (m0 + row < 0) gets a negative offset: out of range, reads 0
    // (every K step keeps it negative: kt * 128 + chunk * 16 < k * 2 <= ldx * 2)
    aoff[i] = ((m0 + row) * static_cast<int>(q.ldx)) * 2 + chunk * 16;
  }
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int o = (wave * GB + i) * 1024 + lane * 16;
    const int row = o / R, chunk = ic_slot(row, (o % R) >> 4);
    boff[i] = ((n0 + row) * static_cast<int>(q.ldw)) * 2 + chunk * 16;
  }
  auto issue = [&](int kt, int buf) {
    char* sa = dsm + buf * kIcStage;
#pragma unroll
    for (int i = 0; i < GA; ++i) dma16(xr, sa + (wave * GA + i) * 1024, aoff[i] + kt * R);
    char* sb = sa + 128 * R;
#pragma unroll
    for (int i = 0; i < GB; ++i) dma16(wr, sb + (wave * GB + i) * 1024, boff[i] + kt * R);
  };

  ic_f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = ic_f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) {
    const char* sA = dsm + buf * kIcStage;
    const char* sB = sA + 128 * R;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      ic_bf16x8 af[TM], bw[TN];
      const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const ic_bf16x8*>(sA + row * R + ic_slot(row, chunk) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + (lane & 15);
        bw[j] = *reinterpret_cast<const ic_bf16x8*>(sB + row * R + ic_slot(row, chunk) * 16);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bw[j], acc[i][j], 0, 0, 0);
    }
  };

  // ---- x tiles: the epilogue's operands, loaded during the last K step (registers) ----
  const int c0 = sp * 128;           // this split's channels
  const int c = c0 + 2 * lane;       // a thread's channel pair in the conv
  const int W = p.width;
  const int tok_lo = m0 + kIcHalo;   // first output token of an x tile
  constexpr int kWI = (NB * 16 * 16 + NT - 1) / NT;     // 16-B W_x pieces per thread
  constexpr int kCI = (kIcCsSeq * 3 * 128 + NT - 1) / NT;  // conv-state taps per thread
  uint4 wv[kWI];
  float cv[kCI];
  float wl[4], wh[4], bl = 0.0f, bh = 0.0f;  // conv taps right-aligned to 4 (conv_xproj_tm_kernel)
  const int b_lo = tok_lo / p.out_len;
  const int nbs = (xt && p.csi)
                      ? min(p.batch - 1, (tok_lo + kIcOut - 1) / p.out_len) - b_lo + 1 : 0;
  // every epilogue operand as a branch-free buffer load (absent / padding pieces read 0
  // through out-of-range offsets): a divergent "load or zero" makes hipcc wait vmcnt(0) at
  // its join, which would also drain the last K step's stage
  auto epi_loads = [&]() {
    const auto cwr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.cw), 0, p.dim * W * 4, 0x00020000);
    const auto cbr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.cb), 0, p.cb ? p.dim * 4 : 0, 0x00020000);
    const auto wxr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.wx), 0, p.e_pad * p.dim * 2, 0x00020000);
    constexpr int kOut = static_cast<int>(0x80000000u);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int kk = k - (4 - W);  // taps right-aligned: leading taps of a short filter are 0
      wl[k] = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(cwr, kk >= 0 ? (c * W + kk) * 4 : kOut, 0, 0));
      wh[k] = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(cwr, kk >= 0 ? ((c + 1) * W + kk) * 4 : kOut, 0, 0));
    }
    bl = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(cbr, c * 4, 0, 0));
    bh = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(cbr, (c + 1) * 4, 0, 0));
#pragma unroll
    for (int k = 0; k < kWI; ++k) {
      const int i = tid + k * NT;
      const int e = i >> 4, qd = i & 15;
      const int off = i < NB * 16 * 16 ? (e * p.dim + c0 + qd * 8) * 2 : kOut;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(wxr, off, 0, 0);
      wv[k] = make_uint4(v[0], v[1], v[2], v[3]);
    }
    if (nbs > 0) {  // uniform: only tiles holding a sequence start read the old conv state
#pragma unroll
      for (int k = 0; k < kCI; ++k) {
        const int i = tid + k * NT;
        const int bb = i / (3 * 128), m = (i / 128) % 3, ch = i % 128;
        const int tap = W - 1 - m;  // state column of step -(m + 1)
        cv[k] = 0.0f;
        if (bb < nbs && tap >= 0)
          cv[k] = load_dyn(p.csi, (b_lo + bb) * p.csi_sb + (long long)(c0 + ch) * p.csi_sd + tap,
                           p.csi_dtype);
      }
    }
  };

  issue(0, 0);
#pragma unroll
  for (int kt = 0; kt < NK; ++kt) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);  // stage kt has landed
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (kt + 1 < NK) issue(kt + 1, (kt + 1) & 1);
    if (kt + 1 == NK && xt) epi_loads();  // in flight during the last K step's MFMAs
    compute(kt & 1);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();  // every wave is past its last fragment reads

  // D[4(lane/16) + r][lane % 16] of every 16 x 16 block -> LDS tile [row][col] (bf16: the
  // value in_proj stores)
  bf16_t* sO = reinterpret_cast<bf16_t*>(dsm);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WN + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * WM + i * 16 + (lane >> 4) * 4 + r;
        // (+ 0.0f: linear_dma_kernel adds its zero bias, which makes a -0 sum +0)
        sO[row * kIcPitch + col] = from_f32<bf16_t>(acc[i][j][r] + 0.0f);
      }
    }
  if (!xt) {  // ---- z tile: 16-byte row stores (z column = n0 - dim), write-through ----
    ic_lds_barrier();
    const auto zr = __builtin_amdgcn_make_buffer_rsrc(
        q.z + (long long)m0 * q.ldz, 0,
        static_cast<int>(max(0, min(q.ntok - m0, 128)) * q.ldz * 2), 0x00020000);
    for (int pc = tid; pc < 128 * 16; pc += NT) {
      const int row = pc >> 4, cq = pc & 15;
      const int gm = m0 + row;
      if (gm < q.ntok)
        __builtin_amdgcn_raw_buffer_store_b128(
            *reinterpret_cast<const ic_i32x4*>(&sO[row * kIcPitch + cq * 8]), zr,
            (row * static_cast<int>(q.ldz) + (n0 - p.dim) + cq * 8) * 2, 0, kSmallStoreWT);
    }
    return;
  }

  // ---- x tile epilogue (every barrier LDS-only: the u / partial / conv-state stores stay in
  // flight until the kernel ends) ----
  bf16_t* sW = reinterpret_cast<bf16_t*>(dsm + kIcOBytes);                  // [e][kIcPitch]
  float* sC = reinterpret_cast<float*>(dsm + kIcOBytes + kIcWBytes);        // [seq][3][128]
#pragma unroll
  for (int k = 0; k < kWI; ++k) {
    const int i = tid + k * NT;
    if (i < NB * 16 * 16) *reinterpret_cast<uint4*>(&sW[(i >> 4) * kIcPitch + (i & 15) * 8]) = wv[k];
  }
#pragma unroll
  for (int k = 0; k < kCI; ++k) {
    const int i = tid + k * NT;
    if (i / (3 * 128) < nbs) sC[i] = cv[k];
  }
  ic_lds_barrier();

  // new conv state: the last `width` raw inputs of every sequence whose last step lies in
  // this tile's output rows (its W - 1 <= 3 rows before are in the halo rows)
  if (p.cso && tid < 128) {
    const int b1 = min(p.batch - 1, (tok_lo + kIcOut - 1) / p.out_len);
    for (int b = tok_lo / p.out_len; b <= b1; ++b) {
      const int tl = b * p.out_len + p.seqlen - 1;
      if (tl < tok_lo || tl >= tok_lo + kIcOut || tl >= q.ntok) continue;
      const int ch = c0 + tid;
      for (int s = 0; s < W; ++s) {
        const int te = p.seqlen - W + s;
        float v = 0.0f;
        if (te >= 0)
          v = to_f32(sO[(b * p.out_len + te - m0) * kIcPitch + tid]);
        else if (p.csi)
          v = load_dyn(p.csi, b * p.csi_sb + (long long)ch * p.csi_sd + W + te, p.csi_dtype);
        store_dyn(p.cso, b * p.cso_sb + (long long)ch * p.cso_sd + s, p.cso_dtype, v);
      }
    }
  }

  // conv + SiLU: channels c, c + 1 (one packed word), output rows 14 w .. 14 w + 13
  constexpr int kRows = kIcOut / NW;  // 14
  const int r0 = kIcHalo + wave * kRows;  // tile row of the wave's first output token
  uint32_t xw[kRows + 3];
#pragma unroll
  for (int r = 0; r < kRows + 3; ++r)
    xw[r] = *reinterpret_cast<const uint32_t*>(&sO[(r0 - 3 + r) * kIcPitch + 2 * lane]);
  const int tw = m0 + r0;  // the wave's first token
  const int bw = tw / p.out_len;
  const int sw = tw - bw * p.out_len;
  auto pack = [&](float al, float ah, bool live) -> uint32_t {
    const float ul = live ? al * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-al * kLog2e)) : 0.0f;
    const float uh = live ? ah * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-ah * kLog2e)) : 0.0f;
    return static_cast<uint32_t>(from_f32<bf16_t>(ul)) |
           (static_cast<uint32_t>(from_f32<bf16_t>(uh)) << 16);
  };
  // every row from the tile (branch-free); the rows in the first 3 steps of a sequence are
  // redone below.  (out_len >= 56 > 14: a wave's rows span at most one sequence boundary)
  uint32_t upk[kRows];
#pragma unroll
  for (int i = 0; i < kRows; ++i) {
    float al = bl, ah = bh;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      al = fmaf(wl[k], __uint_as_float(xw[i + k] << 16), al);
      ah = fmaf(wh[k], __uint_as_float(xw[i + k] & 0xffff0000u), ah);
    }
    const int st = sw + i >= p.out_len ? sw + i - p.out_len : sw + i;
    upk[i] = pack(al, ah, st < p.seqlen && tw + i < q.ntok);
  }
  // rows with step < 3: i0 + r (r = step 0, 1, 2) — the taps before the sequence are the
  // old conv state (staged in sC) or zeros, as conv_xproj_tm_kernel's redo
  const int i0 = sw < 3 ? -sw : p.out_len - sw;
  if (i0 < kRows) {  // uniform
    const int bs = sw < 3 ? bw : bw + 1;  // the sequence whose steps 0 .. 2 these rows are
    uint32_t red[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int i = i0 + r;
      red[r] = 0;
      if (i >= 0 && i < kRows) {  // uniform
        float al = bl, ah = bh;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int j = r - 3 + k;  // input step in the virtual sequence
          float vl = 0.0f, vh = 0.0f;
          if (j >= 0) {
            const uint32_t xv = *reinterpret_cast<const uint32_t*>(&sO[(r0 + i - 3 + k) * kIcPitch + 2 * lane]);
            vl = __uint_as_float(xv << 16);
            vh = __uint_as_float(xv & 0xffff0000u);
          } else if (p.csi && tw + i < q.ntok && k >= 4 - W) {
            const float2 cs = *reinterpret_cast<const float2*>(&sC[((bs - b_lo) * 3 - j - 1) * 128 + 2 * lane]);
            vl = cs.x;
            vh = cs.y;
          }
          al = fmaf(wl[k], vl, al);
          ah = fmaf(wh[k], vh, ah);
        }
        red[r] = pack(al, ah, r < p.seqlen && tw + i < q.ntok);
      }
    }
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int r = i - i0;
      upk[i] = r == 0 ? red[0] : r == 1 ? red[1] : r == 2 ? red[2] : upk[i];
    }
  }
  ic_lds_barrier();  // every wave is past its reads of the x tile: u takes its rows
  bf16_t* sU = sO;  // [112][kIcPitch]: output row i at row i
#pragma unroll
  for (int i = 0; i < kRows; ++i) {
    *reinterpret_cast<uint32_t*>(&sU[(wave * kRows + i) * kIcPitch + 2 * lane]) = upk[i];
    const int tok = tw + i;
    if (tok < q.ntok)  // write-through (agent-scope relaxed store: sc1)
      __hip_atomic_store(reinterpret_cast<uint32_t*>(p.u + (long long)tok * p.u_tl + c), upk[i],
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  ic_lds_barrier();

  // x_proj partial (conv_xproj_tm_kernel's MFMA layout): waves 0..6, tokens 16 w .. 16 w + 15
  // x all e_pad columns, K = the split's 128 channels in four 32-deep steps
  typedef __attribute__((ext_vector_type(8))) __bf16 ic_bv8;
  typedef __attribute__((ext_vector_type(4))) float ic_f4;
  ic_f4 pacc[NB];
  const bool mw = wave < kIcOut / 16;
  if (mw) {
#pragma unroll
    for (int j = 0; j < NB; ++j) pacc[j] = ic_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const ic_bv8 av = *reinterpret_cast<const ic_bv8*>(
          &sU[(wave * 16 + (lane & 15)) * kIcPitch + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const ic_bv8 bv = *reinterpret_cast<const ic_bv8*>(
            &sW[(j * 16 + (lane & 15)) * kIcPitch + ks * 32 + (lane >> 4) * 8]);
        pacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, pacc[j], 0, 0, 0);
      }
    }
  }
  ic_lds_barrier();  // the u / W_x tiles are free: stage the partial rows there
  constexpr int kPP = kSkMaxEp;
  float* sP = reinterpret_cast<float*>(dsm) + wave * 16 * kPP;
  if (mw) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int e = j * 16 + (lane & 15);
        if (e < q.ep) sP[((lane >> 4) * 4 + r) * kPP + e] = pacc[j][r];
      }
  }
  __builtin_amdgcn_wave_barrier();
  if (mw) {
    const int nq = q.ep >> 2;
    const auto pr = __builtin_amdgcn_make_buffer_rsrc(
        q.part, 0, static_cast<int>((long long)q.nsplit * q.ntok * q.ep * 4), 0x00020000);
    for (int i = lane; i < 16 * nq; i += 64) {
      const int r = i / nq, qd = i - r * nq;
      const int tok = tok_lo + wave * 16 + r;
      if (tok < q.ntok)
        __builtin_amdgcn_raw_buffer_store_b128(
            *reinterpret_cast<const ic_i32x4*>(&sP[r * kPP + 4 * qd]), pr,
            (((sp * q.ntok + tok) * q.ep) + 4 * qd) * 4, 0, kSmallStoreWT);
    }
  }
}

// x_dbl = bf16(sum of the split partials in split order) — xdbl_dt_tm_kernel's sum (from
// 0, split 0 first, fp32) without its dt phase, one thread per (token, 4 columns) so the
// whole reduction is one round of loads (that kernel's 64-token tiles take two dependent
// rounds on a 50-workgroup grid at B = 1).  dt == NULL only (the scan computes dt).
template <int NSPL>
__global__ __launch_bounds__(256) void xdbl_reduce_kernel(const InConvParams q) {
  const ConvProjTmArgs& p = q.a;
  const int q4 = (p.e + 3) >> 2;
  const int it = blockIdx.x * 256 + threadIdx.x;
  if (it >= q.ntok * q4) return;
  const int t = it / q4, e0 = (it - t * q4) * 4;
  const long long sstride = (long long)q.ntok * q.ep;
  const float* src = q.part + (long long)t * q.ep + e0;
  float4 part[NSPL];
#pragma unroll
  for (int sp = 0; sp < NSPL; ++sp) part[sp] = *reinterpret_cast<const float4*>(src + sp * sstride);
  float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int sp = 0; sp < NSPL; ++sp) {
    sum.x += part[sp].x; sum.y += part[sp].y; sum.z += part[sp].z; sum.w += part[sp].w;
  }
  const float sv[4] = {sum.x, sum.y, sum.z, sum.w};
  bf16_t* dst = p.xdbl + (long long)t * p.xd_tl + e0;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
    if (e0 + kk < p.e) dst[kk] = from_f32<bf16_t>(sv[kk]);
}

bool inproj_conv_ok(int k, const ConvProjTmArgs& a) {
  switch (k / 64) {
    case 3: case 6: case 9: case 12: case 18: case 24: break;
    default: return false;
  }
  const long long ntok = static_cast<long long>(a.batch) * a.out_len;
  return k % 64 == 0 && a.batch >= 1 && a.batch <= kSkMaxBatch && a.dim % 128 == 0 &&
         a.dim <= 2048 && a.out_len >= 56 && a.e_pad <= 80 && a.e_pad % 16 == 0 &&
         (a.e + 3) / 4 * 4 <= kSkMaxEp && (a.wdt == nullptr || a.r_pad <= 64) &&
         a.width >= 1 && a.width <= 4 && ntok * a.u_tl * 2 < (1ll << 31);
}

void inproj_conv_launch(const InConvParams& q0, hipStream_t s) {
  InConvParams q = q0;
  const unsigned grid = static_cast<unsigned>((q.nxr + q.nzr) * q.nsplit);
  const size_t lds = kIcLds;
  switch ((q.k / 64) * 16 + q.a.e_pad / 16) {
#define VM_IC(NKV, NBV)                                                                    \
    case NKV * 16 + NBV:                                                                   \
      hipLaunchKernelGGL((inproj_conv_kernel<NKV, NBV>), dim3(grid), dim3(512), lds, s, q); \
      break;
#define VM_IC_K(NKV) VM_IC(NKV, 1) VM_IC(NKV, 2) VM_IC(NKV, 3) VM_IC(NKV, 4) VM_IC(NKV, 5)
    VM_IC_K(3) VM_IC_K(6) VM_IC_K(9) VM_IC_K(12) VM_IC_K(18) VM_IC_K(24)
#undef VM_IC_K
#undef VM_IC
    default: break;
  }
}

}  // namespace vm

using namespace vm;

extern "C" long long vm_in_proj_conv_proj_workspace_bytes(int batch, int out_len, int dim, int e) {
  return conv_proj_sk_workspace_bytes(batch, out_len, dim, e);
}

extern "C" int vm_in_proj_conv_proj_fits(int k, int batch, int out_len, int dim, int e, int e_pad,
                                         int r_pad, int width, int has_dt) {
  ConvProjTmArgs a{};
  a.batch = batch; a.out_len = out_len; a.dim = dim; a.e = e; a.e_pad = e_pad;
  a.r_pad = r_pad; a.width = width; a.u_tl = dim;
  a.wdt = has_dt ? reinterpret_cast<const bf16_t*>(16) : nullptr;
  return inproj_conv_ok(k, a) ? 1 : 0;
}

extern "C" int vm_in_proj_conv_proj_fwd(
    const void* hn, long long ldh, const void* w_in, long long ldw, int k,
    void* z, long long ldz, const float* conv_weight, const float* conv_bias,
    const void* cs_in, int cs_in_dtype, long long csi_sb, long long csi_sd,
    void* cs_out, int cs_out_dtype, long long cso_sb, long long cso_sd,
    const void* wx_pad, int e, int e_pad, const void* wdt_pad, int r, int r_pad,
    void* u, long long u_tl, void* xdbl, long long xd_tl, void* dt, long long dt_tl,
    int out_len, int batch, int dim, int seqlen, int width, void* workspace,
    long long workspace_bytes, vm_stream_t stream) {
  if (!hn || !w_in || !z || !conv_weight || !wx_pad || !u || !xdbl || (dt && !wdt_pad)) {
    vmhost::set_error("vm_in_proj_conv_proj_fwd: null required pointer");
    return VM_E_INVALID;
  }
  ConvProjTmArgs a{};
  a.x = nullptr; a.x_tl = 0; a.cw = conv_weight; a.cb = conv_bias;
  a.csi = cs_in; a.csi_dtype = cs_in_dtype; a.csi_sb = csi_sb; a.csi_sd = csi_sd;
  a.cso = cs_out; a.cso_dtype = cs_out_dtype; a.cso_sb = cso_sb; a.cso_sd = cso_sd;
  a.wx = static_cast<const bf16_t*>(wx_pad); a.e = e; a.e_pad = e_pad;
  a.wdt = dt ? static_cast<const bf16_t*>(wdt_pad) : nullptr; a.r = r; a.r_pad = r_pad;
  a.u = static_cast<bf16_t*>(u); a.u_tl = u_tl; a.xdbl = static_cast<bf16_t*>(xdbl);
  a.xd_tl = xd_tl; a.dt = static_cast<bf16_t*>(dt); a.dt_tl = dt_tl;
  a.out_len = out_len; a.batch = batch; a.dim = dim; a.seqlen = seqlen; a.width = width;
  const long long ntok = static_cast<long long>(batch) * out_len;
  if (!inproj_conv_ok(k, a) || seqlen < 1 || seqlen > out_len || r < 1 || r > e ||
      (dt && r_pad != 32 && r_pad != 64) || (cs_in && !vmhost::dtype_ok(cs_in_dtype)) ||
      (cs_out && !vmhost::dtype_ok(cs_out_dtype)) || ldh < k || ldw < k || ldz < dim ||
      ldh % 8 || ldw % 8 || ldz % 8 || u_tl < dim || u_tl % 2 || xd_tl < e || xd_tl % 2 ||
      (dt && (dt_tl < dim || dt_tl % 8)) || out_len % 2 || e % 2 ||
      !vmhost::aligned16(hn) || !vmhost::aligned16(w_in) || !vmhost::aligned16(z) ||
      !vmhost::aligned16(wx_pad) || (dt && !vmhost::aligned16(dt)) ||
      (dt && !vmhost::aligned16(wdt_pad)) || (reinterpret_cast<uintptr_t>(u) & 3) ||
      (reinterpret_cast<uintptr_t>(xdbl) & 3) || ntok * ldh * 2 >= (1ll << 31) ||
      2ll * dim * ldw * 2 >= (1ll << 31) || ntok > (1 << 30)) {
    vmhost::set_error("vm_in_proj_conv_proj_fwd: unsupported shape (bf16; k in {192 .. 1536} "
                      "by 64-steps; batch <= %d, out_len >= 56 and even, dim %% 128 == 0 and "
                      "<= 2048, R + 2N <= %d, e_pad <= 80, width <= 4; 16-byte aligned rows; "
                      "hn under 2 GB)", kSkMaxBatch, kSkMaxEp);
    return VM_E_INVALID;
  }
  if (cs_out && cs_in == cs_out) {
    vmhost::set_error("vm_in_proj_conv_proj_fwd: conv_state_out must not alias conv_state_in");
    return VM_E_INVALID;
  }
  const long long need = conv_proj_sk_workspace_bytes(batch, out_len, dim, e);
  if (!workspace || workspace_bytes < need) {
    vmhost::set_error("vm_in_proj_conv_proj_fwd: needs a workspace of %lld bytes "
                      "(vm_in_proj_conv_proj_workspace_bytes)", need);
    return VM_E_INVALID;
  }
  InConvParams q{};
  q.x = static_cast<const bf16_t*>(hn); q.ldx = ldh;
  q.w = static_cast<const bf16_t*>(w_in); q.ldw = ldw;
  q.z = static_cast<bf16_t*>(z); q.ldz = ldz;
  q.a = a;
  q.part = static_cast<float*>(workspace);
  q.ntok = static_cast<int>(ntok);
  q.nsplit = dim / 128;
  q.ep = (e + 3) / 4 * 4;
  q.k = k;
  q.nxr = static_cast<int>((ntok + kIcOut - 1) / kIcOut);
  q.nzr = static_cast<int>((ntok + 127) / 128);
  hipStream_t s = static_cast<hipStream_t>(stream);
  inproj_conv_launch(q, s);
  if (dt) {
    conv_proj_sk_reduce_launch(a, q.part, s);
  } else {
    const unsigned blocks = static_cast<unsigned>((ntok * ((e + 3) / 4) + 255) / 256);
    switch (q.nsplit) {
#define VM_XR(NS) case NS: hipLaunchKernelGGL(xdbl_reduce_kernel<NS>, dim3(blocks), dim3(256), 0, s, q); break;
      VM_XR(1) VM_XR(2) VM_XR(3) VM_XR(4) VM_XR(5) VM_XR(6) VM_XR(7) VM_XR(8)
      VM_XR(9) VM_XR(10) VM_XR(11) VM_XR(12) VM_XR(13) VM_XR(14) VM_XR(15) VM_XR(16)
#undef VM_XR
      default: break;
    }
  }
  return vmhost::launch_status("vm_in_proj_conv_proj_fwd");
}
