// Token-major selective scan for gfx950: one lane per channel, sequential in time.
//
// Same math as vm_scan.hip (_selective_scan_ref, models/videomamba/mamba_simple.py:30-106)
// on the token-major layout the mixer uses: u / delta / z / out rows are (batch, step,
// channel) with channel stride 1, so one wave reads one 128-byte line per operand per step.
// A lane owns one channel and keeps its 16 states in registers as 8 packed fp32 pairs; per
// (step, state) the work is the irreducible  a = exp2(delta*A),  h = a*h + (delta*u)*B,
// y += h*C  (delta and the states in log2 units) — 4 VALU + 1 transcendental, no
// cross-lane scan and no re-sweep.  B_t / C_t (shared by every channel of a batch row) are
// one wave-uniform scalar load per step (both rows of the mixer's x_dbl in one
// s_load_dwordx16), used directly as SGPR operands; u / delta / z are buffer loads
// prefetched 8 steps ahead.  The kernels of this file:
//   scan_seq_kernel (MODE 0)   single pass per (batch row, 128 channels), chip-filling batches;
//   scan_seq_dtp_kernel        the same with dt_proj folded in (dt from the x_dbl rows on
//                              MFMA, no delta stream) — the bench's kernel at B > 8;
//   scan_chunk_kernel          small batches (e.g. the B = 1 streaming chunk): the sequence
//                              cut into segments of T steps, 8 segments per workgroup;
//                              PASS 1 (zero entry state -> end state and delta sum, composed
//                              per workgroup into a block aggregate), PASS 2 (entry state
//                              from h0 and the preceding blocks' aggregates, then the steps
//                              again emitting y), either as two launches or as ONE launch
//                              whose blocks hand their aggregates on through a sync buffer
//                              (PASS 3 below);
//   scan_seq_kernel MODE 1 / 2 + scan_seq_carry_kernel: the summary / carry / final form for
//                              operands the scalar-load path cannot take (LDS-staged B / C).

#include <stdlib.h>

#include "vm_scan.h"

namespace vm {

struct SeqWork {
  float* hend;  // [B][S][D][kMaxN]  segment end states from a zero entry state (pass 1)
  float* sdel;  // [B][S][D]         segment delta sums (pass 1)
  float* hin;   // [B][S][D][kMaxN]  segment entry states (carry)
  int S, seg_len;
};

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kTS = 32;       // steps per LDS block
constexpr int kPF = 8;        // u / delta / z prefetch distance in steps
constexpr int kMaxSeg = 256;  // segments per sequence
constexpr int kSeqNW = 2;     // waves (channel groups of 64) per workgroup
constexpr bool kSeqXcdRemap = true;  // grids renumbered per XCD (see scan_seq_kernel)
constexpr bool kSeqDeltaAhead = true;  // next step's delta computed a step early
constexpr bool kSeqGateAhead = true;   // next step's output-gate factor computed a step early

// Buffer descriptor over a wave-uniform base: per-step byte offsets go in soffset (SGPR),
// the lane's channel offset in voffset, so no per-lane 64-bit address math runs per step.
// Host guarantees every in-range byte offset is < kSeqRange; kSeqDead (>= the records
// count) makes a store a hardware no-op, so stores need no branch.
constexpr int kSeqRange = 1 << 30;
constexpr int kSeqDead = 0x7ffffff0;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  void* ub = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(ub, 0, kSeqRange, 0x00020000);
}
// Logical workgroup ids in XCD order: the hardware hands workgroup H to XCD H % 8, so the
// renumbering H -> (H % 8) * (n / 8) + H / 8 gives each XCD a contiguous range of logical
// ids (n % 8 == 0; otherwise the ids are left alone).
__device__ __forceinline__ void xcd_order(int& gx, int& gy, int& gz) {
  const int n = gridDim.x * gridDim.y * gridDim.z;
  if ((n & 7) != 0) return;
  const int h = gx + gridDim.x * (gy + gridDim.y * gz);
  const int l = (h & 7) * (n >> 3) + (h >> 3);
  gx = l % gridDim.x;
  gy = (l / gridDim.x) % gridDim.y;
  gz = l / (gridDim.x * gridDim.y);
}

template <typename T>
__device__ __forceinline__ uint32_t bload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  if constexpr (sizeof(T) == 2)
    return __builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0);
  else
    return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}
template <typename T, int POL = 0>
__device__ __forceinline__ void bstore(T v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  if constexpr (sizeof(T) == 2)
    __builtin_amdgcn_raw_buffer_store_b16(v, r, voff, soff, POL);
  else
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, soff, POL);
}
template <typename T>
__device__ __forceinline__ float raw_f32(uint32_t r) {
  if constexpr (sizeof(T) == 2) return __uint_as_float(r << 16);
  else return __uint_as_float(r);
}

// MODE 0: single pass (entry state h0), MODE 1: summary, MODE 2: final with entry states.
// SB: B_t / C_t (16 states, unit state stride, 4-byte aligned rows) come in as scalar
// loads — wave-uniform SGPR operands of the VALU ops, one step ahead — instead of the LDS
// staging + broadcast reads.
// PK (requires SB): the four per-state VALU ops run as packed-f32 ops over state pairs
// (v_pk_mul_f32 delta*A and (delta*u)*B, v_pk_fma_f32 for h and y) — B/C pairs are SGPR
// pairs — leaving the 16 v_exp_f32 unpaired.  Measured in the step mix
// (tools/probes/pk_rate.hip) a pair costs ~4.7 cycles per packed op against ~3.6 per
// scalar op in dependent chains, so the step drops from ~343 to ~265 cycles per wave.
template <typename T, int NW, int MODE, bool SP, bool HZ, bool SB, bool PK, bool BC1 = false,
          bool PAIR = false>
__global__ __launch_bounds__(64 * NW) void scan_seq_kernel(const ScanParams p, const SeqWork w) {
  static_assert(!PK || SB, "packed pairs take B/C from SGPR pairs");
  static_assert(NW * 64 >= 4 * kTS, "B/C staging needs 4 threads per block step");
  typedef __attribute__((address_space(4))) const uint32_t* cptr;
  constexpr int NWD = kMaxN * sizeof(T) / 4;  // 32-bit words per B (or C) row
  __shared__ __attribute__((aligned(16))) float sbc[2][kTS][2 * kMaxN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD order: the channel groups of one batch row (consecutive logical ids) share an
  // XCD, so their common B / C rows come into one L2 instead of up to eight (calibrated
  // fetch 9.9 -> 7.6 GB per launch at B = 336, time unchanged; profiles/r02_scan_xcd_pmc.txt)
  int gx = blockIdx.x, gy = blockIdx.y, gz = blockIdx.z;
  if constexpr (kSeqXcdRemap) xcd_order(gx, gy, gz);
  const int seg = gy;
  const int b = gz;
  const int d_raw = (gx * NW + wave) * 64 + lane;
  const bool active = d_raw < p.dim;
  const int d = active ? d_raw : p.dim - 1;
  const int N = p.dstate;
  const int L = p.seqlen;
  const int t_beg = seg * w.seg_len;
  const int t_end = min(L, t_beg + w.seg_len);
  const PairSel ps = pair_sel<PAIR>(p, b);
  const long long ws_row = (static_cast<long long>(b) * w.S + seg) * p.dim + d;

  // LG (single pass with softplus): delta is carried in log2 units, dl' = softplus(x)*log2e
  // = log2(1 + 2^(x*log2e)), so the exp argument is dl'*A with A unscaled and the softplus
  // loses its two scaling multiplies.  Then du' = du*log2e, so the states run as
  // h' = h*log2e (converted once at entry and exit), D is pre-scaled the same way, and the
  // output's ln2 factor rides on the SiLU gate's 1+e term as an FMA.
  constexpr bool LG = MODE == 0 && SP;
  const float lg_in = LG ? kLog2e : 1.0f;

  // state pairs (n, n+1) live in f2 register pairs: scalar code addresses .x / .y, the
  // packed form operates on whole pairs
  f2 A2[kMaxN / 2], h[kMaxN / 2];
#pragma unroll
  for (int n = 0; n < kMaxN; ++n) {
    const float a = n < N ? ps.A[d * N + n] * (LG ? 1.0f : kLog2e) : 0.0f;
    float h_init = 0.0f;
    if constexpr (MODE == 0) {
      if (n < N && ps.h0)
        h_init = load_dyn(ps.h0, ps.hb * p.h0_sb + d * p.h0_sd + n, p.h0_dtype) * lg_in;
    }
    if constexpr (MODE == 2) h_init = w.hin[ws_row * kMaxN + n];
    if (n & 1) {
      A2[n >> 1].y = a;
      h[n >> 1].y = h_init;
    } else {
      A2[n >> 1].x = a;
      h[n >> 1].x = h_init;
    }
  }
  const float Dv = (ps.D ? ps.D[d] : 0.0f) * lg_in;
  const float bias = (ps.dbias ? ps.dbias[d] : 0.0f) * lg_in;
  // Wave-uniform row bases (buffer descriptors) + the lane's channel byte offset.
  const int d0 = __builtin_amdgcn_readfirstlane((gx * NW + wave) * 64 < p.dim
                                                    ? (gx * NW + wave) * 64
                                                    : p.dim - 1);
  constexpr int ES = sizeof(T);
  const int voff = (d - d0) * ES;
  const int voff_st = active ? voff : kSeqDead;
  const auto ur = uniform_rsrc(static_cast<const T*>(p.u) + b * p.u_sb + d0);
  const auto dr_ = uniform_rsrc(static_cast<const T*>(p.delta) + b * p.dl_sb + d0);
  const auto zr = uniform_rsrc(HZ ? static_cast<const T*>(p.z) + b * p.z_sb + d0
                                  : static_cast<const T*>(p.u));
  const auto orr = uniform_rsrc(static_cast<T*>(p.out) + b * p.o_sb + d0);
  const int us = static_cast<int>(p.u_sl) * ES, ds = static_cast<int>(p.dl_sl) * ES;
  const int zs = static_cast<int>(p.z_sl) * ES, os = static_cast<int>(p.o_sl) * ES;

  // B/C staging role: thread -> (block step sr, operand B|C, states sn0..sn0+7)
  const int sr = tid >> 2;
  const int sq = tid & 3;
  const bool stager = tid < 4 * kTS;
  const bool isC = (sq >> 1) != 0;
  const T* ssrc = static_cast<const T*>(isC ? p.C : p.B) + b * (isC ? p.c_sb : p.b_sb);
  const long long ssl = isC ? p.c_sl : p.b_sl;
  const long long ssn = isC ? p.c_sn : p.b_sn;
  const int sn0 = (sq & 1) * 8;
  auto stage_load = [&](int tb, float (&v)[8]) {
    const int t = tb + sr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = sn0 + j;
      v[j] = (stager && t < L && n < N) ? to_f32(ssrc[t * ssl + n * ssn]) : 0.0f;
    }
  };
  auto stage_store = [&](int buf, const float (&v)[8]) {
    if (stager) {
      float* dst = &sbc[buf][sr][(isC ? kMaxN : 0) + sn0];
      *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
  };

  // SGPR B/C needs no LDS blocks: step in groups of kPF so a short segment does not run a
  // whole 32-step block of masked steps
  constexpr int kBlk = SB ? kPF : kTS;
  const int nblk = t_end > t_beg ? (t_end - t_beg + kBlk - 1) / kBlk : 0;
  float stg[8];
  if constexpr (!SB) {
    if (nblk > 0) {
      stage_load(t_beg, stg);
      stage_store(0, stg);
    }
    __syncthreads();
  }
  const T* Bq = static_cast<const T*>(p.B) + b * p.b_sb;
  const T* Cq = static_cast<const T*>(p.C) + b * p.c_sb;
  uint32_t bcw[2][2 * NWD];  // [step parity][B words | C words]
  // byte offsets of a step's B / C rows within this batch row fit 32 bits (host checks),
  // so a step costs one scalar multiply; BC1: C directly follows B in the same row
  // (the mixer's x_dbl layout) and both arrive in one s_load_dwordx16
  const uint32_t bsl = static_cast<uint32_t>(p.b_sl * sizeof(T));
  const uint32_t csl = static_cast<uint32_t>(p.c_sl * sizeof(T));
  auto bc_load = [&](int t, uint32_t (&dst)[2 * NWD]) {
    const cptr bp = (cptr)(reinterpret_cast<const char*>(Bq) + static_cast<uint32_t>(t) * bsl);
    if constexpr (BC1) {
#pragma unroll
      for (int i = 0; i < 2 * NWD; ++i) dst[i] = bp[i];
    } else {
      const cptr cp = (cptr)(reinterpret_cast<const char*>(Cq) + static_cast<uint32_t>(t) * csl);
#pragma unroll
      for (int i = 0; i < NWD; ++i) {
        dst[i] = bp[i];
        if constexpr (MODE != 1) dst[NWD + i] = cp[i];
      }
    }
  };

  // Drain the parameter loads (A, D, bias, entry state) here: left pending they merge into
  // the step loop's header and force a conservative vmcnt wait on every iteration.
  __builtin_amdgcn_s_waitcnt(0);
  uint32_t ru[kPF], rd[kPF], rz[kPF];
  const int tlast = L > 0 ? L - 1 : 0;
  if constexpr (SB) {
    if (nblk > 0) bc_load(t_beg, bcw[0]);
  }
  if (nblk > 0) {
#pragma unroll
    for (int j = 0; j < kPF; ++j) {
      const int t = min(t_beg + j, tlast);
      ru[j] = bload<T>(ur, voff, t * us);
      rd[j] = bload<T>(dr_, voff, t * ds);
      rz[j] = HZ && MODE != 1 ? bload<T>(zr, voff, t * zs) : 0u;
      // keep the loop's per-step (u, delta, z) issue order: a prologue the scheduler
      // regroups (all u, then all delta, ...) makes the compiler's loop-header vmcnt waits
      // 8 / 16 loads tighter than the steady state needs
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  float sdel = 0.0f;
  // delta of a step from its raw dt (log2 units under LG)
  auto delta_of = [&](uint32_t raw) {
    const float dr = raw_f32<T>(raw);
    float dl;
    if constexpr (LG) {
      const float x = fmaf(dr, kLog2e, bias);  // (dt + bias) * log2e
      dl = x > 20.0f * kLog2e ? x : __builtin_amdgcn_logf(1.0f + __builtin_amdgcn_exp2f(x));
    } else {
      dl = dr + bias;
      if (SP) dl = softplus_fast(dl);
    }
    return dl;
  };
  // The next step's delta is computed at the end of the current step (its dt landed kPF - 1
  // steps ago), so the softplus chain shares a scheduling region with this step's y
  // reduction instead of heading the next step's dependent chain (kSeqDeltaAhead).
  float dl_nx = 0.0f;
  // likewise the output gate's factor z / ((1 + e^-z) log2e) of the next step (LG with z)
  constexpr bool kGA = kSeqGateAhead && LG && HZ && MODE != 1;
  auto gate_of = [&](uint32_t raw) {
    const float zz = raw_f32<T>(raw);
    return zz * __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_exp2f(-zz * kLog2e), kLog2e, kLog2e));
  };
  float g_nx = 0.0f;
  // One step of the recurrence (step t, prefetch slot j): consume the registers loaded
  // kPF steps ago and refill the slot at the given (per-lane voffset, SGPR soffset) pairs.
  const float* blk = &sbc[0][0][0];
  int tb_lds = t_beg;  // first step of the LDS block `blk` holds (non-SB path)
  auto step = [&](uint32_t (&ru)[kPF], uint32_t (&rd)[kPF], uint32_t (&rz)[kPF], const int t,
                  const int j, const bool live, const int vu, const int su, const int vd,
                  const int sd, const int vz, const int sz) {
      const float uu = raw_f32<T>(ru[j]);
      const uint32_t rdj = rd[j];
      const float zz = raw_f32<T>(rz[j]);
      ru[j] = bload<T>(ur, vu, su);
      rd[j] = bload<T>(dr_, vd, sd);
      if (HZ && MODE != 1) rz[j] = bload<T>(zr, vz, sz);
      if constexpr (SB) {
        // this step's B/C rows (issued one step ago) have landed — explicit lgkmcnt(0),
        // scalar loads return out of order — then fetch the next step's rows
        __builtin_amdgcn_s_waitcnt(0xC07F);
        bc_load(t + 1 < tlast ? t + 1 : tlast, bcw[(j + 1) & 1]);
      }
      // keep each step's refill loads at the step head: the scheduler would otherwise
      // sink them below all eight steps, collapsing the prefetch distance to zero
      // (letting ALU work cross this barrier, mask 0x787, measured 10-25 % slower)
      __builtin_amdgcn_sched_barrier(0);
      float dl = kSeqDeltaAhead ? dl_nx : delta_of(rdj);
      if constexpr (kSeqDeltaAhead) dl_nx = delta_of(rd[(j + 1) & (kPF - 1)]);
      float gf = 0.0f;
      if constexpr (kGA) {
        gf = g_nx;
        g_nx = gate_of(rz[(j + 1) & (kPF - 1)]);
      }
      dl = live ? dl : 0.0f;
      const float du = dl * uu;
      // output gate; under LG it also carries y's ln2 factor: z / ((1 + e) * log2e)
      auto gate = [&](float y) {
        if constexpr (LG) {
          if constexpr (kGA) return y * gf;
          if (HZ)
            return y * (zz * __builtin_amdgcn_rcpf(
                                 fmaf(__builtin_amdgcn_exp2f(-zz * kLog2e), kLog2e, kLog2e)));
          return y * kLn2f;
        } else {
          return HZ ? y * silu_fast(zz) : y;
        }
      };
      if constexpr (PK) {
        const uint32_t (&cw)[2 * NWD] = bcw[j & 1];
        const f2 dl2 = {dl, dl}, du2 = {du, du};
        f2 ya = {Dv * uu, 0.0f}, yb = {0.0f, 0.0f};  // two pair chains
#pragma unroll
        for (int q = 0; q < kMaxN / 2; ++q) {
          f2 Bp, Cp;
          if constexpr (sizeof(T) == 2) {
            Bp = f2{__uint_as_float(cw[q] << 16), __uint_as_float(cw[q] & 0xffff0000u)};
            Cp = f2{__uint_as_float(cw[NWD + q] << 16), __uint_as_float(cw[NWD + q] & 0xffff0000u)};
          } else {
            Bp = f2{__uint_as_float(cw[2 * q]), __uint_as_float(cw[2 * q + 1])};
            Cp = f2{__uint_as_float(cw[NWD + 2 * q]), __uint_as_float(cw[NWD + 2 * q + 1])};
          }
          const f2 x = dl2 * A2[q];
          const f2 a = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
          h[q] = __builtin_elementwise_fma(a, h[q], du2 * Bp);
          if constexpr (MODE != 1) {
            if (q & 1) yb = __builtin_elementwise_fma(h[q], Cp, yb);
            else ya = __builtin_elementwise_fma(h[q], Cp, ya);
          }
        }
        if constexpr (MODE == 1) {
          sdel += dl;
        } else {
          const f2 ys = ya + yb;
          const float y = gate(ys.x + ys.y);
          bstore<T>(from_f32<T>(y), orr, live ? voff_st : kSeqDead, ps.orow(t) * os);
        }
        return;
      }
      float Bv[kMaxN], Cv[kMaxN];
      if constexpr (SB) {
        const uint32_t (&cw)[2 * NWD] = bcw[j & 1];
#pragma unroll
        for (int n = 0; n < kMaxN; ++n) {
          if constexpr (sizeof(T) == 2) {
            const uint32_t wb = cw[n >> 1], wc = cw[NWD + (n >> 1)];
            Bv[n] = __uint_as_float((n & 1) ? (wb & 0xffff0000u) : (wb << 16));
            Cv[n] = __uint_as_float((n & 1) ? (wc & 0xffff0000u) : (wc << 16));
          } else {
            Bv[n] = __uint_as_float(cw[n]);
            Cv[n] = __uint_as_float(cw[NWD + n]);
          }
        }
      } else {
        const float4* row = reinterpret_cast<const float4*>(blk + (t - tb_lds) * 2 * kMaxN);
#pragma unroll
        for (int q = 0; q < kMaxN / 4; ++q) {
          const float4 bq = row[q];
          Bv[4 * q] = bq.x; Bv[4 * q + 1] = bq.y; Bv[4 * q + 2] = bq.z; Bv[4 * q + 3] = bq.w;
          if constexpr (MODE != 1) {
            const float4 cq = row[kMaxN / 4 + q];
            Cv[4 * q] = cq.x; Cv[4 * q + 1] = cq.y; Cv[4 * q + 2] = cq.z; Cv[4 * q + 3] = cq.w;
          }
        }
      }
      if constexpr (MODE == 1) {
        sdel += dl;
#pragma unroll
        for (int q = 0; q < kMaxN / 2; ++q) {
          h[q].x = fmaf(__builtin_amdgcn_exp2f(dl * A2[q].x), h[q].x, du * Bv[2 * q]);
          h[q].y = fmaf(__builtin_amdgcn_exp2f(dl * A2[q].y), h[q].y, du * Bv[2 * q + 1]);
        }
      } else {
        float y0 = Dv * uu, y1 = 0.0f;  // two chains: ILP for the 16-term dot product
#pragma unroll
        for (int q = 0; q < kMaxN / 2; ++q) {
          h[q].x = fmaf(__builtin_amdgcn_exp2f(dl * A2[q].x), h[q].x, du * Bv[2 * q]);
          h[q].y = fmaf(__builtin_amdgcn_exp2f(dl * A2[q].y), h[q].y, du * Bv[2 * q + 1]);
          y0 = fmaf(h[q].x, Cv[2 * q], y0);
          y1 = fmaf(h[q].y, Cv[2 * q + 1], y1);
        }
        const float y = gate(y0 + y1);
        // unconditional store (a branch here makes the loop-carried vmcnt accounting
        // conservative): dead lanes / steps get an out-of-range voffset instead
        bstore<T>(from_f32<T>(y), orr, live ? voff_st : kSeqDead, ps.orow(t) * os);
      }
  };

  if constexpr (kSeqDeltaAhead) dl_nx = delta_of(rd[0]);
  if constexpr (kGA) g_nx = gate_of(rz[0]);
  int k0 = 0;
  if constexpr (SB) {
    // Main loop: whole 8-step groups that are all live and whose refills (kPF steps
    // ahead) stay inside the sequence — per-lane step offsets in VGPRs, one SGPR base per
    // group, no clamps.  Measured ~5 % faster than the clamped form (scan_lab "voff").
    // (u and delta share their step stride here — the mixer's layout — so one offset
    // table serves both and the kernel stays at <= 96 VGPRs)
    int vou[kPF], voz[kPF];
#pragma unroll
    for (int j = 0; j < kPF; ++j) {
      vou[j] = voff + j * us;
      voz[j] = voff + j * zs;
    }
    int t0 = t_beg;
    if (ds == us) {
      for (; t0 + kPF <= t_end && t0 + 2 * kPF <= L; t0 += kPF) {
        const int su = (t0 + kPF) * us, sz = (t0 + kPF) * zs;
#pragma unroll
        for (int j = 0; j < kPF; ++j)
          step(ru, rd, rz, t0 + j, j, true, vou[j], su, vou[j], su, voz[j], sz);
      }
    }
    // Tail (SGPR path): clamped steps on registers of their own.  Re-issuing the tail's
    // prefetch (instead of continuing on the main loop's registers) keeps the main loop's
    // prefetch registers loop-local: carried into a second loop they made the register
    // allocator shuffle in-flight load destinations at the loop head (v_mov + vmcnt(0)).
    if (t0 < t_end) {
      uint32_t tu[kPF], td[kPF], tz[kPF];
#pragma unroll
      for (int j = 0; j < kPF; ++j) {
        const int t = min(t0 + j, tlast);
        tu[j] = bload<T>(ur, voff, t * us);
        td[j] = bload<T>(dr_, voff, t * ds);
        tz[j] = HZ && MODE != 1 ? bload<T>(zr, voff, t * zs) : 0u;
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (kSeqDeltaAhead) dl_nx = delta_of(td[0]);
      if constexpr (kGA) g_nx = gate_of(tz[0]);
      for (int tb = t0; tb < t_end; tb += kPF) {
#pragma unroll
        for (int j = 0; j < kPF; ++j) {
          const int t = tb + j;
          const int tn = min(t + kPF, tlast);
          step(tu, td, tz, t, j, t < t_end, voff, tn * us, voff, tn * ds, voff, tn * zs);
        }
      }
    }
    k0 = nblk;
  }
  // LDS path: clamped blocks.
  for (int k = k0; k < nblk; ++k) {
    const int tb = t_beg + k * kBlk;
    const bool more = k + 1 < nblk;
    if constexpr (!SB) {
      if (more) stage_load(tb + kTS, stg);
      blk = &sbc[k & 1][0][0];
      tb_lds = tb;
    }
    for (int g = 0; g < kBlk; g += kPF) {
#pragma unroll
      for (int j = 0; j < kPF; ++j) {
        const int t = tb + g + j;
        const int tn = min(t + kPF, tlast);
        step(ru, rd, rz, t, j, t < t_end, voff, tn * us, voff, tn * ds, voff, tn * zs);
      }
    }
    if constexpr (!SB) {
      if (more) stage_store((k + 1) & 1, stg);
      __syncthreads();
    }
  }
  if constexpr (MODE == 1) {
    if (active) {
#pragma unroll
      for (int n = 0; n < kMaxN; ++n) w.hend[ws_row * kMaxN + n] = (n & 1) ? h[n >> 1].y : h[n >> 1].x;
      w.sdel[ws_row] = sdel;
    }
  } else {
    if (t_end >= L && active) {  // the segment that ends the sequence
      if (ps.hl) {
#pragma unroll
        for (int n = 0; n < kMaxN; ++n)
          if (n < N)
            store_dyn(ps.hl, ps.hb * p.hl_sb + d * p.hl_sd + n, p.hl_dtype,
                      ((n & 1) ? h[n >> 1].y : h[n >> 1].x) * (LG ? kLn2f : 1.0f));
      }
      for (int t = L; t < p.out_len; ++t) bstore<T>(from_f32<T>(0.0f), orr, voff, t * os);
    }
  }
}

// ============================================================ dt_proj inside the scan
// scan_seq_dtp_kernel: the single-pass bench kernel (MODE 0, scalar B|C rows, packed state
// pairs, delta in log2 units) with dt_proj folded in.  Instead of reading a precomputed
// dt row (written by conv_proj and read straight back: 2 * B*L*D bytes of HBM traffic per
// layer), every wave computes the dt of its 64 channels for 16 steps at a time on the
// matrix cores,  dt[t][c] = bf16( sum_k dt_low[t][k] * W_dt[c][k] )  (mamba_simple.py:
// 409-413: dt = dt_proj.weight @ x_dbl[:, :R]^T, rounded to the model dtype there), from
// the x_dbl rows the scan already reads for B|C:
//   A = dt_low rows (16 steps x 16*NKS k, v_mfma_f32_16x16x16_bf16 fragments by buffer
//       load, one block ahead), B = W_dt^T (this wave's 64 channels, staged in LDS once),
//   D (16 steps x 16 channels per tile, 4 tiles) -> bf16 pairs -> an LDS block
//   [channel][16 steps], from which each lane reads its own channel's steps 4 at a time.
// Per step the arithmetic is the single-pass kernel's; the buffer load of dt becomes an
// LDS read, and per 16 steps a wave adds 4 * NKS MFMAs, 8 bf16 packs and 4 + 4 LDS ops.
// Every token's dt is computed from its own x_dbl row in a fixed order, so the result does
// not depend on the sequence length (chunked == full stays exact).
constexpr int kDtG = 16;    // steps per dt block
// the y epilogue of a step (pair sum, gate, bf16 round, store) runs in the next step's
// scheduling region, where the independent state updates fill the dependent chain's hazard
// gaps (s_nop) instead of the step's tail
constexpr bool kDtpYLate = true;
constexpr int kDtRow = 10;  // dwords per channel row of the LDS dt block (16 bf16 + pad)
typedef short dtp_s4 __attribute__((ext_vector_type(4)));
typedef __bf16 dtp_b2 __attribute__((ext_vector_type(2)));
typedef float dtp_f2 __attribute__((ext_vector_type(2)));
// two fp32 -> two bf16 (round to nearest even) in one v_cvt_pk_bf16_f32: lo = a, hi = b
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(dtp_f2{a, b}, dtp_b2));
}
typedef float dtp_f4 __attribute__((ext_vector_type(4)));

template <int NKS>
__global__ __launch_bounds__(64 * kSeqNW) void scan_seq_dtp_kernel(const ScanParams p,
                                                                    const DtpArgs q) {
  typedef __attribute__((address_space(4))) const uint32_t* cptr;
  typedef bf16_t T;
  constexpr int NW = kSeqNW;
  constexpr int NWD = kMaxN * 2 / 4;  // 32-bit words per B (or C) row
  constexpr int ES = 2;
  constexpr int KP = 16 * NKS + 4;    // bf16 per LDS W_dt row (8-byte pad: fewer bank conflicts)
  __shared__ __attribute__((aligned(16))) bf16_t sW[NW][64 * KP];
  constexpr int DR = kDtRow;
  __shared__ __attribute__((aligned(16))) uint32_t sD[NW][64 * DR];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int gx = blockIdx.x, gy = blockIdx.y, gz = blockIdx.z;
  xcd_order(gx, gy, gz);
  const int b = gz;
  const int d0 = __builtin_amdgcn_readfirstlane((gx * NW + wave) * 64);  // dim % 128 == 0
  const int d = d0 + lane;
  const int L = p.seqlen;
  const int tlast = L > 0 ? L - 1 : 0;

  // W_dt rows of this wave's channels -> LDS (lane = channel, 16*NKS bf16)
  {
    const bf16_t* wrow = q.wdt + static_cast<long long>(d) * q.wdt_ld;
    bf16_t* srow = &sW[wave][lane * KP];
#pragma unroll
    for (int i = 0; i < 4 * NKS; ++i) {  // 16 * NKS bf16 as 4-element (8-byte) pieces
      const uint2 v = *reinterpret_cast<const uint2*>(wrow + 4 * i);
      *reinterpret_cast<uint2*>(srow + 4 * i) = v;
    }
  }

  f2 A2[kMaxN / 2], h[kMaxN / 2];
#pragma unroll
  for (int n = 0; n < kMaxN; ++n) {
    const float a = p.A[d * kMaxN + n];
    const float h_init =
        p.h0 ? load_dyn(p.h0, b * p.h0_sb + d * p.h0_sd + n, p.h0_dtype) * kLog2e : 0.0f;
    if (n & 1) {
      A2[n >> 1].y = a;
      h[n >> 1].y = h_init;
    } else {
      A2[n >> 1].x = a;
      h[n >> 1].x = h_init;
    }
  }
  const float Dv = (p.D ? p.D[d] : 0.0f) * kLog2e;
  const float bias = (p.dbias ? p.dbias[d] : 0.0f) * kLog2e;
  const int voff = lane * ES;
  const auto ur = uniform_rsrc(static_cast<const T*>(p.u) + b * p.u_sb + d0);
  const auto zr = uniform_rsrc(static_cast<const T*>(p.z) + b * p.z_sb + d0);
  const auto orr = uniform_rsrc(static_cast<T*>(p.out) + b * p.o_sb + d0);
  // dt_low rows of this batch row; rows past out_len read as 0 (bounded descriptor)
  const auto dtr = [&]() {
    const uint64_t a = reinterpret_cast<uint64_t>(q.dtl + b * q.dtl_sb);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
    void* ub = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(
        ub, 0, static_cast<int>(static_cast<long long>(p.out_len) * q.dtl_sl * ES), 0x00020000);
  }();
  const int us = static_cast<int>(p.u_sl) * ES, zs = static_cast<int>(p.z_sl) * ES;
  const int os = static_cast<int>(p.o_sl) * ES, dls = static_cast<int>(q.dtl_sl) * ES;
  const T* Bq = static_cast<const T*>(p.B) + b * p.b_sb;
  const uint32_t bsl = static_cast<uint32_t>(p.b_sl * ES);
  uint32_t bcw[2][2 * NWD];
  auto bc_load = [&](int t, uint32_t (&dst)[2 * NWD]) {
    const cptr bp = (cptr)(reinterpret_cast<const char*>(Bq) + static_cast<uint32_t>(t) * bsl);
#pragma unroll
    for (int i = 0; i < 2 * NWD; ++i) dst[i] = bp[i];
  };

  // ---- the dt block: A fragments (dt_low rows tg .. tg+15) in `af`, W_dt^T from LDS ----
  const int a_voff = ((lane & 15) * static_cast<int>(q.dtl_sl) + 4 * (lane >> 4)) * ES;
  // the last 16-column block's lanes past dt_rank (dt_rank % 4 == 0) read 0 through an
  // out-of-range offset instead of the row's B values: the reference's dt never reads
  // them, and a non-finite B times the zero W_dt padding would make dt NaN
  const int a_last = 16 * (NKS - 1) + 4 * (lane >> 4) < q.dt_rank
                         ? a_voff + 16 * (NKS - 1) * ES
                         : static_cast<int>(0x80000000u);
  auto a_load = [&](int tg, uint2 (&af)[NKS]) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int off = ks == NKS - 1 ? a_last : a_voff + 16 * ks * ES;
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(dtr, off, tg * dls, 0);
      af[ks] = uint2{v[0], v[1]};
    }
  };
  // in stages, so no step waits on a dependent MFMA / LDS chain: the MFMAs of channel
  // tiles [t0, t1) into dacc, later the bf16 pack + LDS store of all four tiles
  dtp_f4 dacc[4];
  auto dt_mfma = [&](const uint2 (&af)[NKS], const int t0, const int t1) {
#pragma unroll
    for (int tile = t0; tile < t1; ++tile) {
      dacc[tile] = dtp_f4{0.0f, 0.0f, 0.0f, 0.0f};
      const bf16_t* wb = &sW[wave][(16 * tile + (lane & 15)) * KP + 4 * (lane >> 4)];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const uint2 bw = *reinterpret_cast<const uint2*>(wb + 16 * ks);
        dacc[tile] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(
            __builtin_bit_cast(dtp_s4, af[ks]), __builtin_bit_cast(dtp_s4, bw), dacc[tile], 0,
            0, 0);
      }
    }
  };
  typedef unsigned dq_t __attribute__((ext_vector_type(2)));
  auto dt_store = [&]() {
#pragma unroll
    for (int tile = 0; tile < 4; ++tile) {
      // D[4 (lane>>4) + i][lane & 15] -> channel 16 tile + (lane & 15), steps 4 (lane>>4) + i
      const uint32_t p01 = cvt_pk_bf16(dacc[tile][0], dacc[tile][1]);
      const uint32_t p23 = cvt_pk_bf16(dacc[tile][2], dacc[tile][3]);
      *reinterpret_cast<dq_t*>(&sD[wave][(16 * tile + (lane & 15)) * DR + 2 * (lane >> 4)]) =
          dq_t{p01, p23};
    }
  };
  // a lane's own channel, steps 4k .. 4k+3 of the block
  auto dq_read = [&](int k) {
    return *reinterpret_cast<const dq_t*>(&sD[wave][lane * DR + 2 * k]);
  };
  auto dt_of = [&](const dq_t& dq, int j) {  // step j % 4 of a quad
    const uint32_t w = (j & 2) ? dq[1] : dq[0];
    return __uint_as_float((j & 1) ? (w & 0xffff0000u) : (w << 16));
  };
  auto delta_of = [&](float dr) {  // delta' = softplus(dt + bias) * log2e (log2 units)
    const float x = fmaf(dr, kLog2e, bias);
    return x > 20.0f * kLog2e ? x : __builtin_amdgcn_logf(1.0f + __builtin_amdgcn_exp2f(x));
  };
  auto gate_of = [&](uint32_t raw) {
    const float zz = raw_f32<T>(raw);
    return zz * __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_exp2f(-zz * kLog2e), kLog2e, kLog2e));
  };

  // prologue: block 0's dt, the first quad, u / z / B|C of the first kPF steps
  uint2 af[NKS];
  a_load(0, af);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();  // sW is written (each wave reads only its own rows; one barrier is cheap)
  dt_mfma(af, 0, 4);
  dt_store();
  dq_t dqa[4];  // the block's four quads (steps 4k .. 4k+3), each read a quad ahead
  dqa[0] = dq_read(0);
  dqa[1] = dqa[2] = dqa[3] = dqa[0];
  // ru / rz hold the raw bf16 of u / z
  uint32_t ru[kPF], rz[kPF];
  bc_load(0, bcw[0]);
#pragma unroll
  for (int j = 0; j < kPF; ++j) {
    const int t = min(j, tlast);
    ru[j] = bload<T>(ur, voff, t * us);
    rz[j] = bload<T>(zr, voff, t * zs);
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_s_waitcnt(0);
  float dl_nx = delta_of(dt_of(dqa[0], 0));
  float g_nx = gate_of(rz[0]);
  // kDtpYLate: the previous step's y accumulators, gate and store offset (dead: out of range)
  f2 ya_p = {0.0f, 0.0f}, yb_p = {0.0f, 0.0f};
  float gf_p = 0.0f;
  int vo_p = kSeqDead, so_p = 0;
  auto y_finish = [&](const f2& ya, const f2& yb, float gf, int vo, int so) {
    const f2 ys = ya + yb;
    const float y = (ys.x + ys.y) * gf;
    bstore<T>(from_f32<T>(y), orr, vo, so);
  };

  // One step: t, slot j = t % 16 within the dt block; refill slot j % kPF at (vu, su)/(vz, sz).
  auto step = [&](const int t, const int j, const bool live, const int vu, const int su,
                  const int vz, const int sz, auto&& mid) {
    const int s = j & (kPF - 1);
    float dl = dl_nx;
    dl = live ? dl : 0.0f;
    const f2 dl2 = {dl, dl};
    const float uu = raw_f32<T>(ru[s]);
    ru[s] = bload<T>(ur, vu, su);
    rz[s] = bload<T>(zr, vz, sz);
    // du as a genuine register pair (one packed multiply): a {du, du} pair formed with
    // op_sel leaves its unused half free for the allocator, which can make it the
    // destination of an in-flight refill load — the packed read then waits for that load
    // (a vmcnt(1) at the block head)
    const f2 du2 = dl2 * f2{uu, uu};
    f2 ya = f2{Dv * uu, 0.0f};
    __builtin_amdgcn_s_waitcnt(0xC07F);  // this step's B|C rows have landed
    bc_load(t + 1 < tlast ? t + 1 : tlast, bcw[(j + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);
    // the block bookkeeping goes after that wait, so the next step's lgkmcnt(0) (a step
    // later) is the first to wait for its LDS reads / writes
    mid();
    if constexpr (kDtpYLate) y_finish(ya_p, yb_p, gf_p, vo_p, so_p);
    // the next step's delta and gate a step early (as scan_seq_kernel); its dt sits in the
    // current quad, the next quad (j % 4 == 3), or the next block's first quad (j == 15)
    dl_nx = delta_of(dt_of(dqa[((j + 1) >> 2) & 3], (j + 1) & 3));
    const float gf = g_nx;
    g_nx = gate_of(rz[(s + 1) & (kPF - 1)]);
    const uint32_t (&cw)[2 * NWD] = bcw[j & 1];
    f2 yb = {0.0f, 0.0f};
#pragma unroll
    for (int qq = 0; qq < kMaxN / 2; ++qq) {
      const f2 Bp = f2{__uint_as_float(cw[qq] << 16), __uint_as_float(cw[qq] & 0xffff0000u)};
      const f2 Cp = f2{__uint_as_float(cw[NWD + qq] << 16),
                       __uint_as_float(cw[NWD + qq] & 0xffff0000u)};
      const f2 x = dl2 * A2[qq];
      const f2 a = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
      h[qq] = __builtin_elementwise_fma(a, h[qq], du2 * Bp);
      if (qq & 1) yb = __builtin_elementwise_fma(h[qq], Cp, yb);
      else ya = __builtin_elementwise_fma(h[qq], Cp, ya);
    }
    if constexpr (kDtpYLate) {
      ya_p = ya;
      yb_p = yb;
      gf_p = gf;
      vo_p = live ? voff : kSeqDead;
      so_p = t * os;
    } else {
      y_finish(ya, yb, gf, live ? voff : kSeqDead, t * os);
    }
  };
  // block bookkeeping in step j of the block starting at tg: prefetch the next block's
  // A fragments at j == 0, the next quad at j % 4 == 0 (j < 12); the next block's dt: the
  // MFMAs at j == 9 / 10, the pack + LDS store at j == 12 (after the last quad read of this
  // block, j == 8), its first quad read at j == 14 (consumed from step 15 on)
  uint2 afn[NKS];
  auto around = [&](const int tg, const int j) {
    if (j == 0) a_load(tg + kDtG, afn);
    if ((j & 3) == 0 && j < 12) dqa[(j >> 2) + 1] = dq_read((j >> 2) + 1);
    if (j == 9) dt_mfma(afn, 0, 2);
    if (j == 10) dt_mfma(afn, 2, 4);
    if (j == 12) dt_store();
    if (j == 14) dqa[0] = dq_read(0);
  };

  int t0 = 0;
  // Main loop: whole 16-step blocks whose u / z refills (kPF ahead) stay in the sequence:
  // no clamps; the refill byte offsets are two running SGPRs advanced by one scalar add per
  // step (asm: left to itself the compiler precomputes all 32 of a block's offsets and
  // spills them to VGPR lanes, which costs a v_readlane per load)
  int su = kPF * us, sz = kPF * zs;
  for (; t0 + kDtG + kPF <= L; t0 += kDtG) {
#pragma unroll
    for (int j = 0; j < kDtG; ++j) {
      step(t0 + j, j, true, voff, su, voff, sz, [&]() { around(t0, j); });
      asm volatile("s_add_u32 %0, %0, %1" : "+s"(su) : "s"(us) : "scc");
      asm volatile("s_add_u32 %0, %0, %1" : "+s"(sz) : "s"(zs) : "scc");
    }
  }
  // Tail: clamped refills and live masks, same block structure.
  for (; t0 < L; t0 += kDtG) {
#pragma unroll
    for (int j = 0; j < kDtG; ++j) {
      const int t = t0 + j;
      const int tn = min(t + kPF, tlast);
      step(t, j, t < L, voff, tn * us, voff, tn * zs, [&]() { around(t0, j); });
    }
  }
  if constexpr (kDtpYLate) y_finish(ya_p, yb_p, gf_p, vo_p, so_p);  // the last step's y
  if (L > 0) {
#pragma unroll
    for (int n = 0; n < kMaxN; ++n)
      if (p.hl)
        store_dyn(p.hl, b * p.hl_sb + d * p.hl_sd + n, p.hl_dtype,
                  ((n & 1) ? h[n >> 1].y : h[n >> 1].x) * kLn2f);
  }
  for (int t = L; t < p.out_len; ++t) bstore<T>(from_f32<T>(0.0f), orr, voff, t * os);
}

// ============================================================ chunked form (small batches)
// The sequence is cut into segments of T steps; a workgroup holds kChW consecutive segments
// of one 64-channel group (one wave per segment, lane = channel), so the chip fills even at
// B = 1 (M-16f: 18 groups x 25 blocks x 8 waves = 3,600 waves).  Two launches:
//   PASS 1: each wave runs its segment from a zero state (no output) -> end state and delta
//     sum to LDS; the workgroup composes its 8 segments there (wave w owns states 2w, 2w+1)
//     -> every segment's entry offset E_j and delta prefix P_j relative to the block entry,
//     and the block aggregate (H, S) -> workspace.
//   PASS 2: the workgroup first walks the block aggregates before it from h0 to its block
//     entry H_blk (wave w: states 2w, 2w+1; shared through LDS), then segment j enters at
//     exp2(A P_j) H_blk + E_j and runs its T steps emitting y (and h_last at the end of the
//     sequence).  (A separate carry launch between the passes cost ~5 us + a kernel
//     boundary per layer at B = 1.)
// Per step the math is the single-pass kernel's packed-pair recurrence in log2 units
// (delta' = softplus(x) log2e, states h' = h log2e), B_t / C_t rows as scalar loads.
// Compared with the summary / carry / final form it replaces for SGPR-eligible operands,
// the carry never leaves the chip's LDS except for one aggregate per block.
constexpr int kChW = 8;  // segments (waves) per workgroup
// chunked scan, PASS 1 step loop: B|C rows fetched in pairs of steps, two steps ahead (a
// 4-slot SGPR ring, one lgkmcnt(0) per pair): scalar loads return out of order, so a ring
// deeper than one step needs the wait to cover whole groups.  PASS 2 keeps one row one step
// ahead (its C rows double the ring: SGPR spills in its loop cost more than the wait saves)
constexpr bool kChBcPairs = true;
constexpr int kChSPW = kMaxN / kChW;  // states a wave composes / publishes / walks
// LBC (one-launch bf16 B|C rows, blocks of at most kChLbcRows steps): the block's B|C rows
// staged once into LDS as fp32, read per step by a broadcast ds_read one step ahead instead
// of scalar loads (out-of-order returns, so the SGPR ring could not run deeper than a pair)
// and their SALU unpacking
constexpr int kChLbcRows = 256;
constexpr int kChLbcPer = kChLbcRows * 4 / (64 * kChW);  // 16-byte row pieces per thread
constexpr int kChPoll = kChSPW == 2 ? 8 : 4;  // preceding blocks polled per round (one-launch)
static_assert(kMaxN % kChW == 0 && (kChSPW == 1 || kChSPW == 2), "1 or 2 states per wave");

struct ChunkWork {
  float* segE;  // [B][nblk][kChW][D][kMaxN]  entry offsets (log2 units)
  float* segP;  // [B][nblk][kChW][D]         delta' prefixes
  float* aggH;  // [B][nblk][D][kMaxN]        block end states from a zero entry
  float* aggS;  // [B][nblk][D]               block delta' sums
  int T;        // steps per segment
  int nblk;     // blocks per sequence
  // one-launch form (PASS 3), all in the caller's zero-initialised sync buffer:
  unsigned* err;     // word 0: sticky error word
  unsigned* epoch;   // word 1: the tag of the last launch that used the buffer
  unsigned* done;    // word 2: blocks of the current launch that have read the epoch
  unsigned long long* gran;  // [B][groups][nblk][kMaxN + 1][64] {tag, value} granules
};

template <bool V> struct BoolTag { static constexpr bool value = V; };
// a thread's share of a block aggregate row (K consecutive states of one channel), loaded as
// one 4 * K-byte access
template <int K> struct alignas(4 * K) AggShare { float v[K] = {}; };

// dt_proj inside the chunked scan (DTP, ABI v11): each wave computes its own segment's dt
// (at most kChDtpT steps) on the matrix cores into an LDS block before its step loops, with
// exactly the fused conv_proj's dt_proj arithmetic (vm_conv_proj_sk.hip: A = the x_dbl rows'
// first R columns zero-padded to r_pad, B = W_dt rows, v_mfma_f32_16x16x32_bf16 over
// r_pad / 32 k-steps in order, bf16 by round-to-nearest-even), so dt is bit-identical to the
// rows conv_proj would have written: conv_proj skips them and the scan reads x_dbl instead.
constexpr int kChDtpT = 64;              // max segment length with dt_proj inside
constexpr int kChDtpPitch = kChDtpT + 8;  // bf16 per channel row of a wave's dt block
constexpr int kChDtpWPitch = 64 + 8;      // bf16 per W_dt row in LDS (r_pad <= 64)

template <typename T, int PASS, bool SP, bool HZ, bool BC1, bool PAIR, bool DTP = false,
          bool LBC = false>
__global__ __launch_bounds__(64 * kChW) void scan_chunk_kernel(const ScanParams p, const ChunkWork w,
                                                               const DtpArgs q) {
  typedef __attribute__((address_space(4))) const uint32_t* cptr;
  constexpr int NWD = kMaxN * sizeof(T) / 4;  // 32-bit words per B (or C) row
  constexpr int ES = sizeof(T);
  static_assert(!DTP || sizeof(T) == 2, "dt_proj inside the scan is bf16 only");
  static_assert(!LBC || (PASS == 3 && BC1 && sizeof(T) == 2), "LDS B|C rows: one launch, bf16 B|C");
  // sH: PASS 1 segment end states; PASS 2 the staged block aggregates, then H_blk in sH[0].
  // sA: A of the workgroup's 64 channels, transposed to [state][channel].
  __shared__ float sH[kChW][kMaxN][64];
  __shared__ float sS[kChW][64];
  __shared__ float sA[kMaxN][64];
  __shared__ float sHb[PASS == 3 ? kMaxN : 1][64];  // one-launch form: the block entry state
  __shared__ unsigned s_tag;  // one-launch form: this launch's hand-off tag
  // DTP: the group's W_dt rows [channel][r_pad] and each wave's dt block [channel][step]
  __shared__ __attribute__((aligned(16))) bf16_t sWd[DTP ? 64 * kChDtpWPitch : 8];
  __shared__ __attribute__((aligned(16))) bf16_t sDT[DTP ? kChW * 64 * kChDtpPitch : 8];
  // LBC: the block's B|C rows (step t at row t - block start), fp32
  __shared__ __attribute__((aligned(16))) float sBC[LBC ? kChLbcRows : 1][2 * kMaxN];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int gx = blockIdx.x, gy = blockIdx.y, gz = blockIdx.z;
  const int blk = gy;
  const int b = gz;
  const int d0 = __builtin_amdgcn_readfirstlane(gx * 64);
  const int d_raw = d0 + lane;
  const bool active = d_raw < p.dim;
  const int d = active ? d_raw : p.dim - 1;
  const int N = p.dstate;
  const int L = p.seqlen;
  const int t_beg = (blk * kChW + wave) * w.T;
  const int t_end = min(L, t_beg + w.T);
  const long long D = p.dim;
  const long long rowE = ((static_cast<long long>(b) * w.nblk + blk) * kChW) * D;  // + j*D + d
  const long long rowA = (static_cast<long long>(b) * w.nblk) * D;                  // + k*D + d
  const PairSel ps = pair_sel<PAIR>(p, b);
  const int nch = min(64, p.dim - d0);  // live channels of this group

  // Start-up loads are issued as whole-line, lane-contiguous accesses and waited for once:
  // per-lane strided loads (A[d][n] at a 64-byte lane stride, the aggregates' state pairs)
  // touched ~32 cache lines per wave-instruction, and with 8 waves each issuing ~80 of them
  // the address path, not the memory, set the kernel's start-up time at B = 1.
  //   A: the group's 64 x N floats are contiguous — 2 coalesced dwords per thread
  // Every start-up load is a buffer load whose range ends where its operand does (0 bytes
  // for an absent one), so none sits behind a branch: hipcc waits vmcnt(0) at the join of
  // a "load or zero" branch, and round 4's form paid five dependent round trips here.
  float aval[kChSPW];
  {
    const auto ar = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(ps.A + static_cast<long long>(d0) * N), 0, nch * N * 4, 0x00020000);
#pragma unroll
    for (int k = 0; k < kChSPW; ++k) {
      const int e = tid + k * 64 * kChW;  // element of the [64][N] tile
      aval[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ar, e * 4, 0, 0));
    }
  }
  auto vec_load = [&](const float* v) {  // v[d], 0 when v is null
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(v), 0, v ? p.dim * 4 : 0,
                                                     0x00020000);
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, d * 4, 0, 0));
  };
  const float Dv = vec_load(ps.D) * kLog2e;
  const float bias = vec_load(ps.dbias) * kLog2e;
  // states this wave composes across segments / blocks: kChSPW * wave (+ 1)
  const int n0 = kChSPW * wave;

  // PASS 2 entry operands: this segment's entry offset and delta prefix, the entry state's
  // two composed states, and the aggregates of up to kCW preceding blocks (each block's 64
  // channels x 16 states are one contiguous 4 KB row: a coalesced float2 per thread)
  constexpr int kCW = 16;
  // one thread's share of a block aggregate's 64 channels x 16 states: kChSPW consecutive
  // states of channel tid / (16 / kChSPW)
  constexpr int kTPC = kMaxN / kChSPW;  // threads per channel
  typedef AggShare<kChSPW> agv_t;
  float Pj = 0.0f;
  float Hs[kChSPW];
#pragma unroll
  for (int i = 0; i < kChSPW; ++i) Hs[i] = 0.0f;
  f2 Ej[kMaxN / 2];
  agv_t agH[kCW];
  float agS[kCW * 64 / (64 * kChW)];
  if constexpr (PASS == 3) {
    // h0 (fp32 or bf16): both forms issued, the absent one over a 0-byte range
    const bool h32 = ps.h0 && p.h0_dtype != VM_DTYPE_BF16, h16 = ps.h0 && p.h0_dtype == VM_DTYPE_BF16;
    const long long hrow = static_cast<long long>(ps.hb) * p.h0_sb;
    const int hspan = static_cast<int>((p.dim - 1) * p.h0_sd + N);  // elements of the row
    const auto hr32 = __builtin_amdgcn_make_buffer_rsrc(
        h32 ? const_cast<float*>(static_cast<const float*>(ps.h0) + hrow) : nullptr, 0,
        h32 ? hspan * 4 : 0, 0x00020000);
    const auto hr16 = __builtin_amdgcn_make_buffer_rsrc(
        h16 ? const_cast<bf16_t*>(static_cast<const bf16_t*>(ps.h0) + hrow) : nullptr, 0,
        h16 ? hspan * 2 : 0, 0x00020000);
#pragma unroll
    for (int i = 0; i < kChSPW; ++i) {
      int el = n0 + i < N ? static_cast<int>(d * p.h0_sd) + n0 + i : 0x1ffffff0;
      asm volatile("" : "+v"(el));  // a select, not a branch around the loads
      const float v32 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(hr32, el * 4, 0, 0));
      const uint32_t v16 = __builtin_amdgcn_raw_buffer_load_b16(hr16, el * 2, 0, 0);
      Hs[i] = __uint_as_float(v16 << 16) + v32;  // one of the two read 0 (no select to sink into)
    }
  }
  if constexpr (PASS == 2) {
    Pj = w.segP[rowE + wave * D + d];
    const float4* ep = reinterpret_cast<const float4*>(&w.segE[(rowE + wave * D + d) * kMaxN]);
#pragma unroll
    for (int q = 0; q < kMaxN / 4; ++q) {
      const float4 v = ep[q];
      Ej[2 * q] = f2{v.x, v.y};
      Ej[2 * q + 1] = f2{v.z, v.w};
    }
    if (ps.h0) {
#pragma unroll
      for (int i = 0; i < kChSPW; ++i)
        if (n0 + i < N) Hs[i] = load_dyn(ps.h0, ps.hb * p.h0_sb + d * p.h0_sd + n0 + i, p.h0_dtype);
    }
    const int ci = tid / kTPC;  // channel of this thread's states
#pragma unroll
    for (int j = 0; j < kCW; ++j) {
      agH[j] = agv_t{};
      if (j < blk && ci < nch)
        agH[j] = *reinterpret_cast<const agv_t*>(&w.aggH[(rowA + j * D + d0) * kMaxN + kChSPW * tid]);
    }
#pragma unroll
    for (int k = 0; k < kCW / kChW; ++k) {
      const int j = k * kChW + (tid >> 6);
      agS[k] = j < blk && lane < nch ? w.aggS[rowA + j * D + d0 + lane] : 0.0f;
    }
  }
  // a thread's aggregate share -> LDS sH[j][state][channel]
  auto stage_agg = [&](int j, const agv_t& v) {
    const int c = tid / kTPC, n = kChSPW * (tid % kTPC);
#pragma unroll
    for (int i = 0; i < kChSPW; ++i) sH[j][n + i][c] = v.v[i];
  };
  const int voff = lane * ES;
  const int voff_st = active ? voff : kSeqDead;
  const auto ur = uniform_rsrc(static_cast<const T*>(p.u) + b * p.u_sb + d0);
  const auto dr_ = uniform_rsrc(static_cast<const T*>(p.delta) + b * p.dl_sb + d0);
  const auto zr = uniform_rsrc(HZ ? static_cast<const T*>(p.z) + b * p.z_sb + d0
                                  : static_cast<const T*>(p.u));
  const auto orr = uniform_rsrc(static_cast<T*>(p.out) + b * p.o_sb + d0);
  const int us = static_cast<int>(p.u_sl) * ES, ds = static_cast<int>(p.dl_sl) * ES;
  const int zs = static_cast<int>(p.z_sl) * ES, os = static_cast<int>(p.o_sl) * ES;
  const T* Bq = static_cast<const T*>(p.B) + b * p.b_sb;
  const T* Cq = static_cast<const T*>(p.C) + b * p.c_sb;
  const uint32_t bsl = static_cast<uint32_t>(p.b_sl * ES);
  const uint32_t csl = static_cast<uint32_t>(p.c_sl * ES);
  constexpr int kBcSlots = kChBcPairs ? 4 : 2;
  uint32_t bcw[kBcSlots][2 * NWD];
  auto bc_load = [&](int t, uint32_t (&dst)[2 * NWD]) {
    const cptr bp = (cptr)(reinterpret_cast<const char*>(Bq) + static_cast<uint32_t>(t) * bsl);
    if constexpr (BC1) {
#pragma unroll
      for (int i = 0; i < 2 * NWD; ++i) dst[i] = bp[i];
    } else {
      const cptr cp = (cptr)(reinterpret_cast<const char*>(Cq) + static_cast<uint32_t>(t) * csl);
#pragma unroll
      for (int i = 0; i < NWD; ++i) {
        dst[i] = bp[i];
        if constexpr (PASS != 1) dst[NWD + i] = cp[i];
      }
    }
  };
  const int tlast = L > 0 ? L - 1 : 0;
  // Warm this XCD's L2 with the block's B / C rows (one dword per 128-byte line, issued with
  // the start-up loads): the per-step scalar row loads, one step ahead, then hit L2 instead
  // of paying an infinity-cache / HBM round trip every step.
  uint32_t warm[2] = {0u, 0u};
  const int blk_t0 = blk * kChW * w.T;
  typedef __attribute__((ext_vector_type(4))) unsigned lbc_u4;
  lbc_u4 lbcv[LBC ? kChLbcPer : 1];
  if constexpr (LBC) {  // the block's B|C rows, 16-byte pieces, consumed after the start-up wait
    const int bt1 = min(L, blk_t0 + kChW * w.T);
    const char* base = reinterpret_cast<const char*>(Bq) + static_cast<long long>(blk_t0) * bsl;
    const int span = bt1 > blk_t0 ? (bt1 - blk_t0 - 1) * static_cast<int>(bsl) + 2 * kMaxN * ES : 0;
    const auto lr = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, span, 0x00020000);
#pragma unroll
    for (int k = 0; k < kChLbcPer; ++k) {
      const int pc = static_cast<int>(threadIdx.x) + k * 64 * kChW;
      lbcv[k] = __builtin_bit_cast(lbc_u4, __builtin_amdgcn_raw_buffer_load_b128(
                                               lr, (pc >> 2) * static_cast<int>(bsl) + (pc & 3) * 16, 0, 0));
    }
  } else {
    const int bt0 = blk_t0;
    const int bt1 = min(L, bt0 + kChW * w.T);
    if (bt1 > bt0) {
      const char* base = reinterpret_cast<const char*>(Bq) + static_cast<long long>(bt0) * bsl;
      const int span = (bt1 - bt0 - 1) * static_cast<int>(bsl) + 2 * kMaxN * ES;
      const int line = static_cast<int>(threadIdx.x) * 128;
      // (the loads' values are consumed only after the start-up wait below: a consumer here
      // made hipcc wait for each warm-up load on the spot)
      const auto wr0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, span, 0x00020000);
      warm[0] = __builtin_amdgcn_raw_buffer_load_b32(wr0, line, 0, 0);
      if constexpr (!BC1) {
        const char* cb = reinterpret_cast<const char*>(Cq) + static_cast<long long>(bt0) * csl;
        const int cspan = (bt1 - bt0 - 1) * static_cast<int>(csl) + kMaxN * ES;
        const auto wr1 = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(cb), 0,
                                                           PASS != 1 ? cspan : 0, 0x00020000);
        warm[1] = __builtin_amdgcn_raw_buffer_load_b32(wr1, line, 0, 0);
      }
    }
  }
  uint32_t ru[kPF], rd[kPF], rz[kPF];
  float sdel = 0.0f;
  if (t_beg < t_end) {
    if constexpr (!LBC) {
      bc_load(t_beg, bcw[0]);
      if constexpr (kChBcPairs) bc_load(min(t_beg + 1, tlast), bcw[1]);
    }
#pragma unroll
    for (int j = 0; j < kPF; ++j) {
      const int t = min(t_beg + j, tlast);
      ru[j] = bload<T>(ur, voff, t * us);
      rd[j] = DTP ? 0u : bload<T>(dr_, voff, t * ds);
      rz[j] = HZ && PASS == 2 ? bload<T>(zr, voff, t * zs) : 0u;
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // DTP: the group's W_dt rows (64 x r_pad <= 64 x 64 bf16: one 16-byte piece per thread;
  // rows past dim read 0), written to LDS after the start-up wait
  typedef __attribute__((ext_vector_type(4))) unsigned wv4;
  wv4 wdt_piece = {0u, 0u, 0u, 0u};
  const int wdt_ppr = DTP ? q.wdt_ld >> 3 : 1;  // pieces per row (r_pad 32 or 64)
  static_assert(64 * 8 <= 64 * kChW, "one W_dt piece per thread");
  if constexpr (DTP) {
    const int rp = q.wdt_ld;
    const auto wr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(q.wdt + static_cast<long long>(d0) * rp), 0, nch * rp * 2, 0x00020000);
    const int row = tid / wdt_ppr, pc = tid - row * wdt_ppr;
    int off = tid < 64 * wdt_ppr ? (row * rp + pc * 8) * 2 : 0x7ffffff0;
    asm volatile("" : "+v"(off));
    wdt_piece = __builtin_bit_cast(wv4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0));
  }
  // This launch's hand-off tag (PASS 3): the buffer's epoch + 1 (never 0, the zeroed
  // buffer's value).  Every block reads the epoch here, with the start-up loads, and adds
  // itself to `done` at its very end; the block that completes the count (so every block
  // has read the epoch) resets the count and advances the epoch for the next launch.  Tags
  // only grow over a buffer's launches, so granules left by an earlier launch — of any
  // shape — never match (until 2^32 - 1 launches wrap).  (Round 4 counted itself in here,
  // before PASS 1: two dependent agent-scope round trips on every block's start-up path.)
  unsigned ep = 0;
  if constexpr (PASS == 3)  // (every thread: a tid == 0 branch would wait at its join)
    ep = __hip_atomic_load(w.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // one wait for every start-up load (parameters, entry operands, prologue, the epoch): left
  // pending they would merge into the step loop's header waits
  __builtin_amdgcn_s_waitcnt(0);
  asm volatile("" ::"v"(warm[0]), "v"(warm[1]));  // the L2 warm-up loads are not dead
  if constexpr (LBC) {  // bf16 -> fp32 (exact), into sBC before the start-up barrier
#pragma unroll
    for (int k = 0; k < kChLbcPer; ++k) {
      const int pc = static_cast<int>(threadIdx.x) + k * 64 * kChW;
      float* dst = &sBC[pc >> 2][(pc & 3) * 8];
      *reinterpret_cast<float4*>(dst) =
          make_float4(__uint_as_float(lbcv[k][0] << 16), __uint_as_float(lbcv[k][0] & 0xffff0000u),
                      __uint_as_float(lbcv[k][1] << 16), __uint_as_float(lbcv[k][1] & 0xffff0000u));
      *reinterpret_cast<float4*>(dst + 4) =
          make_float4(__uint_as_float(lbcv[k][2] << 16), __uint_as_float(lbcv[k][2] & 0xffff0000u),
                      __uint_as_float(lbcv[k][3] << 16), __uint_as_float(lbcv[k][3] & 0xffff0000u));
    }
  }
  if constexpr (DTP) {
    const int row = tid / wdt_ppr, pc = tid - row * wdt_ppr;
    if (tid < 64 * wdt_ppr) *reinterpret_cast<wv4*>(&sWd[row * kChDtpWPitch + pc * 8]) = wdt_piece;
  }
  if (PASS == 3 && tid == 0) s_tag = ep + 1u == 0u ? 1u : ep + 1u;
  // A transposed into LDS: sA[n][c] (zero for n >= N and for channels past dim)
#pragma unroll
  for (int k = 0; k < kChSPW; ++k) {
    const int e = tid + k * 64 * kChW;
    if (e < 64 * N) sA[e % N][e / N] = aval[k];
    if (e >= 64 * N && e < 64 * kMaxN) sA[e >> 6][e & 63] = 0.0f;
  }
  if constexpr (PASS == 2) {
    // the first kChW block aggregates go to LDS with A: [block][state][channel]
#pragma unroll
    for (int j = 0; j < kChW; ++j) stage_agg(j, agH[j]);
    sS[tid >> 6][lane] = agS[0];
  }
  __syncthreads();
  // DTP: this wave's dt for steps t_beg .. t_end - 1 (blocks of 16) -> sDT[wave][ch][step]
  bf16_t* myDT = &sDT[DTP ? wave * 64 * kChDtpPitch : 0];
  auto dt_lds = [&](int t) -> uint32_t {  // the raw bf16 of step t (clamped into the block)
    const int i = min(max(t - t_beg, 0), kChDtpPitch - 1);
    return static_cast<uint32_t>(*reinterpret_cast<const unsigned short*>(&myDT[lane * kChDtpPitch + i]));
  };
  if constexpr (DTP) {
    typedef __attribute__((ext_vector_type(8))) __bf16 dbf16x8;
    typedef __attribute__((ext_vector_type(4))) float df32x4;
    typedef __attribute__((ext_vector_type(2))) unsigned du2;
    const int rp = q.wdt_ld;
    const int R = q.dt_rank;
    const auto dtr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(q.dtl + static_cast<long long>(b) * q.dtl_sb), 0,
        static_cast<int>(static_cast<long long>(p.out_len) * q.dtl_sl * 2), 0x00020000);
    constexpr int kOut = 0x7ffffff0;
    for (int t0 = t_beg; t0 < t_end; t0 += 16) {
      dbf16x8 af[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        // A = x_dbl row t0 + lane % 16, k = 32 ks + 8 (lane / 16) .. + 7; k >= R reads 0
        const int k0 = 32 * ks + 8 * (lane >> 4);
        const int off = ((t0 + (lane & 15)) * static_cast<int>(q.dtl_sl) + k0) * 2;
        const du2 lo = __builtin_bit_cast(du2, __builtin_amdgcn_raw_buffer_load_b64(
                                                   dtr, k0 + 4 <= R && 32 * ks < rp ? off : kOut, 0, 0));
        const du2 hi = __builtin_bit_cast(du2, __builtin_amdgcn_raw_buffer_load_b64(
                                                   dtr, k0 + 8 <= R && 32 * ks < rp ? off + 8 : kOut, 0, 0));
        af[ks] = __builtin_bit_cast(dbf16x8, (__attribute__((ext_vector_type(4))) unsigned){lo.x, lo.y, hi.x, hi.y});
      }
#pragma unroll
      for (int tile = 0; tile < 4; ++tile) {
        df32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          if (32 * ks < rp) {
            const dbf16x8 bw = *reinterpret_cast<const dbf16x8*>(
                &sWd[(16 * tile + (lane & 15)) * kChDtpWPitch + 32 * ks + 8 * (lane >> 4)]);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], bw, acc, 0, 0, 0);
          }
        }
        // D[step 4 (lane/16) + i][channel 16 tile + lane % 16] -> [channel][step]
        const uint32_t p01 = cvt_pk_bf16(acc[0], acc[1]), p23 = cvt_pk_bf16(acc[2], acc[3]);
        *reinterpret_cast<uint2*>(&myDT[(16 * tile + (lane & 15)) * kChDtpPitch + (t0 - t_beg) +
                                        4 * (lane >> 4)]) = uint2{p01, p23};
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the block is written
#pragma unroll
    for (int j = 0; j < kPF; ++j) rd[j] = dt_lds(min(t_beg + j, tlast));
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
  f2 A2[kMaxN / 2], h[kMaxN / 2];
#pragma unroll
  for (int q = 0; q < kMaxN / 2; ++q) {
    A2[q] = f2{sA[2 * q][lane], sA[2 * q + 1][lane]};
    h[q] = f2{0.0f, 0.0f};
  }
  float Ans[kChSPW];
#pragma unroll
  for (int i = 0; i < kChSPW; ++i) Ans[i] = sA[n0 + i][lane];
  if constexpr (PASS == 2) {
#pragma unroll
    for (int i = 0; i < kChSPW; ++i) Hs[i] *= kLog2e;  // log2 units
    // walk the preceding blocks' aggregates from h0 to this block's entry, kChW at a time
    // through LDS (the second group from registers loaded with the start-up round)
    for (int r0 = 0; r0 < blk; r0 += kChW) {
      if (r0 > 0) {
        __syncthreads();  // every wave is done reading the previous group
        if (r0 < kCW) {
#pragma unroll
          for (int j = 0; j < kChW; ++j) stage_agg(j, agH[(kChW + j) % kCW]);
          sS[tid >> 6][lane] = agS[(kCW / kChW) - 1];
        } else {  // long sequences: later groups are loaded here
          const int ci = tid / kTPC;
#pragma unroll
          for (int j = 0; j < kChW; ++j) {
            agv_t v{};
            if (r0 + j < blk && ci < nch)
              v = *reinterpret_cast<const agv_t*>(
                  &w.aggH[(rowA + (r0 + j) * D + d0) * kMaxN + kChSPW * tid]);
            stage_agg(j, v);
          }
          const int j = r0 + (tid >> 6);
          sS[tid >> 6][lane] = j < blk && lane < nch ? w.aggS[rowA + j * D + d0 + lane] : 0.0f;
        }
        __syncthreads();
      }
      const int nj = min(kChW, blk - r0);
      for (int j = 0; j < nj; ++j) {
        const float Sj = sS[j][lane];
#pragma unroll
        for (int i = 0; i < kChSPW; ++i)
          Hs[i] = fmaf(__builtin_amdgcn_exp2f(Ans[i] * Sj), Hs[i], sH[j][n0 + i][lane]);
      }
    }
    __syncthreads();  // sH[0] is rewritten with the block entry
#pragma unroll
    for (int i = 0; i < kChSPW; ++i) sH[0][n0 + i][lane] = Hs[i];
    __syncthreads();
    // this segment's entry: exp2(A P_j) * H_blk + E_j
#pragma unroll
    for (int q = 0; q < kMaxN / 2; ++q) {
      const f2 x = A2[q] * f2{Pj, Pj};
      h[q] = f2{fmaf(__builtin_amdgcn_exp2f(x.x), sH[0][2 * q][lane], Ej[q].x),
                fmaf(__builtin_amdgcn_exp2f(x.y), sH[0][2 * q + 1][lane], Ej[q].y)};
    }
  }
  // The step loop: EMIT runs the PASS 2 form (z gate, y stores), otherwise the PASS 1 form
  // (end state and delta sum only).  The prefetch registers hold steps t_beg .. + kPF.
  auto delta_of = [&](uint32_t raw) {  // delta' = softplus(dt + bias) * log2e
    const float x = fmaf(raw_f32<T>(raw), kLog2e, bias);  // (dt + bias) * log2e
    if constexpr (SP)
      return x > 20.0f * kLog2e ? x : __builtin_amdgcn_logf(1.0f + __builtin_amdgcn_exp2f(x));
    return x;
  };
  auto run_steps = [&](auto emit_tag) {
    constexpr bool EMIT = decltype(emit_tag)::value;
    // the next step's delta and output-gate factor are computed a step early (as in
    // scan_seq_kernel)
    constexpr bool GA = kSeqGateAhead && EMIT && HZ;
    auto gate_of = [&](uint32_t raw) {
      const float zz = raw_f32<T>(raw);
      return zz * __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_exp2f(-zz * kLog2e), kLog2e, kLog2e));
    };
    float dl_nx = delta_of(rd[0]);
    float g_nx = GA ? gate_of(rz[0]) : 0.0f;
    // LBC: the next step's B (and, emitting, C) row from LDS, one step ahead
    constexpr int NBC = EMIT ? 2 * kMaxN : kMaxN;
    float bcn[LBC ? NBC : 1];
    auto lbc_read = [&](int t) {
      if constexpr (LBC) {
        const float* src = &sBC[t - blk_t0][0];
#pragma unroll
        for (int i = 0; i < NBC / 4; ++i) {
          const float4 v = *reinterpret_cast<const float4*>(src + 4 * i);
          bcn[4 * i] = v.x; bcn[4 * i + 1] = v.y; bcn[4 * i + 2] = v.z; bcn[4 * i + 3] = v.w;
        }
      }
    };
    if constexpr (LBC) lbc_read(min(t_beg, t_end - 1));
    for (int tg = t_beg; tg < t_end; tg += kPF) {
      // The two waves of a SIMD (w, w + 4) share its issue slots, and the hardware favours
      // the older one: left alone, one wave finished its loop ~1.7x before the other, which
      // then ran its rest alone at a wave's latency-bound rate while the block waited at its
      // next barrier (r05 stamps: 7.2 vs 12.4 us in PASS 1).  Each wave raises its priority
      // for one half of the segment and its SIMD partner for the other, so the two finish
      // together: B = 1 chunk -2.5 to -3 %, B = 2 -2.4 % (r06r).  Issue order
      // only: every value is unchanged.
      if ((2 * (tg - t_beg) + kPF >= t_end - t_beg) != ((wave >> 2) & 1)) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
#pragma unroll
      for (int j = 0; j < kPF; ++j) {
        const int t = tg + j;
        const bool live = t < t_end;
        const float uu = raw_f32<T>(ru[j]);
        const float zz = raw_f32<T>(rz[j]);
        const int tn = min(t + kPF, tlast);
        ru[j] = bload<T>(ur, voff, tn * us);
        if constexpr (!DTP) rd[j] = bload<T>(dr_, voff, tn * ds);
        if (HZ && EMIT) rz[j] = bload<T>(zr, voff, tn * zs);
        float bcc[LBC ? NBC : 1];
        if constexpr (LBC) {  // this step's row (read a step ago); fetch the next one
#pragma unroll
          for (int i = 0; i < NBC; ++i) bcc[i] = bcn[i];
          lbc_read(min(t + 1, t_end - 1));
        } else if constexpr (kChBcPairs && !EMIT) {
          if ((j & 1) == 0) {  // a pair starts: its two rows have landed; fetch the next pair's
            __builtin_amdgcn_s_waitcnt(0xC07F);
            bc_load(min(t + 2, tlast), bcw[(j + 2) & 3]);
            bc_load(min(t + 3, tlast), bcw[(j + 3) & 3]);
          }
        } else {
          __builtin_amdgcn_s_waitcnt(0xC07F);  // this step's B/C rows have landed
          bc_load(min(t + 1, tlast), bcw[(j + 1) & 1]);
        }
        // DTP: the LDS read goes after that wait, so the next step's wait is its first
        if constexpr (DTP) rd[j] = dt_lds(tn);
        __builtin_amdgcn_sched_barrier(0);  // (without: 10-40 % slower, scripts/diag)
        float dl = dl_nx;
        dl_nx = delta_of(rd[(j + 1) & (kPF - 1)]);
        dl = live ? dl : 0.0f;
        float gf = 0.0f;
        if constexpr (GA) {
          gf = g_nx;
          g_nx = gate_of(rz[(j + 1) & (kPF - 1)]);
        }
        const float du = dl * uu;
        const uint32_t (&cw)[2 * NWD] = bcw[j & ((kChBcPairs && !EMIT) ? 3 : 1)];
        const f2 dl2 = {dl, dl}, du2 = {du, du};
        f2 ya = {Dv * uu, 0.0f}, yb = {0.0f, 0.0f};
#pragma unroll
        for (int q = 0; q < kMaxN / 2; ++q) {
          f2 Bp, Cp;
          if constexpr (LBC) {
            Bp = f2{bcc[2 * q], bcc[2 * q + 1]};
            Cp = EMIT ? f2{bcc[(NBC / 2) + 2 * q], bcc[(NBC / 2) + 2 * q + 1]} : Bp;
          } else if constexpr (sizeof(T) == 2) {
            Bp = f2{__uint_as_float(cw[q] << 16), __uint_as_float(cw[q] & 0xffff0000u)};
            Cp = f2{__uint_as_float(cw[NWD + q] << 16), __uint_as_float(cw[NWD + q] & 0xffff0000u)};
          } else {
            Bp = f2{__uint_as_float(cw[2 * q]), __uint_as_float(cw[2 * q + 1])};
            Cp = f2{__uint_as_float(cw[NWD + 2 * q]), __uint_as_float(cw[NWD + 2 * q + 1])};
          }
          const f2 x = dl2 * A2[q];
          const f2 a = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
          h[q] = __builtin_elementwise_fma(a, h[q], du2 * Bp);
          if constexpr (EMIT) {
            if (q & 1) yb = __builtin_elementwise_fma(h[q], Cp, yb);
            else ya = __builtin_elementwise_fma(h[q], Cp, ya);
          }
        }
        if constexpr (!EMIT) {
          sdel += dl;
        } else {
          const f2 ys = ya + yb;
          float y = ys.x + ys.y;
          // output gate with y's ln2 factor: z / ((1 + e) * log2e)
          if constexpr (GA) y *= gf;
          else
            y = HZ ? y * (zz * __builtin_amdgcn_rcpf(
                                   fmaf(__builtin_amdgcn_exp2f(-zz * kLog2e), kLog2e, kLog2e)))
                   : y * kLn2f;
          bstore<T, kSmallStoreWT>(from_f32<T>(y), orr, live ? voff_st : kSeqDead, ps.orow(t) * os);
        }
      }
    }
  };
  // the final segment's h_last and the zeroed padding steps (PASS 2 / the one-launch form)
  auto finish = [&]() {
    if (t_beg <= tlast && tlast < t_end && active && L > 0) {  // the segment that ends the sequence
      if (ps.hl) {
#pragma unroll
        for (int n = 0; n < kMaxN; ++n)
          if (n < N)
            store_dyn(ps.hl, ps.hb * p.hl_sb + d * p.hl_sd + n, p.hl_dtype,
                      ((n & 1) ? h[n >> 1].y : h[n >> 1].x) * kLn2f);
      }
      for (int t = L; t < p.out_len; ++t) bstore<T, kSmallStoreWT>(from_f32<T>(0.0f), orr, voff, t * os);
    }
  };

  if constexpr (PASS == 2) {
    run_steps(BoolTag<true>{});
    finish();
    return;
  }
  run_steps(BoolTag<false>{});
#pragma unroll
  for (int q = 0; q < kMaxN / 2; ++q) {
    sH[wave][2 * q][lane] = h[q].x;
    sH[wave][2 * q + 1][lane] = h[q].y;
  }
  sS[wave][lane] = sdel;
  // LDS-only barrier: the step loop's last refill loads (for steps past the segment) are
  // still in flight and need not land before the composition
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  // compose the block's segments for states n0, n0 + 1: entry offsets E_j, delta prefixes
  // P_j and the block aggregate (PASS 1: all to the workspace; one-launch form: E_j back into
  // sH[j] in place, the aggregate to the workspace for the blocks after this one)
  float Es[kChSPW], P = 0.0f, Pw = 0.0f;
#pragma unroll
  for (int i = 0; i < kChSPW; ++i) Es[i] = 0.0f;
#pragma unroll
  for (int j = 0; j < kChW; ++j) {
    const float Sj = sS[j][lane];
    float Hj[kChSPW];
#pragma unroll
    for (int i = 0; i < kChSPW; ++i) Hj[i] = sH[j][n0 + i][lane];
    if constexpr (PASS == 1) {
      if (active) {
#pragma unroll
        for (int i = 0; i < kChSPW; ++i) w.segE[(rowE + j * D + d) * kMaxN + n0 + i] = Es[i];
        if (wave == 0) w.segP[rowE + j * D + d] = P;
      }
    } else {
#pragma unroll
      for (int i = 0; i < kChSPW; ++i) sH[j][n0 + i][lane] = Es[i];
      if (j == wave) Pw = P;
    }
#pragma unroll
    for (int i = 0; i < kChSPW; ++i) Es[i] = fmaf(__builtin_amdgcn_exp2f(Ans[i] * Sj), Es[i], Hj[i]);
    P += Sj;
  }
  if constexpr (PASS != 3) {
    if (active) {
#pragma unroll
      for (int i = 0; i < kChSPW; ++i) w.aggH[(rowA + blk * D + d) * kMaxN + n0 + i] = Es[i];
      if (wave == 0) w.aggS[rowA + blk * D + d] = P;
    }
  }
  if constexpr (PASS == 3) {
    // ---- publish this block's aggregate: the data is the flag ----
    // Every value goes out as one aligned 8-byte {tag, value} granule by an agent-scope
    // atomic store (an sc1 store to the coherence point); a reader polls the granules it
    // needs until every tag is this launch's.  No drain, no separate flag, no second load
    // round (cdna_hip_programming.md Guideline 16, R2): the round-2 form (aggregate stores,
    // vmcnt(0), barrier, flag store, flag polls, then aggregate loads) spent ~11 us of the
    // B = 1 scan between PASS 1 and PASS 2 (scripts/diag/stamp_scan.py).
    // Granule layout [row][group][block][state 0..15 | delta sum][channel lane].
    const unsigned tag = s_tag;
    const unsigned long long tg = static_cast<unsigned long long>(tag) << 32;
    unsigned long long* gb =
        w.gran + ((static_cast<long long>(b) * gridDim.x + gx) * w.nblk) * ((kMaxN + 1) * 64);
    unsigned long long* gmine = gb + static_cast<long long>(blk) * ((kMaxN + 1) * 64);
#pragma unroll
    for (int i = 0; i < kChSPW; ++i)
      __hip_atomic_store(gmine + (n0 + i) * 64 + lane, tg | __float_as_uint(Es[i]),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wave == 0)
      __hip_atomic_store(gmine + kMaxN * 64 + lane, tg | __float_as_uint(P), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    // every wave's E_j is in sH (an LDS-only barrier: the granule stores need no drain)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    // PASS 2 operands of the first kPF steps, in flight during the wait
    if (t_beg < t_end) {
      if constexpr (!LBC) bc_load(t_beg, bcw[0]);
#pragma unroll
      for (int j = 0; j < kPF; ++j) {
        const int t = min(t_beg + j, tlast);
        ru[j] = bload<T>(ur, voff, t * us);
        rd[j] = DTP ? dt_lds(t) : bload<T>(dr_, voff, t * ds);
        rz[j] = HZ ? bload<T>(zr, voff, t * zs) : 0u;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // ---- walk the preceding blocks' aggregates from h0 to this block's entry ----
    // Wave w needs only its own states n0 (, n0 + 1) and the delta sums of each preceding
    // block: kChSPW + 1 granules per block and lane, polled kChPoll blocks at a time.  Blocks are
    // dispatched in order and the host launches this form only when the whole grid is
    // co-resident, so every block waited on is running or done; the poll is bounded anyway
    // so a broken assumption can never hang the GPU: a wave whose poll runs out sets the
    // sticky error word and poisons its states with NaN, so every output and h_last of the
    // block is NaN — never a plausible wrong value.
#pragma unroll
    for (int i = 0; i < kChSPW; ++i) Hs[i] *= kLog2e;  // log2 units
    for (int r0 = 0; r0 < blk; r0 += kChPoll) {
      const int nj = min(kChPoll, blk - r0);
      unsigned long long gh[kChSPW][kChPoll], gs[kChPoll];
      unsigned spins = 0;
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < kChPoll; ++j) {
          const unsigned long long* gj =
              gb + static_cast<long long>(r0 + (j < nj ? j : 0)) * ((kMaxN + 1) * 64);
#pragma unroll
          for (int i = 0; i < kChSPW; ++i)
            gh[i][j] = __hip_atomic_load(gj + (n0 + i) * 64 + lane, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
          gs[j] = __hip_atomic_load(gj + kMaxN * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int j = 0; j < kChPoll; ++j) {
          ok = ok && static_cast<unsigned>(gs[j] >> 32) == tag;
#pragma unroll
          for (int i = 0; i < kChSPW; ++i) ok = ok && static_cast<unsigned>(gh[i][j] >> 32) == tag;
        }
        if (__all(ok)) break;
        if (++spins >= (1u << 20)) {
          if (lane == 0) __hip_atomic_store(w.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int i = 0; i < kChSPW; ++i) Hs[i] = __builtin_nanf("");
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
#pragma unroll
      for (int j = 0; j < kChPoll; ++j) {
        if (j < nj) {  // (static register indices: a runtime bound would spill the arrays)
          const float Sj = __uint_as_float(static_cast<unsigned>(gs[j]));
#pragma unroll
          for (int i = 0; i < kChSPW; ++i)
            Hs[i] = fmaf(__builtin_amdgcn_exp2f(Ans[i] * Sj), Hs[i],
                         __uint_as_float(static_cast<unsigned>(gh[i][j])));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kChSPW; ++i) sHb[n0 + i][lane] = Hs[i];
    __syncthreads();
    // this segment's entry: exp2(A P_j) * H_blk + E_j (E_j composed into sH[j] above)
#pragma unroll
    for (int q = 0; q < kMaxN / 2; ++q) {
      const f2 x = A2[q] * f2{Pw, Pw};
      h[q] = f2{fmaf(__builtin_amdgcn_exp2f(x.x), sHb[2 * q][lane], sH[wave][2 * q][lane]),
                fmaf(__builtin_amdgcn_exp2f(x.y), sHb[2 * q + 1][lane], sH[wave][2 * q + 1][lane])};
    }
    run_steps(BoolTag<true>{});
    finish();
    if (tid == 0) {  // count this block out (its epoch read completed at the start-up wait)
      const unsigned nwg = gridDim.x * gridDim.y * gridDim.z;
      if (__hip_atomic_fetch_add(w.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nwg - 1) {
        __hip_atomic_store(w.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(w.epoch, s_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// Entry state of every segment: h_in[0] = h0, h_in[s+1] = exp2(A*log2e*sum_delta[s]) *
// h_in[s] + h_end[s].  One thread per (b, d, n), sequential over the S segments; the
// summaries stream through a 16-deep register window so their loads overlap the chain.
__global__ __launch_bounds__(256) void scan_seq_carry_kernel(const ScanParams p, const SeqWork w) {
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  const long long total = static_cast<long long>(p.batch) * p.dim * kMaxN;
  if (i >= total) return;
  const int n = static_cast<int>(i % kMaxN);
  const int d = static_cast<int>((i / kMaxN) % p.dim);
  const int b = static_cast<int>(i / (static_cast<long long>(kMaxN) * p.dim));
  const int N = p.dstate;
  const float A2 = n < N ? p.A[d * N + n] * kLog2e : 0.0f;
  const long long stride = static_cast<long long>(p.dim);
  const long long row0 = static_cast<long long>(b) * w.S * stride + d;
  const float* __restrict__ sdel = w.sdel;
  const float* __restrict__ hend = w.hend;
  float* __restrict__ hin = w.hin;
  constexpr int kWin = 16;
  float h = (n < N && p.h0) ? load_dyn(p.h0, b * p.h0_sb + d * p.h0_sd + n, p.h0_dtype) : 0.0f;
  for (int s0 = 0; s0 < w.S; s0 += kWin) {
    float sd[kWin], he[kWin];
#pragma unroll
    for (int j = 0; j < kWin; ++j) {
      const int s = s0 + j;
      const long long row = row0 + (s + 1 < w.S ? s : 0) * stride;
      sd[j] = sdel[row];
      he[j] = hend[row * kMaxN + n];
    }
#pragma unroll
    for (int j = 0; j < kWin; ++j) {
      const int s = s0 + j;
      if (s < w.S) {
        hin[(row0 + s * stride) * kMaxN + n] = h;
        if (s + 1 < w.S) h = fmaf(__builtin_amdgcn_exp2f(A2 * sd[j]), h, he[j]);
      }
    }
  }
}

// B/C as scalar loads: 16 states, unit state stride, every row 4-byte aligned.
static bool seq_sgpr_bc(const ScanParams& p, int es) {
  auto ok = [&](const void* ptr, long long sb, long long sn, long long sl) {
    return sn == 1 && (reinterpret_cast<uintptr_t>(ptr) & 3) == 0 && (sb * es) % 4 == 0 &&
           (sl * es) % 4 == 0;
  };
  const long long span = static_cast<long long>(p.seqlen > 0 ? p.seqlen : 1) * es;
  return p.dstate == kMaxN && ok(p.B, p.b_sb, p.b_sn, p.b_sl) && ok(p.C, p.c_sb, p.c_sn, p.c_sl) &&
         span * p.b_sl < (1ll << 31) && span * p.c_sl < (1ll << 31);
}

template <typename T, int MODE, bool SP, bool HZ>
static void launch_seq_mode(const ScanParams& p, const SeqWork& w, int segs, hipStream_t s) {
  const int groups = (p.dim + 63) / 64;
  dim3 grid((groups + kSeqNW - 1) / kSeqNW, segs, p.batch);
  const bool bc1 = p.c_sl == p.b_sl && p.c_sb == p.b_sb &&
                   static_cast<const T*>(p.C) == static_cast<const T*>(p.B) + kMaxN;
  if constexpr (MODE == 0) {
    if (p.split < p.batch) {  // paired: scalar B/C single pass only (seq_pair_supported)
      if (bc1)
        hipLaunchKernelGGL((scan_seq_kernel<T, kSeqNW, 0, SP, HZ, true, true, true, true>), grid,
                           dim3(64 * kSeqNW), 0, s, p, w);
      else
        hipLaunchKernelGGL((scan_seq_kernel<T, kSeqNW, 0, SP, HZ, true, true, false, true>),
                           grid, dim3(64 * kSeqNW), 0, s, p, w);
      return;
    }
  }
  if (seq_sgpr_bc(p, sizeof(T))) {
    // BC1: C directly follows B in one row (the mixer's x_dbl): one scalar load for both
    if (bc1)
      hipLaunchKernelGGL((scan_seq_kernel<T, kSeqNW, MODE, SP, HZ, true, true, true>), grid,
                         dim3(64 * kSeqNW), 0, s, p, w);
    else
      hipLaunchKernelGGL((scan_seq_kernel<T, kSeqNW, MODE, SP, HZ, true, true>), grid,
                         dim3(64 * kSeqNW), 0, s, p, w);
  } else {
    hipLaunchKernelGGL((scan_seq_kernel<T, kSeqNW, MODE, SP, HZ, false, false>), grid,
                       dim3(64 * kSeqNW), 0, s, p, w);
  }
}

template <typename T, bool SP, bool HZ>
static void launch_seq_t(const ScanParams& p, const SeqWork& w, hipStream_t s) {
  if (w.S <= 1) {
    launch_seq_mode<T, 0, SP, HZ>(p, w, 1, s);
    return;
  }
  launch_seq_mode<T, 1, SP, HZ>(p, w, w.S - 1, s);  // the last segment's summary is unused
  const long long total = static_cast<long long>(p.batch) * p.dim * kMaxN;
  hipLaunchKernelGGL(scan_seq_carry_kernel, dim3(static_cast<unsigned>((total + 255) / 256)),
                     dim3(256), 0, s, p, w);
  launch_seq_mode<T, 2, SP, HZ>(p, w, w.S, s);
}

template <typename T>
static void launch_seq(const ScanParams& p, const SeqWork& w, hipStream_t s) {
  const bool hz = p.z != nullptr;
  if (p.softplus) {
    if (hz) launch_seq_t<T, true, true>(p, w, s);
    else launch_seq_t<T, true, false>(p, w, s);
  } else {
    if (hz) launch_seq_t<T, false, true>(p, w, s);
    else launch_seq_t<T, false, false>(p, w, s);
  }
}

// (vmhost::device_cus: 0 when it cannot be queried — no device: the size queries then
// assume kCalibCUs)
using vmhost::device_cus;

static constexpr int kCalibCUs = 256;  // the part the cost model below was swept on
static int cus_or_calib(int cus) { return cus > 0 ? cus : kCalibCUs; }

// Segment count.  A chip-filling batch (>= 1,280 waves of 64-channel groups) runs
// single-pass.  Below that the chunked form's time is modelled from a sweep of forced
// segment counts at M-16f geometry (scripts/diag/scan_segments_sweep.py, B = 1 .. 64,
// L = 3,137 and 12,545; profiles/r02_scan_segments_sweep.jsonl):
//   time ~ 16.6 us + 0.69 us x k x T + 0.43 us x nblk
// with T steps per segment, nblk = blocks of kChW segments per sequence and
// k = ceil(workgroups / 256): a CU holding k of the 512-thread workgroups runs their waves'
// steps k-fold interleaved (the passes are issue-bound), and every block adds one aggregate
// to the entry walk.  The model is within ~6 % of the sweep; the round-1 rule (a fixed
// ~1,792-wave target) picked 2-3x slower counts at B >= 4 (T = 126 .. 1,569 steps).
// Depends on (batch, dim, seqlen) and the device's CU count only (the sweep ran on a
// 256-CU MI355X; `cus` rescales k and the chip-filling threshold for other parts).
static int choose_segments(int batch, int dim, int seqlen, int cus) {
  if (seqlen < 64) return 1;
  const long long groups = (dim + 63) / 64;
  if (batch * groups >= 5 * cus) return 1;
  const int max_s = (seqlen + 7) / 8;  // segments of at least 8 steps
  int best = 1;
  double best_cost = 1e30;
  for (int S = 2; S <= max_s && S <= 2048; S += (S < 64 ? 1 : 8)) {
    const int T = (seqlen + S - 1) / S;
    const int segs = (seqlen + T - 1) / T;
    const long long nblk = (segs + kChW - 1) / kChW;
    const long long k = (batch * groups * nblk + cus - 1) / cus;
    const double cost = 0.69 * static_cast<double>(k * T) + 0.43 * static_cast<double>(nblk);
    if (cost < best_cost) {
      best_cost = cost;
      best = S;
    }
  }
  return best;
}

// segments > 0 (an explicit ABI argument: tests and sweeps) forces the segment count;
// 0 lets the cost model choose.
// `cus` = the launch device's CU count (0: the current device's, or kCalibCUs).
static int segments_for(int batch, int dim, int seqlen, int segments, int cus = 0) {
  if (cus <= 0) cus = cus_or_calib(device_cus(nullptr));
  int S = segments > 0 ? segments : choose_segments(batch, dim, seqlen, cus);
  if (S > seqlen) S = seqlen > 0 ? seqlen : 1;
  return S < 1 ? 1 : S;
}

// Chunked-form geometry for S segments: T steps per segment, nblk blocks of kChW segments.
static void chunk_geometry(int seqlen, int S, int* T, int* nblk) {
  *T = (seqlen + S - 1) / S;
  const int segs = (seqlen + *T - 1) / *T;
  *nblk = (segs + kChW - 1) / kChW;
}

static size_t chunk_bytes(int batch, int dim, int seqlen, int S) {
  int T, nblk;
  chunk_geometry(seqlen, S, &T, &nblk);
  const size_t per_blk = static_cast<size_t>(kChW + 1) * dim * (kMaxN + 1);
  return static_cast<size_t>(batch) * nblk * per_blk * sizeof(float);
}

static size_t legacy_bytes(int batch, int dim, int S) {
  if (S > kMaxSeg) S = kMaxSeg;
  return static_cast<size_t>(batch) * S * dim * (2 * kMaxN + 1) * sizeof(float);
}

size_t seq_workspace_bytes(int batch, int dim, int seqlen, int segments, int* chosen,
                           int cus) {
  const int S = segments_for(batch, dim, seqlen, segments, cus);
  if (chosen) *chosen = S;
  if (S <= 1) return 0;
  const size_t a = chunk_bytes(batch, dim, seqlen, S), b = legacy_bytes(batch, dim, S);
  return a > b ? a : b;
}

bool seq_supported(const ScanParams& p, int dtype) {
  // buffer offsets are 31-bit byte offsets from each batch row's base
  const long long es = dtype == VM_DTYPE_BF16 ? 2 : 4;
  const long long span = static_cast<long long>(p.out_len > p.seqlen ? p.out_len : p.seqlen) + 1;
  auto fits = [&](long long sl) { return sl >= 0 && (span * sl + p.dim) * es < (1ll << 30); };
  return p.u_sd == 1 && p.dl_sd == 1 && p.o_sd == 1 && (p.z == nullptr || p.z_sd == 1) &&
         p.dstate <= kMaxN && fits(p.u_sl) && fits(p.dl_sl) && fits(p.o_sl) &&
         (p.z == nullptr || fits(p.z_sl));
}

template <typename T, bool SP, bool HZ, bool BC1, bool PAIR, bool DTP = false>
static void launch_chunk_p(const ScanParams& p, const ChunkWork& w, hipStream_t s,
                           const DtpArgs& q = DtpArgs{}) {
  dim3 grid((p.dim + 63) / 64, w.nblk, p.batch);
  if (w.gran) {  // one launch: blocks hand their aggregates on through the sync buffer
    if constexpr (DTP && BC1 && sizeof(T) == 2) {
      if (kChW * w.T <= kChLbcRows) {  // the block's B|C rows fit the LDS staging block
        hipLaunchKernelGGL((scan_chunk_kernel<T, 3, SP, HZ, BC1, PAIR, DTP, true>), grid,
                           dim3(64 * kChW), 0, s, p, w, q);
        return;
      }
    }
    hipLaunchKernelGGL((scan_chunk_kernel<T, 3, SP, HZ, BC1, PAIR, DTP>), grid, dim3(64 * kChW),
                       0, s, p, w, q);
    return;
  }
  hipLaunchKernelGGL((scan_chunk_kernel<T, 1, SP, HZ, BC1, PAIR, DTP>), grid, dim3(64 * kChW), 0,
                     s, p, w, q);
  hipLaunchKernelGGL((scan_chunk_kernel<T, 2, SP, HZ, BC1, PAIR, DTP>), grid, dim3(64 * kChW), 0,
                     s, p, w, q);
}

template <typename T, bool SP, bool HZ, bool BC1>
static void launch_chunk_t(const ScanParams& p, const ChunkWork& w, hipStream_t s) {
  if (p.split < p.batch) launch_chunk_p<T, SP, HZ, BC1, true>(p, w, s);
  else launch_chunk_p<T, SP, HZ, BC1, false>(p, w, s);
}

template <typename T>
static void launch_chunk(const ScanParams& p, const ChunkWork& w, hipStream_t s) {
  const bool hz = p.z != nullptr;
  const bool bc1 = p.c_sl == p.b_sl && p.c_sb == p.b_sb &&
                   static_cast<const T*>(p.C) == static_cast<const T*>(p.B) + kMaxN;
#define VM_CH(SPV, HZV)                                              \
  if (bc1) launch_chunk_t<T, SPV, HZV, true>(p, w, s);               \
  else launch_chunk_t<T, SPV, HZV, false>(p, w, s);
  if (p.softplus) {
    if (hz) { VM_CH(true, true) } else { VM_CH(true, false) }
  } else {
    if (hz) { VM_CH(false, true) } else { VM_CH(false, false) }
  }
#undef VM_CH
}

// One-launch chunked form: the sticky error word (word 0), the epoch (word 1: the tag of the
// last launch that used the buffer) and the launch's start count (word 2), word 3 pad, then
// one 8-byte {tag, value} granule per (row, channel group, block, state | delta sum,
// channel).  Used when the caller passes a zeroed sync buffer this large and the whole grid
// fits one workgroup per CU (so every block it waits on is resident).
size_t seq_sync_bytes(int batch, int dim, int seqlen, int segments, int cus) {
  const int S = segments_for(batch, dim, seqlen, segments, cus);
  if (S <= 1) return 0;
  int T, nblk;
  chunk_geometry(seqlen, S, &T, &nblk);
  const size_t groups = (dim + 63) / 64;
  return kSyncHeaderWords * sizeof(unsigned) +
         static_cast<size_t>(batch) * groups * nblk * (kMaxN + 1) * 64 * sizeof(unsigned long long);
}

bool seq_pair_supported(const ScanParams& p, int dtype, int segments, size_t workspace_bytes) {
  int S = 1;
  const size_t need = seq_workspace_bytes(p.batch, p.dim, p.seqlen, segments, &S);
  return seq_sgpr_bc(p, dtype == VM_DTYPE_BF16 ? 2 : 4) && (S <= 1 || workspace_bytes >= need);
}

void seq_launch(const ScanParams& p, int dtype, int segments, void* workspace,
                size_t workspace_bytes, void* sync, size_t sync_bytes, hipStream_t s) {
  // the stream's device decides the segment count and whether the grid is co-resident
  const int dev_cus = device_cus(s);
  const int cus = cus_or_calib(dev_cus);
  int S = 1;
  const size_t need = seq_workspace_bytes(p.batch, p.dim, p.seqlen, segments, &S, cus);
  const int es = dtype == VM_DTYPE_BF16 ? 2 : 4;
  if (S > 1 && workspace && workspace_bytes >= need && seq_sgpr_bc(p, es)) {
    ChunkWork w{};
    chunk_geometry(p.seqlen, S, &w.T, &w.nblk);
    const long long grid = static_cast<long long>((p.dim + 63) / 64) * w.nblk * p.batch;
    if (sync && sync_bytes >= seq_sync_bytes(p.batch, p.dim, p.seqlen, segments, cus) &&
        grid <= dev_cus) {
      w.err = static_cast<unsigned*>(sync);
      w.epoch = w.err + 1;
      w.done = w.err + 2;
      w.gran = reinterpret_cast<unsigned long long*>(w.err + kSyncHeaderWords);
    }
    const size_t nb = static_cast<size_t>(p.batch) * w.nblk;
    w.segE = static_cast<float*>(workspace);
    w.segP = w.segE + nb * kChW * p.dim * kMaxN;
    w.aggH = w.segP + nb * kChW * p.dim;
    w.aggS = w.aggH + nb * p.dim * kMaxN;
    if (dtype == VM_DTYPE_BF16) launch_chunk<bf16_t>(p, w, s);
    else launch_chunk<float>(p, w, s);
    return;
  }
  SeqWork w{};
  if (S > kMaxSeg) S = kMaxSeg;
  if (S > 1 && workspace && workspace_bytes >= need) {
    const size_t states = static_cast<size_t>(p.batch) * S * p.dim * kMaxN;
    w.hend = static_cast<float*>(workspace);
    w.hin = w.hend + states;
    w.sdel = w.hin + states;
    w.seg_len = (p.seqlen + S - 1) / S;
    w.S = (p.seqlen + w.seg_len - 1) / w.seg_len;  // every segment non-empty
  } else {
    w.S = 1;
    w.seg_len = p.seqlen;
  }
  if (dtype == VM_DTYPE_BF16) launch_seq<bf16_t>(p, w, s);
  else launch_seq<float>(p, w, s);
}

bool seq_dtp_supported(const ScanParams& p, const DtpArgs& q, int dtype, int dt_rank) {
  const bool bc1 = p.c_sl == p.b_sl && p.c_sb == p.b_sb &&
                   static_cast<const bf16_t*>(p.C) == static_cast<const bf16_t*>(p.B) + kMaxN;
  const int nks = (dt_rank + 15) / 16;
  const long long dl_span = static_cast<long long>(p.out_len) * q.dtl_sl * 2;
  return dtype == VM_DTYPE_BF16 && seq_supported(p, dtype) && seq_sgpr_bc(p, 2) && bc1 &&
         p.dstate == kMaxN && p.z && p.softplus && p.split == p.batch &&
         p.dim % (64 * kSeqNW) == 0 && dt_rank >= 1 && dt_rank <= 64 && dt_rank % 4 == 0 &&
         q.dt_rank == dt_rank && q.dtl && q.wdt &&
         q.wdt_ld >= 16 * nks && q.wdt_ld % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(q.wdt) & 7) == 0 &&
         (reinterpret_cast<uintptr_t>(q.dtl) & 7) == 0 && q.dtl_sl % 4 == 0 &&
         q.dtl_sb % 4 == 0 && q.dtl_sl >= dt_rank && dl_span < (1ll << 31) &&
         static_cast<long long>(p.seqlen) * q.dtl_sl * 2 < (1ll << 31);
}

// Segment length the chunked form would run (0 = the single pass), for the host's choice of
// dt_proj placement (inside the chunked scan up to kChDtpT steps).
int seq_chunk_steps(int batch, int dim, int seqlen, int segments) {
  const int S = segments_for(batch, dim, seqlen, segments, cus_or_calib(device_cus(nullptr)));
  if (S <= 1) return 0;
  int T, nblk;
  chunk_geometry(seqlen, S, &T, &nblk);
  return T;
}

// dt_proj inside the chunked scan (DTP): the mixer's bf16 token-major operands with the
// conv_proj-form W_dt (r_pad = 32 or 64 columns) and segments of at most kChDtpT steps.
bool seq_dtp_chunk_supported(const ScanParams& p, const DtpArgs& q, int dtype, int segments,
                             size_t workspace_bytes) {
  const bool bc1 = p.c_sl == p.b_sl && p.c_sb == p.b_sb &&
                   static_cast<const bf16_t*>(p.C) == static_cast<const bf16_t*>(p.B) + kMaxN;
  int S = 1;
  const size_t need = seq_workspace_bytes(p.batch, p.dim, p.seqlen, segments, &S);
  if (S <= 1) return false;
  int T, nblk;
  chunk_geometry(p.seqlen, S, &T, &nblk);
  return dtype == VM_DTYPE_BF16 && seq_supported(p, dtype) && seq_sgpr_bc(p, 2) && bc1 &&
         p.dstate == kMaxN && p.z && p.softplus && p.split == p.batch && T <= kChDtpT &&
         workspace_bytes >= need &&
         q.dtl && q.wdt && (q.wdt_ld == 32 || q.wdt_ld == 64) && q.dt_rank >= 1 &&
         q.dt_rank <= q.wdt_ld && q.dt_rank % 4 == 0 && q.dtl_sl >= q.dt_rank &&
         (reinterpret_cast<uintptr_t>(q.dtl) & 7) == 0 && q.dtl_sl % 4 == 0 && q.dtl_sb % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(q.wdt) & 15) == 0 &&
         static_cast<long long>(p.out_len) * q.dtl_sl * 2 < (1ll << 31);
}

void seq_dtp_chunk_launch(const ScanParams& p, const DtpArgs& q, int segments, void* workspace,
                          size_t workspace_bytes, void* sync, size_t sync_bytes, hipStream_t s) {
  const int dev_cus = device_cus(s);
  const int cus = cus_or_calib(dev_cus);
  int S = 1;
  seq_workspace_bytes(p.batch, p.dim, p.seqlen, segments, &S, cus);
  ChunkWork w{};
  chunk_geometry(p.seqlen, S, &w.T, &w.nblk);
  const long long grid = static_cast<long long>((p.dim + 63) / 64) * w.nblk * p.batch;
  if (sync && sync_bytes >= seq_sync_bytes(p.batch, p.dim, p.seqlen, segments, cus) &&
      grid <= dev_cus) {
    w.err = static_cast<unsigned*>(sync);
    w.epoch = w.err + 1;
    w.done = w.err + 2;
    w.gran = reinterpret_cast<unsigned long long*>(w.err + kSyncHeaderWords);
  }
  const size_t nb = static_cast<size_t>(p.batch) * w.nblk;
  w.segE = static_cast<float*>(workspace);
  w.segP = w.segE + nb * kChW * p.dim * kMaxN;
  w.aggH = w.segP + nb * kChW * p.dim;
  w.aggS = w.aggH + nb * p.dim * kMaxN;
  launch_chunk_p<bf16_t, true, true, true, false, true>(p, w, s, q);
}

void seq_dtp_launch(const ScanParams& p, const DtpArgs& q, int dt_rank, hipStream_t s) {
  const int groups = p.dim / 64;
  const dim3 grid(groups / kSeqNW, 1, p.batch);
  switch ((dt_rank + 15) / 16) {
    case 1: hipLaunchKernelGGL(scan_seq_dtp_kernel<1>, grid, dim3(64 * kSeqNW), 0, s, p, q); break;
    case 2: hipLaunchKernelGGL(scan_seq_dtp_kernel<2>, grid, dim3(64 * kSeqNW), 0, s, p, q); break;
    case 3: hipLaunchKernelGGL(scan_seq_dtp_kernel<3>, grid, dim3(64 * kSeqNW), 0, s, p, q); break;
    default: hipLaunchKernelGGL(scan_seq_dtp_kernel<4>, grid, dim3(64 * kSeqNW), 0, s, p, q); break;
  }
}

}  // namespace vm
