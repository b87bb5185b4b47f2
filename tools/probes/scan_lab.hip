// Token-major selective-scan lab (tools only, not product): variants of the
// channel-per-lane kernel at the bench shape (B clips, D=1152, L=3137, N=16, bf16,
// token-major rows, z inside xz, B/C inside x_dbl), timed with hipEvents and checked
// against variant 0.  Flags:
//   PK    packed f32 pairs over states (v_pk_mul/v_pk_fma), B/C as SGPR pairs
//   BC32  B/C read from a compact fp32 (rows, 32) side buffer — no SALU bf16 unpack
//   VOFF  per-lane VGPR step offsets for the 8 unrolled steps (one SGPR base per group),
//         main loop without clamps + clamped tail
//   SP/HZ softplus on delta / z gating (off only to price them)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>
#include <algorithm>

#ifndef LAB_ATTR
#define LAB_ATTR
#endif

typedef uint16_t bf16;
typedef float f2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const uint32_t* cptr;
constexpr float kLog2e = 1.4426950408889634f;
constexpr int kDead = 0x7ffffff0;

struct LabP {
  const bf16* u; const bf16* dl; const bf16* xz; const bf16* xdbl; const float* bc32;
  const float* A; const float* Dv; const float* bias; bf16* y; float* hl;
  int B, D, L, Lp, R, N;
  unsigned long long* clk;  // optional per-workgroup (memtime, realtime) stamps
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  void* ub = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(ub, 0, 1 << 30, 0x00020000);
}
__device__ __forceinline__ float softplus_fast(float x) {
  return x > 20.0f ? x : __builtin_amdgcn_logf(1.0f + __builtin_amdgcn_exp2f(x * kLog2e)) * 0.6931471805599453f;
}
__device__ __forceinline__ float silu_fast(float z) {
  return z * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-z * kLog2e));
}
__device__ __forceinline__ uint16_t to_bf16(float v) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %1" : "=v"(r) : "v"(v));
  return static_cast<uint16_t>(r);
}

template <bool PK, bool BC32, bool VOFF, bool SP, bool HZ, int MEM = 0, int kPF = 8, int NWV = 2, int LAY = 0>
__global__ __launch_bounds__(64 * NWV) LAB_ATTR void lab_kernel(const LabP p) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = blockIdx.x * NWV + wave;
  const int b = blockIdx.y;
  const int d0 = g * 64;
  if (d0 >= p.D) return;
  const int d = d0 + lane;
  const int L = p.L;
  unsigned long long* clk = p.clk ? p.clk + (static_cast<long long>(blockIdx.y) * gridDim.x + blockIdx.x) * 4 : nullptr;
  if (clk && threadIdx.x == 0) {
    const unsigned long long mt = __builtin_amdgcn_s_memtime(), rt = __builtin_amdgcn_s_memrealtime();
    clk[0] = mt;
    clk[1] = rt;
  }
  f2 A2[8], h[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    A2[q] = f2{p.A[d * 16 + 2 * q] * kLog2e, p.A[d * 16 + 2 * q + 1] * kLog2e};
    h[q] = f2{0.0f, 0.0f};
  }
  const float Dv = p.Dv[d], bias = p.bias[d];
  const long long row0 = MEM == 3 ? 0ll : static_cast<long long>(b) * p.Lp;  // MEM 3: every clip reads clip 0's rows (cache-resident pricing run)
  // LAY 1: u / delta channel-blocked (B, D/64, Lp, 64) — one contiguous 128-B-per-step
  // stream per wave; LAY 2: z and y blocked as well (pricing: same buffers re-indexed)
  const long long blk = (static_cast<long long>(b) * (p.D / 64) + g) * p.Lp * 64;
  const auto ur = rsrc(LAY >= 1 ? p.u + blk : p.u + row0 * p.D + d0);
  const auto dr = rsrc(LAY >= 1 ? p.dl + blk : p.dl + row0 * p.D + d0);
  const auto zr = rsrc(LAY >= 2 ? p.xz + blk : p.xz + row0 * 2 * p.D + p.D + d0);
  const auto yr = rsrc(LAY >= 2 ? p.y + blk : p.y + row0 * p.D + d0);
  const int us = LAY >= 1 ? 128 : p.D * 2, zs = LAY >= 2 ? 128 : p.D * 4;
  const int voff = lane * 2;
  // B/C rows
  const int bcw = BC32 ? 32 : (p.R + 2 * p.N) / 2;  // row stride in 32-bit words (x_dbl: 34)
  const uint32_t* bcbase = BC32 ? reinterpret_cast<const uint32_t*>(p.bc32 + row0 * 32)
                                : reinterpret_cast<const uint32_t*>(p.xdbl + row0 * (p.R + 2 * p.N) + p.R);
  constexpr int NW = BC32 ? 16 : 8;  // words per B (or C) row
  uint32_t bcv[2][2 * NW];
  auto bc_load = [&](int t, uint32_t (&dst)[2 * NW]) {
    const cptr bp = (cptr)(bcbase + static_cast<long long>(t) * bcw);
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      dst[i] = bp[i];
      dst[NW + i] = bp[NW + i];
    }
  };
  int vo[kPF], vz[kPF];
#pragma unroll
  for (int j = 0; j < kPF; ++j) {
    vo[j] = voff + j * us;
    vz[j] = voff + j * zs;
  }
  __builtin_amdgcn_s_waitcnt(0);
  const int tlast = L - 1;
  uint32_t ru[kPF], rd[kPF], rz[kPF];
#pragma unroll
  for (int j = 0; j < kPF; ++j) {
    const int t = j < L ? j : tlast;
    ru[j] = __builtin_amdgcn_raw_buffer_load_b16(ur, voff, t * us, 0);
    rd[j] = __builtin_amdgcn_raw_buffer_load_b16(dr, voff, t * us, 0);
    rz[j] = HZ ? __builtin_amdgcn_raw_buffer_load_b16(zr, voff, t * zs, 0) : 0u;
    __builtin_amdgcn_sched_barrier(0);  // same (u, delta, z) per-step order as the loop
  }
  bc_load(0, bcv[0]);

  auto step = [&](int t, int j, bool live, int soff_u, int soff_z, int vou, int voz) {
    const float uu = __uint_as_float(ru[j] << 16);
    const float dr_ = __uint_as_float(rd[j] << 16);
    const float zz = __uint_as_float(rz[j] << 16);
    ru[j] = __builtin_amdgcn_raw_buffer_load_b16(ur, vou, soff_u, 0);
    rd[j] = __builtin_amdgcn_raw_buffer_load_b16(dr, vou, soff_u, 0);
    if (HZ) rz[j] = __builtin_amdgcn_raw_buffer_load_b16(zr, voz, soff_z, 0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    bc_load(t + 1 < L ? t + 1 : tlast, bcv[(j + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);
    float dlv = dr_ + bias;
    if (SP) dlv = softplus_fast(dlv);
    dlv = live ? dlv : 0.0f;
    const float du = dlv * uu;
    const uint32_t (&cw)[2 * NW] = bcv[j & 1];
    float y;
    if constexpr (PK) {
      const f2 dl2 = {dlv, dlv}, du2 = {du, du};
      f2 ya = {Dv * uu, 0.0f}, yb = {0.0f, 0.0f};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        f2 Bp, Cp;
        if constexpr (BC32) {
          Bp = f2{__uint_as_float(cw[2 * q]), __uint_as_float(cw[2 * q + 1])};
          Cp = f2{__uint_as_float(cw[NW + 2 * q]), __uint_as_float(cw[NW + 2 * q + 1])};
        } else {
          Bp = f2{__uint_as_float(cw[q] << 16), __uint_as_float(cw[q] & 0xffff0000u)};
          Cp = f2{__uint_as_float(cw[NW + q] << 16), __uint_as_float(cw[NW + q] & 0xffff0000u)};
        }
        const f2 x = dl2 * A2[q];
        const f2 a = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
        h[q] = __builtin_elementwise_fma(a, h[q], du2 * Bp);
        if (q & 1) yb = __builtin_elementwise_fma(h[q], Cp, yb);
        else ya = __builtin_elementwise_fma(h[q], Cp, ya);
      }
      const f2 ys = ya + yb;
      y = ys.x + ys.y;
    } else {
      float y0 = Dv * uu, y1 = 0.0f;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float B0, B1, C0, C1;
        if constexpr (BC32) {
          B0 = __uint_as_float(cw[2 * q]); B1 = __uint_as_float(cw[2 * q + 1]);
          C0 = __uint_as_float(cw[NW + 2 * q]); C1 = __uint_as_float(cw[NW + 2 * q + 1]);
        } else {
          B0 = __uint_as_float(cw[q] << 16); B1 = __uint_as_float(cw[q] & 0xffff0000u);
          C0 = __uint_as_float(cw[NW + q] << 16); C1 = __uint_as_float(cw[NW + q] & 0xffff0000u);
        }
        h[q].x = fmaf(__builtin_amdgcn_exp2f(dlv * A2[q].x), h[q].x, du * B0);
        h[q].y = fmaf(__builtin_amdgcn_exp2f(dlv * A2[q].y), h[q].y, du * B1);
        y0 = fmaf(h[q].x, C0, y0);
        y1 = fmaf(h[q].y, C1, y1);
      }
      y = y0 + y1;
    }
    if (HZ) y *= silu_fast(zz);
    __builtin_amdgcn_raw_buffer_store_b16(to_bf16(y), yr, live ? voff : kDead, t * us, 0);
  };

  int t0 = 0;
  if constexpr (VOFF) {
    // main loop: every step live and every prefetch (t + 8) in range
    for (; t0 + 2 * kPF <= L; t0 += kPF) {
      const int su = (t0 + kPF) * us, sz = (t0 + kPF) * zs;
#pragma unroll
      for (int j = 0; j < kPF; ++j) {
        const int t = t0 + j;
        const float uu = __uint_as_float(ru[j] << 16);
        const float dr_ = __uint_as_float(rd[j] << 16);
        const float zz = __uint_as_float(rz[j] << 16);
        if constexpr (MEM == 0 || MEM == 3 || MEM == 5) {
          ru[j] = __builtin_amdgcn_raw_buffer_load_b16(ur, vo[j], su, 0);
          rd[j] = __builtin_amdgcn_raw_buffer_load_b16(dr, vo[j], su, 0);
          if (HZ) rz[j] = __builtin_amdgcn_raw_buffer_load_b16(zr, vz[j], sz, 0);
        } else if constexpr (MEM == 4) {  // u and delta as one interleaved dword (pricing)
          const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(ur, vo[j] + voff, su, 0);
          ru[j] = w;
          rd[j] = w >> 16;
          if (HZ) rz[j] = __builtin_amdgcn_raw_buffer_load_b16(zr, vz[j], sz, 0);
        } else {
          ru[j] = ru[j] * 0x10001u + 0x3u;  // register-only stand-ins (pricing runs)
          rd[j] = (rd[j] ^ 0x40u) & 0xbfffu;
          rz[j] = rz[j] + 0x11u;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        bc_load(t + 1, bcv[(j + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        float dlv = dr_ + bias;
        if (SP) dlv = softplus_fast(dlv);
        const float du = dlv * uu;
        const uint32_t (&cw)[2 * NW] = bcv[j & 1];
        float y;
        if constexpr (PK) {
          const f2 dl2 = {dlv, dlv}, du2 = {du, du};
          f2 ya = {Dv * uu, 0.0f}, yb = {0.0f, 0.0f};
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            f2 Bp, Cp;
            if constexpr (BC32) {
              Bp = f2{__uint_as_float(cw[2 * q]), __uint_as_float(cw[2 * q + 1])};
              Cp = f2{__uint_as_float(cw[NW + 2 * q]), __uint_as_float(cw[NW + 2 * q + 1])};
            } else {
              Bp = f2{__uint_as_float(cw[q] << 16), __uint_as_float(cw[q] & 0xffff0000u)};
              Cp = f2{__uint_as_float(cw[NW + q] << 16), __uint_as_float(cw[NW + q] & 0xffff0000u)};
            }
            const f2 x = dl2 * A2[q];
            const f2 a = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
            h[q] = __builtin_elementwise_fma(a, h[q], du2 * Bp);
            if (q & 1) yb = __builtin_elementwise_fma(h[q], Cp, yb);
            else ya = __builtin_elementwise_fma(h[q], Cp, ya);
          }
          const f2 ys = ya + yb;
          y = ys.x + ys.y;
        } else {
          float y0 = Dv * uu, y1 = 0.0f;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float B0, B1, C0, C1;
            if constexpr (BC32) {
              B0 = __uint_as_float(cw[2 * q]); B1 = __uint_as_float(cw[2 * q + 1]);
              C0 = __uint_as_float(cw[NW + 2 * q]); C1 = __uint_as_float(cw[NW + 2 * q + 1]);
            } else {
              B0 = __uint_as_float(cw[q] << 16); B1 = __uint_as_float(cw[q] & 0xffff0000u);
              C0 = __uint_as_float(cw[NW + q] << 16); C1 = __uint_as_float(cw[NW + q] & 0xffff0000u);
            }
            h[q].x = fmaf(__builtin_amdgcn_exp2f(dlv * A2[q].x), h[q].x, du * B0);
            h[q].y = fmaf(__builtin_amdgcn_exp2f(dlv * A2[q].y), h[q].y, du * B1);
            y0 = fmaf(h[q].x, C0, y0);
            y1 = fmaf(h[q].y, C1, y1);
          }
          y = y0 + y1;
        }
        if (HZ) y *= silu_fast(zz);
        if ((MEM < 2 || MEM == 3) || y == 12345.0f) __builtin_amdgcn_raw_buffer_store_b16(to_bf16(y), yr, vo[j], t0 * us, 0);
      }
    }
  }
  // clamped tail (or the whole sequence without VOFF)
  for (; t0 < L; t0 += kPF) {
#pragma unroll
    for (int j = 0; j < kPF; ++j) {
      const int t = t0 + j;
      const int tn = t + kPF < L ? t + kPF : tlast;
      step(t, j, t < L, tn * us, tn * zs, voff, voff);
    }
  }
  float* hl = p.hl + (static_cast<long long>(b) * p.D + d) * 16;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    hl[2 * q] = h[q].x;
    hl[2 * q + 1] = h[q].y;
  }
  if (clk && threadIdx.x == 0) {
    const unsigned long long mt = __builtin_amdgcn_s_memtime(), rt = __builtin_amdgcn_s_memrealtime();
    clk[2] = mt;
    clk[3] = rt;
  }
}


// LDS-DMA staged variant: u / delta / z arrive 8 steps x 64 channels (1 KB) per
// global_load_lds_dwordx4 into a per-wave ring of R tiles; each step reads its channel
// with ds_read_u16_d16_hi (the bf16 lands in the high half of a zeroed VGPR = the fp32
// value, no unpack).  Waits are explicit: vmcnt before a tile's first step (DMA), one
// lgkmcnt(0) per step (B/C scalar loads + the three LDS reads).
template <int R>
__global__ __launch_bounds__(128) void lab_dma_kernel(const LabP p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = blockIdx.x * 2 + wave;
  const int b = blockIdx.y;
  const int d0 = g * 64;
  if (d0 >= p.D) return;
  const int d = d0 + lane;
  const int L = p.L;
  f2 A2[8], h[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    A2[q] = f2{p.A[d * 16 + 2 * q] * kLog2e, p.A[d * 16 + 2 * q + 1] * kLog2e};
    h[q] = f2{0.0f, 0.0f};
  }
  const float Dv = p.Dv[d], bias = p.bias[d];
  const long long row0 = static_cast<long long>(b) * p.Lp;
  const bf16* ub = p.u + row0 * p.D + d0;
  const bf16* db = p.dl + row0 * p.D + d0;
  const bf16* zb = p.xz + row0 * 2 * p.D + p.D + d0;
  const auto yr = rsrc(p.y + row0 * p.D + d0);
  const int us = p.D * 2;
  const int voff = lane * 2;
  // wave's LDS ring: [op 0..2][slot 0..R-1][8 steps][64 ch] bf16
  uint8_t* ring = lds_raw + wave * (3 * R * 1024);
  const uint32_t ring_lds = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(ring));
  const int lrow = lane >> 3, lcol = (lane & 7) * 8;
  auto dma = [&](int k) {  // tile k -> slot k % R
    const int slot = k % R;
    int r = k * 8 + lrow;
    r = r < L ? r : L - 1;
    __builtin_amdgcn_global_load_lds((const void*)(ub + (long long)r * p.D + lcol),
        (__attribute__((address_space(3))) void*)(ring + (0 * R + slot) * 1024), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(db + (long long)r * p.D + lcol),
        (__attribute__((address_space(3))) void*)(ring + (1 * R + slot) * 1024), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(zb + (long long)r * 2 * p.D + lcol),
        (__attribute__((address_space(3))) void*)(ring + (2 * R + slot) * 1024), 16, 0, 0);
  };
  const uint32_t* bcbase = reinterpret_cast<const uint32_t*>(p.xdbl + row0 * (p.R + 2 * p.N) + p.R);
  const int bcw = (p.R + 2 * p.N) / 2;
  uint32_t bcv[2][16];
  auto bc_load = [&](int t, uint32_t (&dst)[16]) {
    const cptr bp = (cptr)(bcbase + static_cast<long long>(t) * bcw);
#pragma unroll
    for (int i = 0; i < 16; ++i) dst[i] = bp[i];
  };
  const int ntiles = (L + 7) / 8;
  __builtin_amdgcn_s_waitcnt(0);
  for (int k = 0; k < R - 1 && k < ntiles; ++k) dma(k);
  bc_load(0, bcv[0]);
  uint32_t ru = 0, rd = 0, rz = 0;
  const uint32_t my = ring_lds + voff;
  for (int k = 0; k < ntiles; ++k) {
    if (k + R - 1 < ntiles) dma(k + R - 1);
    // tile k's DMA is the oldest outstanding group but (R-1) x (3 DMA + 8 stores)
    if constexpr (R == 2) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
    else if constexpr (R == 3) asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(33)" ::: "memory");
    const uint32_t su = my + ((0 * R + k % R) * 1024), sdl = my + ((1 * R + k % R) * 1024),
                   sz = my + ((2 * R + k % R) * 1024);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = k * 8 + j;
      asm volatile("ds_read_u16_d16_hi %0, %1 offset:%2" : "+v"(ru) : "v"(su), "i"(j * 128));
      asm volatile("ds_read_u16_d16_hi %0, %1 offset:%2" : "+v"(rd) : "v"(sdl), "i"(j * 128));
      asm volatile("ds_read_u16_d16_hi %0, %1 offset:%2" : "+v"(rz) : "v"(sz), "i"(j * 128));
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this step's B/C + the LDS reads
      asm volatile("" : "+v"(ru), "+v"(rd), "+v"(rz));  // order the reads' uses after it
      bc_load(t + 1 < L ? t + 1 : L - 1, bcv[(j + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      const bool live = t < L;
      const float uu = __uint_as_float(ru), zz = __uint_as_float(rz);
      float dlv = softplus_fast(__uint_as_float(rd) + bias);
      dlv = live ? dlv : 0.0f;
      const float du = dlv * uu;
      const uint32_t (&cw)[16] = bcv[j & 1];
      const f2 dl2 = {dlv, dlv}, du2 = {du, du};
      f2 ya = {Dv * uu, 0.0f}, yb = {0.0f, 0.0f};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const f2 Bp = f2{__uint_as_float(cw[q] << 16), __uint_as_float(cw[q] & 0xffff0000u)};
        const f2 Cp = f2{__uint_as_float(cw[8 + q] << 16), __uint_as_float(cw[8 + q] & 0xffff0000u)};
        const f2 x = dl2 * A2[q];
        const f2 a = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
        h[q] = __builtin_elementwise_fma(a, h[q], du2 * Bp);
        if (q & 1) yb = __builtin_elementwise_fma(h[q], Cp, yb);
        else ya = __builtin_elementwise_fma(h[q], Cp, ya);
      }
      const f2 ys = ya + yb;
      const float y = (ys.x + ys.y) * silu_fast(zz);
      __builtin_amdgcn_raw_buffer_store_b16(to_bf16(y), yr, live ? voff : kDead, t * us, 0);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  float* hl = p.hl + (static_cast<long long>(b) * p.D + d) * 16;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    hl[2 * q] = h[q].x;
    hl[2 * q + 1] = h[q].y;
  }
}

// Pure streaming reference (no scan math): the scan's u / delta / z reads and y writes at
// VEC bf16 channels per lane (VEC 1 = the scan's 2-byte lanes; VEC 8 = 16-byte lanes).
template <int VEC>
__global__ __launch_bounds__(128) void stream_kernel(const LabP p) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = blockIdx.x * 2 + wave;
  const int b = blockIdx.y;
  const int d0 = g * 64 * VEC;
  if (d0 >= p.D) return;
  const bool act = d0 + lane * VEC < p.D;
  const long long row0 = static_cast<long long>(b) * p.Lp;
  const auto ur = rsrc(p.u + row0 * p.D + d0);
  const auto dr = rsrc(p.dl + row0 * p.D + d0);
  const auto zr = rsrc(p.xz + row0 * 2 * p.D + p.D + d0);
  const auto yr = rsrc(p.y + row0 * p.D + d0);
  const int us = p.D * 2, zs = p.D * 4;
  const int voff = act ? lane * 2 * VEC : kDead;
  constexpr int PF = 8;
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  if constexpr (VEC == 1) {
    uint32_t ru[PF], rd[PF], rz[PF];
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      ru[j] = __builtin_amdgcn_raw_buffer_load_b16(ur, voff, j * us, 0);
      rd[j] = __builtin_amdgcn_raw_buffer_load_b16(dr, voff, j * us, 0);
      rz[j] = __builtin_amdgcn_raw_buffer_load_b16(zr, voff, j * zs, 0);
    }
    for (int t0 = 0; t0 < p.L; t0 += PF) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int t = t0 + j;
        const int tn = t + PF < p.L ? t + PF : p.L - 1;
        const uint32_t y = ru[j] + rd[j] + rz[j];
        ru[j] = __builtin_amdgcn_raw_buffer_load_b16(ur, voff, tn * us, 0);
        rd[j] = __builtin_amdgcn_raw_buffer_load_b16(dr, voff, tn * us, 0);
        rz[j] = __builtin_amdgcn_raw_buffer_load_b16(zr, voff, tn * zs, 0);
        __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(y), yr, t < p.L ? voff : kDead, t * us, 0);
      }
    }
  } else {
    v4 ru[PF], rd[PF], rz[PF];
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      ru[j] = __builtin_amdgcn_raw_buffer_load_b128(ur, voff, j * us, 0);
      rd[j] = __builtin_amdgcn_raw_buffer_load_b128(dr, voff, j * us, 0);
      rz[j] = __builtin_amdgcn_raw_buffer_load_b128(zr, voff, j * zs, 0);
    }
    for (int t0 = 0; t0 < p.L; t0 += PF) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int t = t0 + j;
        const int tn = t + PF < p.L ? t + PF : p.L - 1;
        const v4 y = ru[j] + rd[j] + rz[j];
        ru[j] = __builtin_amdgcn_raw_buffer_load_b128(ur, voff, tn * us, 0);
        rd[j] = __builtin_amdgcn_raw_buffer_load_b128(dr, voff, tn * us, 0);
        rz[j] = __builtin_amdgcn_raw_buffer_load_b128(zr, voff, tn * zs, 0);
        __builtin_amdgcn_raw_buffer_store_b128(y, yr, t < p.L ? voff : kDead, t * us, 0);
      }
    }
  }
}

static uint16_t f2bf(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  x += 0x7fff + ((x >> 16) & 1);
  return static_cast<uint16_t>(x >> 16);
}
static float bf2f(uint16_t v) {
  uint32_t x = static_cast<uint32_t>(v) << 16;
  float f;
  memcpy(&f, &x, 4);
  return f;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 336;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int D = 1152, L = argc > 3 ? atoi(argv[3]) : 3137, N = 16, R = 36, Lp = (L + 7) / 8 * 8;
  const long long rows = static_cast<long long>(B) * Lp;
  // synthetic inputs generated on the device side by a simple hash (host memory stays small)
  std::vector<float> hA(D * N), hD(D), hb(D);
  for (int d = 0; d < D; ++d) {
    for (int n = 0; n < N; ++n) hA[d * N + n] = -(n + 1.0f);
    hD[d] = 1.0f;
    hb[d] = -4.0f;
  }
  bf16 *u, *dl, *xz, *xdbl, *y, *y0;
  float *bc32, *A, *Dv, *bias, *hl, *hl0;
  CK(hipMalloc(&u, rows * D * 2));
  CK(hipMalloc(&dl, rows * D * 2));
  CK(hipMalloc(&xz, rows * 2 * D * 2));
  CK(hipMalloc(&xdbl, rows * (R + 2 * N) * 2));
  CK(hipMalloc(&bc32, rows * 32 * 4));
  CK(hipMalloc(&y, rows * D * 2));
  CK(hipMalloc(&y0, rows * D * 2));
  CK(hipMalloc(&A, D * N * 4));
  CK(hipMalloc(&Dv, D * 4));
  CK(hipMalloc(&bias, D * 4));
  CK(hipMalloc(&hl, static_cast<long long>(B) * D * N * 4));
  CK(hipMalloc(&hl0, static_cast<long long>(B) * D * N * 4));
  CK(hipMemcpy(A, hA.data(), D * N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(Dv, hD.data(), D * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, hb.data(), D * 4, hipMemcpyHostToDevice));
  {
    // fill with host-generated pseudo-random bf16 in chunks
    const long long chunk = 1 << 24;
    std::vector<uint16_t> buf(chunk);
    uint64_t s = 0x9e3779b97f4a7c15ull;
    auto rnd = [&]() {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      return ((s >> 11) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0;
    };
    auto fill = [&](bf16* dst, long long n, float scale, float shift) {
      for (long long o = 0; o < n; o += chunk) {
        const long long m = n - o < chunk ? n - o : chunk;
        for (long long i = 0; i < m; ++i) buf[i] = f2bf(static_cast<float>(rnd() * scale + shift));
        CK(hipMemcpy(dst + o, buf.data(), m * 2, hipMemcpyHostToDevice));
      }
    };
    fill(u, rows * D, 1.7f, 0.0f);
    fill(dl, rows * D, 0.9f, -4.0f);
    fill(xz, rows * 2 * D, 1.7f, 0.0f);
    // x_dbl and its fp32 B/C copy (exact: bf16 values widened)
    std::vector<uint16_t> xd(rows * (R + 2 * N));
    for (auto& v : xd) v = f2bf(static_cast<float>(rnd() * 1.7));
    std::vector<float> b32(rows * 32);
    for (long long r = 0; r < rows; ++r)
      for (int k = 0; k < 32; ++k) b32[r * 32 + k] = bf2f(xd[r * (R + 2 * N) + R + k]);
    CK(hipMemcpy(xdbl, xd.data(), xd.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(bc32, b32.data(), b32.size() * 4, hipMemcpyHostToDevice));
  }
  LabP p{u, dl, xz, xdbl, bc32, A, Dv, bias, y, hl, B, D, L, Lp, R, N, nullptr};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double algo = static_cast<double>(B) * D * L * 4 * 2 + 2.0 * B * N * L * 2 + 4.0 * D * N + 8.0 * D;
  auto bench = [&](const char* name, void (*k)(LabP), bool ref, int nwv = 2, size_t lds = 0) {
    dim3 grid(nwv == 16 ? (D / 512 + 2) / 2 : (D / 64 + nwv - 1) / nwv, B);
    LabP q = p;
    if (ref) { q.y = y0; q.hl = hl0; }
    hipLaunchKernelGGL(k, grid, dim3(nwv == 16 ? 128 : 64 * nwv), lds, 0, q);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, grid, dim3(nwv == 16 ? 128 : 64 * nwv), lds, 0, q);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    double maxdiff = 0.0, maxh = 0.0;
    if (!ref) {
      // compare against the reference variant on a sample of rows
      std::vector<uint16_t> a(D * 64), c(D * 64);
      const int nr = L < 64 ? L : 64;
      for (int bb : {0, B / 2, B - 1}) {
        for (long long r0 : {0LL, L > 1600 ? 1500LL : 0LL, static_cast<long long>(L - nr)}) {
          const long long off = (static_cast<long long>(bb) * Lp + r0) * D;
          CK(hipMemcpy(a.data(), y + off, D * nr * 2, hipMemcpyDeviceToHost));
          CK(hipMemcpy(c.data(), y0 + off, D * nr * 2, hipMemcpyDeviceToHost));
          for (int i = 0; i < D * nr; ++i) {
            const double df = fabs(bf2f(a[i]) - bf2f(c[i])) / (1.0 + fabs(bf2f(c[i])));
            if (df > maxdiff) maxdiff = df;
          }
        }
      }
      std::vector<float> ha(static_cast<long long>(B) * D * N), hc(ha.size());
      CK(hipMemcpy(ha.data(), hl, ha.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hc.data(), hl0, hc.size() * 4, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < ha.size(); ++i) {
        const double df = fabs(ha[i] - hc[i]) / (1.0 + fabs(hc[i]));
        if (df > maxh) maxh = df;
      }
    }
    printf("%-34s B=%d %9.1f us  %6.2f us/clip-layer  %6.1f GB/s  frac %.4f  maxdiff y %.2e h %.2e\n",
           name, B, us, us / B, algo / (us * 1e-6) / 1e9, algo / (us * 1e-6) / 8e12, maxdiff, maxh);
  };
  if (argc > 4 && strcmp(argv[4], "clock") == 0) {
    // in-kernel clock (MI355X_MICROARCH.md DVFS item 6): ~2 s of back-to-back launches,
    // then one launch stamping s_memtime / s_memrealtime per workgroup; median over
    // workgroups of dmemtime / drealtime * 100 MHz
    const int nwg = (D / 64 + 1) / 2 * B;
    unsigned long long* clk;
    CK(hipMalloc(&clk, static_cast<size_t>(nwg) * 4 * 8));
    auto clock_of = [&](const char* name, void (*k)(LabP)) {
      dim3 grid((D / 64 + 1) / 2, B);
      LabP q = p;
      CK(hipEventRecord(e0));
      int n = 0;
      float ms = 0.0f;
      for (; n < 2000; ++n) {
        hipLaunchKernelGGL(k, grid, dim3(128), 0, 0, q);
        if (n % 50 == 49) {
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (ms > 2000.0f) break;
        }
      }
      q.clk = clk;
      hipLaunchKernelGGL(k, grid, dim3(128), 0, 0, q);
      std::vector<unsigned long long> c(static_cast<size_t>(nwg) * 4);
      CK(hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost));
      std::vector<double> f;
      for (int i = 0; i < nwg; ++i) {
        const double dm = static_cast<double>(c[4 * i + 2] - c[4 * i]);
        const double dr = static_cast<double>(c[4 * i + 3] - c[4 * i + 1]);
        if (dr > 0) f.push_back(dm / dr * 0.1);  // GHz (realtime ticks at 100 MHz)
      }
      std::sort(f.begin(), f.end());
      printf("%-34s %d launches, %.1f us each; in-kernel clock median %.3f GHz (p10 %.3f, p90 %.3f)\n",
             name, n + 1, ms * 1e3 / (n + 1), f[f.size() / 2], f[f.size() / 10], f[f.size() * 9 / 10]);
      fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
      clock_of("pk voff pf8 (product stream)", lab_kernel<true, false, true, true, true>);
      clock_of("pk voff pf8 no vmem", lab_kernel<true, false, true, true, true, 2>);
      clock_of("pk voff pf8 shared rows (L2)", lab_kernel<true, false, true, true, true, 3>);
    }
    return 0;
  }
  if (argc > 4 && strcmp(argv[4], "calib") == 0) {
    // PMC calibration run: the scan's access pattern (2-byte lanes, one 128-B row segment
    // per wave per operand and step) with a known byte count and no scan math
    bench("stream only, 2 B/lane (calibration)", stream_kernel<1>, false);
    printf("calibration bytes per launch: read %.0f write %.0f\n", 3.0 * rows * D * 2, 1.0 * rows * D * 2);
    return 0;
  }
  bench("ref scalar bf16-BC (baseline)", lab_kernel<false, false, false, true, true>, true);
  if (argc > 4 && strcmp(argv[4], "occupancy") == 0) {
    // waves per SIMD capped by dynamic LDS per 2-wave workgroup (160 KB per CU)
    for (int rep = 0; rep < 2; ++rep) {
      bench("pk voff pf8, 5 waves/SIMD (16 KB)", lab_kernel<true, false, true, true, true>, false, 2, 16 * 1024);
      bench("pk voff pf8, 4 waves/SIMD (20 KB)", lab_kernel<true, false, true, true, true>, false, 2, 20 * 1024);
      bench("pk voff pf8, 3 waves/SIMD (26 KB)", lab_kernel<true, false, true, true, true>, false, 2, 26 * 1024);
    }
    return 0;
  }
  for (int rep = 0; rep < 2; ++rep) {
    bench("pk voff pf8 (ordered prologue)", lab_kernel<true, false, true, true, true>, false);
    bench("pk pf8 (ordered prologue)", lab_kernel<true, false, false, true, true>, false);
    bench("pk voff pf8 no vmem", lab_kernel<true, false, true, true, true, 2>, false);
  }
  return 0;
}
