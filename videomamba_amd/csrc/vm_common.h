// Shared device/host helpers for the VideoMamba gfx950 kernels.
// Storage types: float (VM_DTYPE_F32) and bf16 held as uint16_t (VM_DTYPE_BF16).
// All arithmetic is fp32; bf16 is produced with a round-to-nearest-even cast
// (lowered to v_cvt_pk_bf16_f32 on gfx950, which keeps NaN a NaN).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "../../include/videomamba_hip.h"

namespace vm {

typedef uint16_t bf16_t;

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t from_f32<bf16_t>(float v) {
  __hip_bfloat16 h = __float2bfloat16(v);
  return *reinterpret_cast<bf16_t*>(&h);
}

// One 16-byte-per-lane buffer load straight into LDS: the DMA writes lane l's 16 bytes at
// (wave-uniform LDS base) + 16 l, so the LDS image is lane-linear and any layout is made by
// choosing each lane's source offset.  Out-of-range offsets read as zero.  Kept in a device
// function: written inline in a kernel-template lambda, clang dropped the kernels' host
// stubs (undefined symbols at load time).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           voff, 0, 0, 0);
}

// Round-trip through the storage type (models the reference's "->e" rounding points).
template <typename T> __device__ __forceinline__ float round_to(float v) {
  return to_f32(from_f32<T>(v));
}

// Load/store of a value whose storage dtype is only known at run time (state tensors).
__device__ __forceinline__ float load_dyn(const void* p, long long i, int dtype) {
  if (dtype == VM_DTYPE_BF16) return to_f32(reinterpret_cast<const bf16_t*>(p)[i]);
  return reinterpret_cast<const float*>(p)[i];
}
__device__ __forceinline__ void store_dyn(void* p, long long i, int dtype, float v) {
  if (dtype == VM_DTYPE_BF16) reinterpret_cast<bf16_t*>(p)[i] = from_f32<bf16_t>(v);
  else reinterpret_cast<float*>(p)[i] = v;
}

// 8 consecutive elements <-> 8 floats, 16-byte (bf16) or 2x16-byte (fp32) accesses.
__device__ __forceinline__ void load8(const bf16_t* p, float (&v)[8]) {
  uint4 q = *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void store8(bf16_t* p, const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = static_cast<uint32_t>(from_f32<bf16_t>(v[2 * i])) |
           (static_cast<uint32_t>(from_f32<bf16_t>(v[2 * i + 1])) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ void store8(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }
// torch F.softplus(beta=1, threshold=20)
__device__ __forceinline__ float softplus(float x) { return x <= 20.0f ? log1pf(__expf(x)) : x; }

constexpr float kLog2e = 1.4426950408889634f;
// Store policy of the streaming-chunk kernels (in_proj + conv, the chunked scan's y, the
// 128-row GEMM, add + RMSNorm up to kSmallStoreRows rows): sc1, i.e. written through to
// memory as they go.  A kernel that ends with B bytes dirty in L2 pays about B / 6 TB/s at
// the next dependent boundary (MI355X_MICROARCH.md "boundary"); a B = 1 layer leaves ~40 MB
// so, ~7 us.  Written through, they drain while the kernel runs: B = 1 M-16f chunk replay
// 2.28-2.34 -> 2.17-2.19 ms (profiles/r06ah_b1_xr_xcd_wt_ab.txt; product build r06ai_b1_wt_ab.txt: 2.47-2.49 -> 2.37 ms run()).  Values are unchanged.
constexpr int kSmallStoreWT = 16;
constexpr long long kSmallStoreRows = 32768;
constexpr float kLn2f = 0.6931471805599453f;

// softplus / silu from the hardware exp2 / log2 / rcp.  softplus = ln2*log2(1 + 2^(x/ln2))
// is within ~1.2e-7 absolute of log1p(exp(x)) (the relative error grows only where the
// step itself is < 1e-4 and contributes nothing measurable); threshold 20 as torch.
__device__ __forceinline__ float softplus_fast(float x) {
  return x > 20.0f ? x
                   : __builtin_amdgcn_logf(1.0f + __builtin_amdgcn_exp2f(x * kLog2e)) *
                         0.6931471805599453f;
}
__device__ __forceinline__ float silu_fast(float z) {
  return z * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-z * kLog2e));
}

}  // namespace vm

// ------------------------------------------------------------------ host-side helpers
namespace vmhost {
void set_error(const char* fmt, ...);
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline int dsize(int dtype) { return dtype == VM_DTYPE_BF16 ? 2 : 4; }
inline bool dtype_ok(int dtype) { return dtype == VM_DTYPE_F32 || dtype == VM_DTYPE_BF16; }
int launch_status(const char* what);
// CU count of the device that owns `stream` (the current device for the null stream),
// cached per device id; 0 when it cannot be queried
int device_cus(hipStream_t stream);
}  // namespace vmhost
