// Fused residual-add + RMSNorm / LayerNorm.  Replaces mamba-ssm's rms_norm_fn /
// layer_norm_fn as called at models/videomamba/videomamba.py:152-166 (prenorm, per
// block) and :904-918 (final norm): s = x (+ residual) in fp32, statistics on the fp32
// sum, y = xhat * w (+ b) rounded once to the output dtype, residual_out = s.
//
// One wave per row; each lane keeps its strided slice of the row in registers, so the
// row is read once and written once (HBM-bound: 12 B/elem at bf16 x, fp32 residual).

#include "vm_common.h"

namespace vm {

struct NormParams {
  const void* x; const void* res; const float* w; const float* bias; void* out; void* res_out;
  long long rows; int cols; float eps; int is_rms, x_dtype, res_dtype, out_dtype, ro_dtype;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ void load4_dyn(const void* p, long long i, int dtype, float (&v)[4]) {
  if (dtype == VM_DTYPE_BF16) {
    const uint2 q = *reinterpret_cast<const uint2*>(static_cast<const bf16_t*>(p) + i);
    v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
    v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
  } else {
    const float4 q = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
}
__device__ __forceinline__ void store4_dyn(void* p, long long i, int dtype, const float (&v)[4]) {
  if (dtype == VM_DTYPE_BF16) {
    uint2 q;
    q.x = static_cast<uint32_t>(from_f32<bf16_t>(v[0])) | (static_cast<uint32_t>(from_f32<bf16_t>(v[1])) << 16);
    q.y = static_cast<uint32_t>(from_f32<bf16_t>(v[2])) | (static_cast<uint32_t>(from_f32<bf16_t>(v[3])) << 16);
    *reinterpret_cast<uint2*>(static_cast<bf16_t*>(p) + i) = q;
  } else {
    *reinterpret_cast<float4*>(static_cast<float*>(p) + i) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// The block's common case — bf16 x / out, fp32 residual in / out, RMSNorm, no bias — with
// every access a branch-free buffer access over the wave's own row (chunks past `cols` get
// an out-of-range offset: they read 0 and store nothing) and every load of the row issued
// before the first use.  The dtype-generic form below puts each access behind the dtype
// and column-range branches, and hipcc waits vmcnt(0) at their joins: a chain of dependent
// round trips per row that set the B = 1 chunk's add+norm at ~7 us.  Same arithmetic in
// the same order as add_norm_vec_kernel (bit-identical outputs).
constexpr int kNormOut = 0x7ffffff0;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t norm_row_rsrc(const void* base, int bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  void* ub = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(ub, 0, bytes, 0x00020000);
}
// (no early exit for the rows past the end: their buffers have 0-byte ranges, so every
// access is a no-op, and the kernel-argument loads are not split by a branch into two
// dependent rounds before the first global load)
template <int CPL, bool RES, bool RO, int ST = 0>
__global__ __launch_bounds__(256) void add_rms_bf16_kernel(const NormParams p) {
  const long long row0 = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool live = row0 < p.rows;
  const long long row = live ? row0 : 0;
  const int lane = threadIdx.x & 63;
  const long long base = row * p.cols;
  const int cb2 = live ? p.cols * 2 : 0, cb4 = live ? p.cols * 4 : 0;
  const auto xr = norm_row_rsrc(static_cast<const bf16_t*>(p.x) + base, cb2);
  const auto rr = norm_row_rsrc(RES ? static_cast<const float*>(p.res) + base : p.w, cb4);
  const auto wr = norm_row_rsrc(p.w, p.cols * 4);
  const auto orr = norm_row_rsrc(static_cast<bf16_t*>(p.out) + base, cb2);
  const auto ror = norm_row_rsrc(RO ? static_cast<float*>(p.res_out) + base : p.w, cb4);
  typedef __attribute__((__vector_size__(4 * sizeof(float)))) float v4f;
  auto off = [&](int j, int es) {
    int o = lane * 4 + 256 * j < p.cols ? (lane * 4 + 256 * j) * es : kNormOut;
    asm volatile("" : "+v"(o));  // a select, not a branch around the access
    return o;
  };
  uint32_t xq[CPL][2];
  v4f rq[CPL], wq[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const auto q = __builtin_amdgcn_raw_buffer_load_b64(xr, off(j, 2), 0, 0);
    xq[j][0] = q[0];
    xq[j][1] = q[1];
    if constexpr (RES) rq[j] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rr, off(j, 4), 0, 0));
  }
#pragma unroll
  for (int j = 0; j < CPL; ++j)
    wq[j] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(wr, off(j, 4), 0, 0));
  __builtin_amdgcn_sched_barrier(0);  // all of the row's loads in flight before any use
  float v[CPL][4];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    v[j][0] = __uint_as_float(xq[j][0] << 16); v[j][1] = __uint_as_float(xq[j][0] & 0xffff0000u);
    v[j][2] = __uint_as_float(xq[j][1] << 16); v[j][3] = __uint_as_float(xq[j][1] & 0xffff0000u);
    if constexpr (RES) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[j][i] += rq[j][i];
    }
  }
  float sq = 0.0f;
#pragma unroll
  for (int j = 0; j < CPL; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) sq = fmaf(v[j][i], v[j][i], sq);
  const float rstd = rsqrtf(wave_sum(sq) / p.cols + p.eps);
  const float mean = 0.0f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    float y[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = (v[j][i] - mean) * rstd * wq[j][i];
    typedef __attribute__((__vector_size__(2 * sizeof(int)))) int v2i;
    const v2i o2 = {static_cast<int>(static_cast<uint32_t>(from_f32<bf16_t>(y[0])) |
                                     (static_cast<uint32_t>(from_f32<bf16_t>(y[1])) << 16)),
                    static_cast<int>(static_cast<uint32_t>(from_f32<bf16_t>(y[2])) |
                                     (static_cast<uint32_t>(from_f32<bf16_t>(y[3])) << 16))};
    __builtin_amdgcn_raw_buffer_store_b64(o2, orr, off(j, 2), 0, ST);
    if constexpr (RO) {
      typedef __attribute__((__vector_size__(4 * sizeof(int)))) int v4i;
      const v4i r4 = {static_cast<int>(__float_as_uint(v[j][0])), static_cast<int>(__float_as_uint(v[j][1])),
                      static_cast<int>(__float_as_uint(v[j][2])), static_cast<int>(__float_as_uint(v[j][3]))};
      __builtin_amdgcn_raw_buffer_store_b128(r4, ror, off(j, 4), 0, ST);
    }
  }
}

// Vectorised form for cols % 4 == 0 and 16-byte aligned rows: lane owns 4-element
// chunks lane*4 + 256*j (8-byte bf16 / 16-byte fp32 accesses).
template <int CPL>  // chunks per lane (cols <= 256 * CPL)
__global__ __launch_bounds__(256) void add_norm_vec_kernel(const NormParams p) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const int lane = threadIdx.x & 63;
  const long long base = row * p.cols;
  float v[CPL][4];
  float sum = 0.0f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane * 4 + 256 * j;
    if (c < p.cols) {
      load4_dyn(p.x, base + c, p.x_dtype, v[j]);
      if (p.res) {
        float r[4];
        load4_dyn(p.res, base + c, p.res_dtype, r);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[j][i] += r[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[j][i] = 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) sum += v[j][i];
  }
  float rstd, mean = 0.0f;
  if (p.is_rms) {
    float sq = 0.0f;
#pragma unroll
    for (int j = 0; j < CPL; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) sq = fmaf(v[j][i], v[j][i], sq);
    rstd = rsqrtf(wave_sum(sq) / p.cols + p.eps);
  } else {
    mean = wave_sum(sum) / p.cols;
    float sq = 0.0f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const bool in = lane * 4 + 256 * j < p.cols;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dv = in ? v[j][i] - mean : 0.0f;
        sq = fmaf(dv, dv, sq);
      }
    }
    rstd = rsqrtf(wave_sum(sq) / p.cols + p.eps);
  }
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane * 4 + 256 * j;
    if (c < p.cols) {
      const float4 w = *reinterpret_cast<const float4*>(p.w + c);
      const float wv[4] = {w.x, w.y, w.z, w.w};
      float y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        y[i] = (v[j][i] - mean) * rstd * wv[i];
        if (p.bias) y[i] += p.bias[c + i];
      }
      store4_dyn(p.out, base + c, p.out_dtype, y);
      if (p.res_out) store4_dyn(p.res_out, base + c, p.ro_dtype, v[j]);
    }
  }
}

template <int VPL>  // values per lane (cols <= 64 * VPL)
__global__ __launch_bounds__(256) void add_norm_kernel(const NormParams p) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const int lane = threadIdx.x & 63;
  const long long base = row * p.cols;
  float v[VPL];
  float sum = 0.0f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    float s = 0.0f;
    if (c < p.cols) {
      s = load_dyn(p.x, base + c, p.x_dtype);
      if (p.res) s += load_dyn(p.res, base + c, p.res_dtype);
    }
    v[j] = s;
    sum += s;
  }
  float rstd, mean = 0.0f;
  if (p.is_rms) {
    float sq = 0.0f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) sq = fmaf(v[j], v[j], sq);
    rstd = rsqrtf(wave_sum(sq) / p.cols + p.eps);
  } else {
    mean = wave_sum(sum) / p.cols;
    float sq = 0.0f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + 64 * j;
      const float dv = (c < p.cols) ? v[j] - mean : 0.0f;
      sq = fmaf(dv, dv, sq);
    }
    rstd = rsqrtf(wave_sum(sq) / p.cols + p.eps);
  }
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c < p.cols) {
      float y = (v[j] - mean) * rstd * p.w[c];
      if (p.bias) y += p.bias[c];
      store_dyn(p.out, base + c, p.out_dtype, y);
      if (p.res_out) store_dyn(p.res_out, base + c, p.ro_dtype, v[j]);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Final add + norm fused with the pooling front half (videomamba.py:896-918 then :983-1062).
//
// Rows of one batch row are cut into a head (the CLS row, normalised but not pooled) and
// `groups` contiguous pooling groups (frames; for masked input the host passes the
// frame bounds of the gathered visible tokens).  A workgroup normalises up to kPoolRB
// rows of one group — writing them straight into the contiguous (batch, rows, cols)
// features, so the padded buffer needs no slice copy — and writes the fp32 column sum
// of the rounded outputs to part[b][g][slice].  pool_finish_kernel then sums the slices
// (and groups) in a fixed order, so the result is deterministic and independent of the
// launch geometry; the reference's means are of the rounded patch tokens as well.
constexpr int kPoolRB = 16;
constexpr bool kPoolFast = true;  // bf16 rows through norm_pool_rows_bf16_kernel

struct NormPoolParams {
  const void* x; const void* res; const float* w; const float* bias; void* out;
  long long in_bstride;             // elements between batch rows of x / res (padded L * cols)
  long long out_bstride;            // elements between batch rows of out
  int rows, cols; float eps; int is_rms, x_dtype, res_dtype, out_dtype;
  int rev_frame;                    // > 0: grouped rows read in reversed frame order
  int head, groups, group_rows;     // implicit equal groups when bounds == nullptr
  const int* bounds;                // (batch, groups + 1) row bounds or nullptr
  int slices;                       // kPoolRB-row slices per group
  float* part;                      // (batch, groups, slices, cols) or nullptr
};

template <int CPL>
__global__ __launch_bounds__(256) void norm_pool_rows_kernel(const NormPoolParams p) {
  extern __shared__ float red[];    // [4][cols]
  const int b = blockIdx.z, gy = blockIdx.y, s = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int lo, hi;
  if (gy == 0) {
    if (s) return;
    lo = 0; hi = p.head;
  } else if (p.bounds) {
    lo = p.bounds[(long long)b * (p.groups + 1) + gy - 1];
    hi = p.bounds[(long long)b * (p.groups + 1) + gy];
  } else {
    lo = p.head + (gy - 1) * p.group_rows;
    hi = lo + p.group_rows;
  }
  const int r0 = lo + s * kPoolRB;
  const int r1 = min(hi, r0 + kPoolRB);
  float acc[CPL][4];
#pragma unroll
  for (int j = 0; j < CPL; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = 0.0f;
  for (int r = r0 + wave; r < r1; r += 4) {
    int ri = r;  // input row: frame-order reversal of the grouped rows (BiMamba backward)
    if (p.rev_frame > 0 && r >= p.head) {
      const int x = r - p.head, F = p.rev_frame;
      ri = p.head + x + (p.rows - p.head - F) - 2 * F * (x / F);
    }
    const long long in = (long long)b * p.in_bstride + (long long)ri * p.cols;
    const long long on = (long long)b * p.out_bstride + (long long)r * p.cols;
    float v[CPL][4];
    float sum = 0.0f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane * 4 + 256 * j;
      if (c < p.cols) {
        load4_dyn(p.x, in + c, p.x_dtype, v[j]);
        if (p.res) {
          float q[4];
          load4_dyn(p.res, in + c, p.res_dtype, q);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[j][i] += q[i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[j][i] = 0.0f;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) sum += v[j][i];
    }
    float mean = 0.0f, sq = 0.0f;
    if (!p.is_rms) mean = wave_sum(sum) / p.cols;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const bool in_c = lane * 4 + 256 * j < p.cols;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dv = in_c ? v[j][i] - mean : 0.0f;
        sq = fmaf(dv, dv, sq);
      }
    }
    const float rstd = rsqrtf(wave_sum(sq) / p.cols + p.eps);
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane * 4 + 256 * j;
      if (c < p.cols) {
        const float4 w = *reinterpret_cast<const float4*>(p.w + c);
        const float wv[4] = {w.x, w.y, w.z, w.w};
        float y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          y[i] = (v[j][i] - mean) * rstd * wv[i];
          if (p.bias) y[i] += p.bias[c + i];
          if (p.out_dtype == VM_DTYPE_BF16) y[i] = to_f32(from_f32<bf16_t>(y[i]));
          acc[j][i] += y[i];
        }
        store4_dyn(p.out, on + c, p.out_dtype, y);
      }
    }
  }
  if (gy == 0 || !p.part) return;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane * 4 + 256 * j;
    if (c < p.cols)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wave * p.cols + c + i] = acc[j][i];
  }
  __syncthreads();
  float* dst = p.part + (((long long)b * p.groups + gy - 1) * p.slices + s) * p.cols;
  for (int c = threadIdx.x; c < p.cols; c += 256)
    dst[c] = ((red[c] + red[p.cols + c]) + red[2 * p.cols + c]) + red[3 * p.cols + c];
}

// norm_pool_rows_kernel for bf16 x / out with an fp32 (or no) residual: the same arithmetic
// in the same order, but every one of a wave's (at most kPoolRB / 4) rows is loaded by
// branch-free buffer loads before the first is reduced.  The dtype-generic loads sit behind
// branches whose joins make hipcc wait vmcnt(0): one dependent round trip per row and
// chunk, which set the B = 1 chunk's final norm at ~15 us.
template <int CPL>
__global__ __launch_bounds__(256) void norm_pool_rows_bf16_kernel(const NormPoolParams p) {
  extern __shared__ float red[];    // [4][cols]
  constexpr int RPW = kPoolRB / 4;  // rows per wave
  const int b = blockIdx.z, gy = blockIdx.y, s = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int lo, hi;
  if (gy == 0) {
    if (s) return;
    lo = 0; hi = p.head;
  } else if (p.bounds) {
    lo = p.bounds[(long long)b * (p.groups + 1) + gy - 1];
    hi = p.bounds[(long long)b * (p.groups + 1) + gy];
  } else {
    lo = p.head + (gy - 1) * p.group_rows;
    hi = lo + p.group_rows;
  }
  const int r0 = lo + s * kPoolRB;
  const int r1 = min(hi, r0 + kPoolRB);
  typedef __attribute__((__vector_size__(4 * sizeof(float)))) float v4f;
  auto off = [&](int j, int es) {
    int o = lane * 4 + 256 * j < p.cols ? (lane * 4 + 256 * j) * es : kNormOut;
    asm volatile("" : "+v"(o));
    return o;
  };
  uint32_t xq[RPW][CPL][2];
  v4f rq[RPW][CPL];
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int r = r0 + wave + 4 * k;
    const bool live = r < r1;
    int ri = live ? r : 0;
    if (p.rev_frame > 0 && ri >= p.head) {
      const int x = ri - p.head, F = p.rev_frame;
      ri = p.head + x + (p.rows - p.head - F) - 2 * F * (x / F);
    }
    const long long in = (long long)b * p.in_bstride + (long long)ri * p.cols;
    const auto xr = norm_row_rsrc(static_cast<const bf16_t*>(p.x) + in, live ? p.cols * 2 : 0);
    const auto rr = norm_row_rsrc(p.res ? static_cast<const float*>(p.res) + in : p.w,
                                  live && p.res ? p.cols * 4 : 0);
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const auto q = __builtin_amdgcn_raw_buffer_load_b64(xr, off(j, 2), 0, 0);
      xq[k][j][0] = q[0];
      xq[k][j][1] = q[1];
      rq[k][j] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rr, off(j, 4), 0, 0));
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // every row's loads in flight before any use
  float acc[CPL][4];
#pragma unroll
  for (int j = 0; j < CPL; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = 0.0f;
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int r = r0 + wave + 4 * k;
    if (r >= r1) break;
    const long long on = (long long)b * p.out_bstride + (long long)r * p.cols;
    float v[CPL][4];
    float sum = 0.0f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const bool in_c = lane * 4 + 256 * j < p.cols;
      v[j][0] = __uint_as_float(xq[k][j][0] << 16); v[j][1] = __uint_as_float(xq[k][j][0] & 0xffff0000u);
      v[j][2] = __uint_as_float(xq[k][j][1] << 16); v[j][3] = __uint_as_float(xq[k][j][1] & 0xffff0000u);
      if (p.res) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[j][i] += rq[k][j][i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (!in_c) v[j][i] = 0.0f;
        sum += v[j][i];
      }
    }
    float mean = 0.0f, sq = 0.0f;
    if (!p.is_rms) mean = wave_sum(sum) / p.cols;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const bool in_c = lane * 4 + 256 * j < p.cols;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dv = in_c ? v[j][i] - mean : 0.0f;
        sq = fmaf(dv, dv, sq);
      }
    }
    const float rstd = rsqrtf(wave_sum(sq) / p.cols + p.eps);
    const auto orr = norm_row_rsrc(static_cast<bf16_t*>(p.out) + on, p.cols * 2);
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane * 4 + 256 * j;
      if (c < p.cols) {
        const float4 w = *reinterpret_cast<const float4*>(p.w + c);
        const float wv[4] = {w.x, w.y, w.z, w.w};
        float y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          y[i] = (v[j][i] - mean) * rstd * wv[i];
          if (p.bias) y[i] += p.bias[c + i];
          y[i] = to_f32(from_f32<bf16_t>(y[i]));
          acc[j][i] += y[i];
        }
        typedef __attribute__((__vector_size__(2 * sizeof(int)))) int v2i;
        const v2i o2 = {static_cast<int>(static_cast<uint32_t>(from_f32<bf16_t>(y[0])) |
                                         (static_cast<uint32_t>(from_f32<bf16_t>(y[1])) << 16)),
                        static_cast<int>(static_cast<uint32_t>(from_f32<bf16_t>(y[2])) |
                                         (static_cast<uint32_t>(from_f32<bf16_t>(y[3])) << 16))};
        __builtin_amdgcn_raw_buffer_store_b64(o2, orr, c * 2, 0, 0);
      }
    }
  }
  if (gy == 0 || !p.part) return;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = lane * 4 + 256 * j;
    if (c < p.cols)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wave * p.cols + c + i] = acc[j][i];
  }
  __syncthreads();
  float* dst = p.part + (((long long)b * p.groups + gy - 1) * p.slices + s) * p.cols;
  for (int c = threadIdx.x; c < p.cols; c += 256)
    dst[c] = ((red[c] + red[p.cols + c]) + red[2 * p.cols + c]) + red[3 * p.cols + c];
}

// Pool finish: per (pooled row, batch row) sum the slices of its group(s) in order, take
// the mean (rounded to the output dtype like the reference's bf16 mean), add the CLS row
// for cls+avg, and apply the pool LayerNorm (fp32 statistics, eps of the module).
enum PoolMode { kPoolAvg = 0, kPoolClsAvg = 1, kPoolClsCatAvg = 2, kPoolCls = 3 };

struct PoolFinishParams {
  const float* part; int groups, slices, group_rows; const int* bounds;
  const void* cls; long long cls_bstride; int cls_dtype;
  int mode, keep_temporal;
  const float* lnw; const float* lnb; float ln_eps;
  void* xpool; int xp_dtype; int cols, prow;  // prow = pooled rows per batch row
};

__device__ __forceinline__ float block_sum1024(float v, float* sh) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.0f;
#pragma unroll
  for (int w = 0; w < 16; ++w) t += sh[w];
  return t;
}

// Slice sums: the (group, slice) rows of one pooled row are consecutive in the workspace.
// Thread t owns column quad t % nq and every P-th row from t / nq (P = 1024 / nq threads
// per quad, 4 loads in flight each); the P partial sums combine in LDS in a fixed order.
// (One dependent load per slice and column made this a 140 us tail at B = 1.)
__global__ __launch_bounds__(1024) void pool_finish_kernel(const PoolFinishParams p) {
  constexpr int kMaxPer = 2;  // cols <= 2048
  __shared__ float sh[16];
  __shared__ __attribute__((aligned(16))) float4 red[1024];
  const int q = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x;
  const bool rnd = p.xp_dtype == VM_DTYPE_BF16;
  auto group_count = [&](int g) -> int {
    return p.bounds ? p.bounds[(long long)b * (p.groups + 1) + g + 1] -
                          p.bounds[(long long)b * (p.groups + 1) + g]
                    : p.group_rows;
  };
  const bool use_cls = p.mode == kPoolCls || (p.mode == kPoolClsCatAvg && q == 0);
  const int aq = p.mode == kPoolClsCatAvg ? q - 1 : q;  // index of the averaged row
  const int g0 = p.keep_temporal ? aq : 0;
  const int g1 = p.keep_temporal ? aq + 1 : p.groups;
  int count = 0;
  if (!use_cls)
    for (int g = g0; g < g1; ++g) count += group_count(g);
  const int nq = p.cols >> 2;  // <= 512
  const int P = 1024 / nq;
  const int nrow = (g1 - g0) * p.slices;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int part = tid / nq, qd = tid % nq;
  if (!use_cls && part < P) {
    const float4* base = reinterpret_cast<const float4*>(
        p.part + ((long long)b * p.groups + g0) * p.slices * p.cols) + qd;
    int r = part;
    for (; r + 3 * P < nrow; r += 4 * P) {
      const float4 a0 = base[(long long)r * nq];
      const float4 a1 = base[(long long)(r + P) * nq];
      const float4 a2 = base[(long long)(r + 2 * P) * nq];
      const float4 a3 = base[(long long)(r + 3 * P) * nq];
      acc.x += a0.x; acc.y += a0.y; acc.z += a0.z; acc.w += a0.w;
      acc.x += a1.x; acc.y += a1.y; acc.z += a1.z; acc.w += a1.w;
      acc.x += a2.x; acc.y += a2.y; acc.z += a2.z; acc.w += a2.w;
      acc.x += a3.x; acc.y += a3.y; acc.z += a3.z; acc.w += a3.w;
    }
    for (; r < nrow; r += P) {
      const float4 a0 = base[(long long)r * nq];
      acc.x += a0.x; acc.y += a0.y; acc.z += a0.z; acc.w += a0.w;
    }
  }
  red[tid] = acc;
  __syncthreads();
  float v[kMaxPer];
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    const int c = tid + 1024 * k;
    float x = 0.0f;
    if (c < p.cols) {
      const float cl = p.cls ? load_dyn(p.cls, (long long)b * p.cls_bstride + c, p.cls_dtype)
                             : 0.0f;
      if (use_cls) {
        x = cl;
      } else {
        float sum = 0.0f;
        for (int pp = 0; pp < P; ++pp)
          sum += reinterpret_cast<const float*>(&red[pp * nq + (c >> 2)])[c & 3];
        x = sum / static_cast<float>(count);
        if (rnd) x = to_f32(from_f32<bf16_t>(x));
        if (p.mode == kPoolClsAvg) {
          x += cl;
          if (rnd) x = to_f32(from_f32<bf16_t>(x));
        }
      }
    }
    v[k] = x;
  }
  float s1 = 0.0f;
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) s1 += v[k];
  const float mean = block_sum1024(s1, sh) / p.cols;
  float s2 = 0.0f;
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    const float d = tid + 1024 * k < p.cols ? v[k] - mean : 0.0f;
    s2 = fmaf(d, d, s2);
  }
  const float rstd = rsqrtf(block_sum1024(s2, sh) / p.cols + p.ln_eps);
  const long long o = ((long long)b * p.prow + q) * p.cols;
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    const int c = tid + 1024 * k;
    if (c < p.cols) {
      float y = (v[k] - mean) * rstd;
      if (p.lnw) y *= p.lnw[c];
      if (p.lnb) y += p.lnb[c];
      store_dyn(p.xpool, o + c, p.xp_dtype, y);
    }
  }
}

}  // namespace vm

using namespace vm;

extern "C" long long vm_norm_pool_workspace_bytes(int batch, int groups, int max_group_rows,
                                                  int cols) {
  if (batch < 0 || groups < 0 || max_group_rows < 0 || cols < 0) return -1;
  const long long slices = (max_group_rows + kPoolRB - 1) / kPoolRB;
  return (long long)batch * groups * slices * cols * static_cast<long long>(sizeof(float));
}

extern "C" int vm_norm_pool_fwd(const void* x, int x_dtype, const void* residual, int res_dtype,
                                long long in_batch_stride, const float* weight, const float* bias,
                                float eps, int is_rms, void* out, int out_dtype,
                                long long out_batch_stride, int batch, int rows, int cols,
                                int head, int groups, int group_rows, const int* bounds,
                                int max_group_rows, int rev_frame, void* workspace,
                                long long workspace_bytes, vm_stream_t stream) {
  if (!x || !weight || !out) {
    vmhost::set_error("vm_norm_pool_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (batch < 0 || rows < 0 || cols < 4 || cols > 2048 || cols % 4 || head < 0 || head > rows ||
      groups < 1 || max_group_rows < 0 || in_batch_stride < (long long)rows * cols ||
      in_batch_stride % 4 || out_batch_stride < (long long)rows * cols || out_batch_stride % 4 ||
      rev_frame < 0 || (rev_frame > 0 && (rows - head) % rev_frame) ||
      !vmhost::dtype_ok(x_dtype) || !vmhost::dtype_ok(out_dtype) ||
      (residual && !vmhost::dtype_ok(res_dtype)) ||
      (!bounds && head + (long long)groups * group_rows != rows) ||
      (!bounds && group_rows != max_group_rows)) {
    vmhost::set_error("vm_norm_pool_fwd: bad shape/dtype (cols % 4 == 0, cols <= 2048; "
                      "implicit groups must tile rows after the head)");
    return VM_E_INVALID;
  }
  if (!vmhost::aligned16(x) || !vmhost::aligned16(out) || !vmhost::aligned16(weight) ||
      (residual && !vmhost::aligned16(residual))) {
    vmhost::set_error("vm_norm_pool_fwd: x, residual, out and weight must be 16-byte aligned");
    return VM_E_INVALID;
  }
  const long long need = vm_norm_pool_workspace_bytes(batch, groups, max_group_rows, cols);
  if (workspace && workspace_bytes < need) {
    vmhost::set_error("vm_norm_pool_fwd: workspace smaller than vm_norm_pool_workspace_bytes");
    return VM_E_INVALID;
  }
  if (batch == 0 || rows == 0) return VM_OK;
  NormPoolParams p{};
  p.x = x; p.res = residual; p.w = weight; p.bias = bias; p.out = out;
  p.in_bstride = in_batch_stride; p.out_bstride = out_batch_stride; p.rev_frame = rev_frame;
  p.rows = rows; p.cols = cols; p.eps = eps; p.is_rms = is_rms;
  p.x_dtype = x_dtype; p.res_dtype = res_dtype; p.out_dtype = out_dtype;
  p.head = head; p.groups = groups; p.group_rows = group_rows; p.bounds = bounds;
  p.slices = max_group_rows > 0 ? (max_group_rows + kPoolRB - 1) / kPoolRB : 1;
  p.part = static_cast<float*>(workspace);
  dim3 grid(p.slices, groups + 1, batch);
  const size_t lds = 4 * cols * sizeof(float);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int cpl = (cols + 255) / 256;
  const bool fast = kPoolFast && x_dtype == VM_DTYPE_BF16 && out_dtype == VM_DTYPE_BF16 &&
                    (!residual || res_dtype == VM_DTYPE_F32) && cpl <= 4 &&
                    (long long)(rows + 1) * cols * 4 < (1ll << 31);
  if (fast) {
    if (cpl <= 1) hipLaunchKernelGGL(norm_pool_rows_bf16_kernel<1>, grid, dim3(256), lds, s, p);
    else if (cpl <= 2) hipLaunchKernelGGL(norm_pool_rows_bf16_kernel<2>, grid, dim3(256), lds, s, p);
    else if (cpl <= 3) hipLaunchKernelGGL(norm_pool_rows_bf16_kernel<3>, grid, dim3(256), lds, s, p);
    else hipLaunchKernelGGL(norm_pool_rows_bf16_kernel<4>, grid, dim3(256), lds, s, p);
  } else if (cpl <= 1) hipLaunchKernelGGL(norm_pool_rows_kernel<1>, grid, dim3(256), lds, s, p);
  else if (cpl <= 2) hipLaunchKernelGGL(norm_pool_rows_kernel<2>, grid, dim3(256), lds, s, p);
  else if (cpl <= 4) hipLaunchKernelGGL(norm_pool_rows_kernel<4>, grid, dim3(256), lds, s, p);
  else hipLaunchKernelGGL(norm_pool_rows_kernel<8>, grid, dim3(256), lds, s, p);
  return vmhost::launch_status("vm_norm_pool_fwd");
}

extern "C" int vm_pool_finish_fwd(const void* workspace, int batch, int groups, int group_rows,
                                  const int* bounds, int max_group_rows, const void* cls,
                                  int cls_dtype, long long cls_batch_stride, int mode,
                                  int keep_temporal, const float* ln_weight, const float* ln_bias,
                                  float ln_eps, void* x_pool, int xp_dtype, int cols,
                                  vm_stream_t stream) {
  const bool needs_cls = mode == kPoolClsAvg || mode == kPoolClsCatAvg || mode == kPoolCls;
  const bool needs_avg = mode != kPoolCls;
  if (!x_pool || (needs_cls && !cls) || (needs_avg && !workspace)) {
    vmhost::set_error("vm_pool_finish_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (batch < 0 || groups < 1 || mode < 0 || mode > 3 || cols < 4 || cols > 2048 || cols % 4 ||
      max_group_rows < 1 || !vmhost::dtype_ok(xp_dtype) || (cls && !vmhost::dtype_ok(cls_dtype))) {
    vmhost::set_error("vm_pool_finish_fwd: bad mode/shape/dtype");
    return VM_E_INVALID;
  }
  if (batch == 0) return VM_OK;
  PoolFinishParams p{};
  p.part = static_cast<const float*>(workspace); p.groups = groups;
  p.slices = (max_group_rows + kPoolRB - 1) / kPoolRB; p.group_rows = group_rows;
  p.bounds = bounds; p.cls = cls; p.cls_bstride = cls_batch_stride; p.cls_dtype = cls_dtype;
  p.mode = mode; p.keep_temporal = keep_temporal; p.lnw = ln_weight; p.lnb = ln_bias;
  p.ln_eps = ln_eps; p.xpool = x_pool; p.xp_dtype = xp_dtype; p.cols = cols;
  const int navg = keep_temporal ? groups : 1;
  p.prow = mode == kPoolCls ? 1 : (mode == kPoolClsCatAvg ? 1 + navg : navg);
  hipLaunchKernelGGL(pool_finish_kernel, dim3(p.prow, batch), dim3(1024), 0,
                     static_cast<hipStream_t>(stream), p);
  return vmhost::launch_status("vm_pool_finish_fwd");
}

extern "C" int vm_add_norm_fwd(const void* x, int x_dtype, const void* residual, int res_dtype,
                               const float* weight, const float* bias, void* out, int out_dtype,
                               void* residual_out, int res_out_dtype, long long rows, int cols,
                               float eps, int is_rms, vm_stream_t stream) {
  if (!x || !weight || !out) {
    vmhost::set_error("vm_add_norm_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (rows < 0 || cols < 1 || cols > 64 * 32 || !vmhost::dtype_ok(x_dtype) ||
      !vmhost::dtype_ok(out_dtype) || (residual && !vmhost::dtype_ok(res_dtype)) ||
      (residual_out && !vmhost::dtype_ok(res_out_dtype))) {
    vmhost::set_error("vm_add_norm_fwd: bad shape/dtype (cols must be in [1, 2048])");
    return VM_E_INVALID;
  }
  if (rows == 0) return VM_OK;
  NormParams p{};
  p.x = x; p.res = residual; p.w = weight; p.bias = bias; p.out = out; p.res_out = residual_out;
  p.rows = rows; p.cols = cols; p.eps = eps; p.is_rms = is_rms;
  p.x_dtype = x_dtype; p.res_dtype = res_dtype; p.out_dtype = out_dtype; p.ro_dtype = res_out_dtype;
  dim3 grid(static_cast<unsigned>((rows + 3) / 4));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec = cols % 4 == 0 && vmhost::aligned16(x) && vmhost::aligned16(out) &&
                   vmhost::aligned16(weight) && (!residual || vmhost::aligned16(residual)) &&
                   (!residual_out || vmhost::aligned16(residual_out));
  if (vec && is_rms && !bias && x_dtype == VM_DTYPE_BF16 && out_dtype == VM_DTYPE_BF16 &&
      (!residual || res_dtype == VM_DTYPE_F32) && (!residual_out || res_out_dtype == VM_DTYPE_F32) &&
      cols <= 256 * 4) {
    const int cpl = (cols + 255) / 256;
    // streaming-chunk row counts: the stores write through (kSmallStoreWT)
    const bool wt = rows <= kSmallStoreRows;
#define VM_RMS_BF16(CPLV)                                                                   \
  if (residual && residual_out && wt)                                                       \
    hipLaunchKernelGGL((add_rms_bf16_kernel<CPLV, true, true, kSmallStoreWT>), grid, dim3(256), 0, s, p); \
  else if (residual && residual_out)                                                        \
    hipLaunchKernelGGL((add_rms_bf16_kernel<CPLV, true, true>), grid, dim3(256), 0, s, p);   \
  else if (residual)                                                                        \
    hipLaunchKernelGGL((add_rms_bf16_kernel<CPLV, true, false>), grid, dim3(256), 0, s, p);  \
  else if (residual_out)                                                                    \
    hipLaunchKernelGGL((add_rms_bf16_kernel<CPLV, false, true>), grid, dim3(256), 0, s, p);  \
  else                                                                                      \
    hipLaunchKernelGGL((add_rms_bf16_kernel<CPLV, false, false>), grid, dim3(256), 0, s, p);
    if (cpl <= 1) { VM_RMS_BF16(1) }
    else if (cpl <= 2) { VM_RMS_BF16(2) }
    else if (cpl <= 3) { VM_RMS_BF16(3) }
    else { VM_RMS_BF16(4) }
#undef VM_RMS_BF16
    return vmhost::launch_status("vm_add_norm_fwd");
  }
  if (vec) {
    const int cpl = (cols + 255) / 256;
    if (cpl <= 1) hipLaunchKernelGGL(add_norm_vec_kernel<1>, grid, dim3(256), 0, s, p);
    else if (cpl <= 2) hipLaunchKernelGGL(add_norm_vec_kernel<2>, grid, dim3(256), 0, s, p);
    else if (cpl <= 4) hipLaunchKernelGGL(add_norm_vec_kernel<4>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(add_norm_vec_kernel<8>, grid, dim3(256), 0, s, p);
    return vmhost::launch_status("vm_add_norm_fwd");
  }
  const int vpl = (cols + 63) / 64;
  if (vpl <= 4) hipLaunchKernelGGL(add_norm_kernel<4>, grid, dim3(256), 0, s, p);
  else if (vpl <= 8) hipLaunchKernelGGL(add_norm_kernel<8>, grid, dim3(256), 0, s, p);
  else if (vpl <= 16) hipLaunchKernelGGL(add_norm_kernel<16>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(add_norm_kernel<32>, grid, dim3(256), 0, s, p);
  return vmhost::launch_status("vm_add_norm_fwd");
}
