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

}  // namespace vm

using namespace vm;

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
