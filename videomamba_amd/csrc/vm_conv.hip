// Depthwise causal conv1d (+bias, SiLU) with streaming conv_state, and the one-token
// update.  Replaces causal-conv1d's causal_conv1d_fn / causal_conv1d_update as called
// at models/videomamba/mamba_simple.py:381-404 and :468-474.
//
// Layout: channel rows (b, d) with the sequence contiguous.  One thread produces 8
// consecutive outputs of one row from a 16-byte vector load plus the (width-1) halo;
// threads are laid out row-major over (row, 8-chunk) so a wave reads contiguous bytes.
// The virtual input is e[j] = x[j] (j >= 0), conv_state[width + j] (-width <= j < 0) or
// 0 without state; out[t] = bias + sum_i w[i] * e[t - width + 1 + i].

#include "vm_common.h"

namespace vm {

constexpr int kMaxW = 8;

struct ConvParams {
  const void* x; const float* w; const float* bias; const void* csi; void* cso; void* out;
  long long x_sb, x_sd, csi_sb, csi_sd, cso_sb, cso_sd, o_sb, o_sd;
  int batch, dim, seqlen, width, out_len, silu, csi_dtype, cso_dtype, vec;
};

template <typename T>
__device__ __forceinline__ float conv_elem(const ConvParams& p, const T* xr, long long csb, int j) {
  if (j >= 0) return to_f32(xr[j]);
  if (p.csi && j >= -p.width) return load_dyn(p.csi, csb + p.width + j, p.csi_dtype);
  return 0.0f;
}

template <typename T>
__global__ __launch_bounds__(256) void conv_fwd_kernel(const ConvParams p) {
  const int nchunk = max((p.out_len + 7) >> 3, 1);
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long rows = (long long)p.batch * p.dim;
  if (gid >= rows * nchunk) return;
  const int row = static_cast<int>(gid / nchunk);
  const int chunk = static_cast<int>(gid - (long long)row * nchunk);
  const int b = row / p.dim;
  const int d = row - b * p.dim;
  const int W = p.width;
  const T* xr = static_cast<const T*>(p.x) + b * p.x_sb + d * p.x_sd;
  T* orow = static_cast<T*>(p.out) + b * p.o_sb + d * p.o_sd;
  const long long csb = b * p.csi_sb + d * p.csi_sd;
  const int L = p.seqlen;
  const int t0 = chunk * 8;

  float wv[kMaxW];
#pragma unroll
  for (int i = 0; i < kMaxW; ++i) wv[i] = (i < W) ? p.w[d * W + i] : 0.0f;
  const float bias = p.bias ? p.bias[d] : 0.0f;

  // window e[t0 - (W-1) ... t0 + 7]; halo first
  float win[kMaxW - 1 + 8];
#pragma unroll
  for (int i = 0; i < kMaxW - 1; ++i) {
    const int j = t0 - (kMaxW - 1) + i;
    win[i] = (i >= kMaxW - W) ? conv_elem<T>(p, xr, csb, j) : 0.0f;
  }
  if (p.vec && t0 + 8 <= L) {
    float v[8];
    load8(xr + t0, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) win[kMaxW - 1 + i] = v[i];
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) win[kMaxW - 1 + i] = (t0 + i < L) ? to_f32(xr[t0 + i]) : 0.0f;
  }
  float o[8];
  // tap k of W multiplies e[t - W + 1 + k] = win[i + (kMaxW - W) + k]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float acc = bias;
#pragma unroll
    for (int k = 0; k < kMaxW; ++k)
      if (k < W) acc = fmaf(wv[k], win[i + (kMaxW - W) + k], acc);
    if (p.silu) acc = silu(acc);
    o[i] = (t0 + i < L) ? acc : 0.0f;
  }
  if (!p.out) {
  } else if (p.vec && t0 + 8 <= p.out_len) {
    store8(orow + t0, o);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (t0 + i < p.out_len) orow[t0 + i] = from_f32<T>(o[i]);
  }

  // new conv state: the last W entries of the virtual sequence
  if (p.cso && chunk == 0) {
    const long long ob = b * p.cso_sb + d * p.cso_sd;
    for (int i = 0; i < W; ++i)
      store_dyn(p.cso, ob + i, p.cso_dtype, conv_elem<T>(p, xr, csb, L - W + i));
  }
}

struct ConvStepParams {
  const void* x; void* cs; const float* w; const float* bias; void* out;
  long long x_sb, cs_sb, cs_sd, o_sb;
  int batch, dim, width, silu, cs_dtype;
};

template <typename T>
__global__ __launch_bounds__(256) void conv_update_kernel(const ConvStepParams p) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= p.batch * p.dim) return;
  const int b = gid / p.dim;
  const int d = gid - b * p.dim;
  const long long sb = b * p.cs_sb + d * p.cs_sd;
  const float x = to_f32(static_cast<const T*>(p.x)[b * p.x_sb + d]);
  float acc = p.bias ? p.bias[d] : 0.0f;
  for (int i = 0; i < p.width; ++i) {
    const float v = (i + 1 < p.width) ? load_dyn(p.cs, sb + i + 1, p.cs_dtype) : x;
    store_dyn(p.cs, sb + i, p.cs_dtype, v);
    acc = fmaf(p.w[d * p.width + i], load_dyn(p.cs, sb + i, p.cs_dtype), acc);
  }
  if (p.silu) acc = silu(acc);
  static_cast<T*>(p.out)[b * p.o_sb + d] = from_f32<T>(acc);
}

}  // namespace vm

using namespace vm;

extern "C" int vm_causal_conv1d_fwd(const void* x, long long x_sb, long long x_sd,
                                    const float* weight, const float* bias,
                                    const void* cs_in, int cs_in_dtype, long long csi_sb, long long csi_sd,
                                    void* cs_out, int cs_out_dtype, long long cso_sb, long long cso_sd,
                                    void* out, long long o_sb, long long o_sd, int out_len,
                                    int batch, int dim, int seqlen, int width, int silu, int dtype,
                                    vm_stream_t stream) {
  if (!x || !weight || !out) {
    vmhost::set_error("vm_causal_conv1d_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (batch < 0 || dim < 0 || seqlen < 0 || out_len < seqlen || width < 1 || width > kMaxW ||
      !vmhost::dtype_ok(dtype) || (cs_in && !vmhost::dtype_ok(cs_in_dtype)) ||
      (cs_out && !vmhost::dtype_ok(cs_out_dtype))) {
    vmhost::set_error("vm_causal_conv1d_fwd: bad shape/dtype (width must be in [1, %d], "
                      "out_len >= seqlen)", kMaxW);
    return VM_E_INVALID;
  }
  if (cs_out && cs_in == cs_out) {
    vmhost::set_error("vm_causal_conv1d_fwd: conv_state_out must not alias conv_state_in");
    return VM_E_INVALID;
  }
  if (batch == 0 || dim == 0) return VM_OK;
  ConvParams p{};
  p.x = x; p.w = weight; p.bias = bias; p.csi = cs_in; p.cso = cs_out; p.out = out;
  p.x_sb = x_sb; p.x_sd = x_sd; p.csi_sb = csi_sb; p.csi_sd = csi_sd;
  p.cso_sb = cso_sb; p.cso_sd = cso_sd; p.o_sb = o_sb; p.o_sd = o_sd;
  p.batch = batch; p.dim = dim; p.seqlen = seqlen; p.width = width; p.out_len = out_len;
  p.silu = silu; p.csi_dtype = cs_in_dtype; p.cso_dtype = cs_out_dtype;
  const long long m = dtype == VM_DTYPE_BF16 ? 8 : 4;
  p.vec = vmhost::aligned16(x) && vmhost::aligned16(out) && x_sb % m == 0 && x_sd % m == 0 &&
          o_sb % m == 0 && o_sd % m == 0;
  const int nchunk = out_len > 0 ? (out_len + 7) / 8 : 1;
  const long long total = 1LL * batch * dim * nchunk;
  dim3 grid(static_cast<unsigned>((total + 255) / 256));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (dtype == VM_DTYPE_BF16) hipLaunchKernelGGL(conv_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(conv_fwd_kernel<float>, grid, dim3(256), 0, s, p);
  return vmhost::launch_status("vm_causal_conv1d_fwd");
}

extern "C" int vm_causal_conv1d_update(const void* x, long long x_sb, void* conv_state, int cs_dtype,
                                       long long cs_sb, long long cs_sd, const float* weight,
                                       const float* bias, void* out, long long o_sb,
                                       int batch, int dim, int width, int silu, int dtype,
                                       vm_stream_t stream) {
  if (!x || !conv_state || !weight || !out) {
    vmhost::set_error("vm_causal_conv1d_update: null required pointer");
    return VM_E_INVALID;
  }
  if (batch < 0 || dim < 0 || width < 1 || width > kMaxW || !vmhost::dtype_ok(dtype) ||
      !vmhost::dtype_ok(cs_dtype)) {
    vmhost::set_error("vm_causal_conv1d_update: bad shape/dtype");
    return VM_E_INVALID;
  }
  if (batch == 0 || dim == 0) return VM_OK;
  ConvStepParams p{};
  p.x = x; p.cs = conv_state; p.w = weight; p.bias = bias; p.out = out;
  p.x_sb = x_sb; p.cs_sb = cs_sb; p.cs_sd = cs_sd; p.o_sb = o_sb;
  p.batch = batch; p.dim = dim; p.width = width; p.silu = silu; p.cs_dtype = cs_dtype;
  dim3 grid((batch * dim + 255) / 256);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (dtype == VM_DTYPE_BF16) hipLaunchKernelGGL(conv_update_kernel<bf16_t>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(conv_update_kernel<float>, grid, dim3(256), 0, s, p);
  return vmhost::launch_status("vm_causal_conv1d_update");
}
