// Depthwise causal conv1d (+bias, SiLU) with streaming conv_state, and the one-token
// update.  Replaces causal-conv1d's causal_conv1d_fn / causal_conv1d_update as called
// at models/videomamba/mamba_simple.py:381-404 and :468-474.
//
// Two layouts, chosen by stride:
//  * channel-major (step stride 1): one thread produces 8 consecutive outputs of one
//    (b, d) row from a 16-byte vector load plus the (width-1) halo;
//  * token-major (channel stride 1, the large-batch mixer layout): one thread owns CPT
//    adjacent channels (a 16-byte row segment), walks a 64-step time tile and keeps the
//    (width-1)-row history in registers, so every input byte is read once per tile and a
//    wave reads 1 KB contiguous per step.
// The virtual input is e[j] = x[j] (j >= 0), conv_state[width + j] (-width <= j < 0) or
// 0 without state; out[t] = bias + sum_i w[i] * e[t - width + 1 + i].

#include "vm_common.h"

namespace vm {

constexpr int kMaxW = 8;

struct ConvParams {
  const void* x; const float* w; const float* bias; const void* csi; void* cso; void* out;
  long long x_sb, x_sd, csi_sb, csi_sd, cso_sb, cso_sd, o_sb, o_sd;
  long long x_sl, o_sl;
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

// ------------------------------------------------------------------ token-major
constexpr int kConvTT = 64;  // steps per time tile

template <typename T, int CPT>
__device__ __forceinline__ void load_cpt(const T* p, float (&v)[CPT]) {
  if constexpr (sizeof(T) == 2 && CPT == 8) {
    load8(p, v);
  } else if constexpr (sizeof(T) == 2 && CPT == 4) {
    const uint2 q = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
    v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
  } else if constexpr (sizeof(T) == 4 && CPT == 4) {
    const float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
#pragma unroll
    for (int c = 0; c < CPT; ++c) v[c] = to_f32(p[c]);
  }
}
template <typename T, int CPT>
__device__ __forceinline__ void store_cpt(T* p, const float (&v)[CPT]) {
  if constexpr (sizeof(T) == 2 && CPT == 8) {
    store8(p, v);
  } else if constexpr (sizeof(T) == 2 && CPT == 4) {
    uint2 q;
    q.x = static_cast<uint32_t>(from_f32<bf16_t>(v[0])) | (static_cast<uint32_t>(from_f32<bf16_t>(v[1])) << 16);
    q.y = static_cast<uint32_t>(from_f32<bf16_t>(v[2])) | (static_cast<uint32_t>(from_f32<bf16_t>(v[3])) << 16);
    *reinterpret_cast<uint2*>(p) = q;
  } else if constexpr (sizeof(T) == 4 && CPT == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int c = 0; c < CPT; ++c) p[c] = from_f32<T>(v[c]);
  }
}

// thread -> (b, channels d0..d0+CPT-1, steps [t0, t0+kConvTT)); WM >= width taps, the
// missing leading taps are zero.
template <typename T, int CPT, int WM>
__global__ __launch_bounds__(64) void conv_tm_kernel(const ConvParams p) {
  const int d0 = (blockIdx.x * 64 + threadIdx.x) * CPT;
  if (d0 >= p.dim) return;
  const int b = blockIdx.z;
  const int t0 = blockIdx.y * kConvTT;
  const int W = p.width, L = p.seqlen;
  const T* __restrict__ xb = static_cast<const T*>(p.x) + b * p.x_sb + d0;
  T* __restrict__ ob = static_cast<T*>(p.out) + b * p.o_sb + d0;
  float w[WM][CPT], bias[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int d = d0 + c < p.dim ? d0 + c : p.dim - 1;
#pragma unroll
    for (int k = 0; k < WM; ++k) {  // right-aligned taps: w[WM-1] multiplies e[t]
      const int i = k - (WM - W);
      w[k][c] = i >= 0 ? p.w[d * W + i] : 0.0f;
    }
    bias[c] = p.bias ? p.bias[d] : 0.0f;
  }
  auto elem_row = [&](int j, float (&v)[CPT]) {  // e[j] for the thread's channels
    if (j >= 0 && j < L) {
      load_cpt<T, CPT>(xb + j * p.x_sl, v);
    } else {
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const int d = d0 + c < p.dim ? d0 + c : p.dim - 1;
        v[c] = (j < 0 && p.csi && j >= -W)
                   ? load_dyn(p.csi, b * p.csi_sb + d * p.csi_sd + W + j, p.csi_dtype)
                   : 0.0f;
      }
    }
  };
  float hist[WM][CPT];  // hist[k] = e[t - (WM-1) + k], k = WM-1 is the current row
#pragma unroll
  for (int k = 0; k < WM - 1; ++k) elem_row(t0 - (WM - 1) + k, hist[k]);
  const int t_end = min(t0 + kConvTT, p.out_len);
  for (int tb = t0; tb < t_end; tb += 8) {
    float rows[8][CPT];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = tb + i;
      if (t < L) load_cpt<T, CPT>(xb + t * p.x_sl, rows[i]);
      else {
#pragma unroll
        for (int c = 0; c < CPT; ++c) rows[i][c] = 0.0f;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = tb + i;
#pragma unroll
      for (int c = 0; c < CPT; ++c) hist[WM - 1][c] = rows[i][c];
      float o[CPT];
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        float acc = bias[c];
#pragma unroll
        for (int k = 0; k < WM; ++k) acc = fmaf(w[k][c], hist[k][c], acc);
        if (p.silu) acc = silu(acc);
        o[c] = t < L ? acc : 0.0f;
      }
      if (t < t_end) store_cpt<T, CPT>(ob + t * p.o_sl, o);
#pragma unroll
      for (int k = 0; k < WM - 1; ++k)
#pragma unroll
        for (int c = 0; c < CPT; ++c) hist[k][c] = hist[k + 1][c];
    }
  }
  // new conv state (last W raw inputs) from the tile holding the last step
  const int tl = L > 0 ? L - 1 : 0;
  if (p.cso && tl >= t0 && tl < t0 + kConvTT) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int d = d0 + c;
      if (d >= p.dim) break;
      const long long sb = b * p.cso_sb + d * p.cso_sd;
      for (int i = 0; i < W; ++i) {
        const int j = L - W + i;
        float v = 0.0f;
        if (j >= 0) v = to_f32(static_cast<const T*>(p.x)[b * p.x_sb + d + j * p.x_sl]);
        else if (p.csi) v = load_dyn(p.csi, b * p.csi_sb + d * p.csi_sd + W + j, p.csi_dtype);
        store_dyn(p.cso, sb + i, p.cso_dtype, v);
      }
    }
  }
}

template <typename T, int CPT>
static void launch_conv_tm(const ConvParams& p, hipStream_t s) {
  const int groups = (p.dim + CPT - 1) / CPT;
  const int tiles = p.out_len > 0 ? (p.out_len + kConvTT - 1) / kConvTT : 1;
  dim3 grid((groups + 63) / 64, tiles, p.batch);
  if (p.width <= 4) hipLaunchKernelGGL((conv_tm_kernel<T, CPT, 4>), grid, dim3(64), 0, s, p);
  else hipLaunchKernelGGL((conv_tm_kernel<T, CPT, kMaxW>), grid, dim3(64), 0, s, p);
}

template <typename T>
static void dispatch_conv_tm(const ConvParams& p, hipStream_t s) {
  const long long es = sizeof(T);
  auto ok = [&](int cpt) {
    const long long bytes = cpt * es;
    return p.dim % cpt == 0 && reinterpret_cast<uintptr_t>(p.x) % bytes == 0 &&
           reinterpret_cast<uintptr_t>(p.out) % bytes == 0 && (p.x_sb * es) % bytes == 0 &&
           (p.x_sl * es) % bytes == 0 && (p.o_sb * es) % bytes == 0 && (p.o_sl * es) % bytes == 0;
  };
  if (sizeof(T) == 2 && ok(8)) launch_conv_tm<T, 8>(p, s);
  else if (ok(4)) launch_conv_tm<T, 4>(p, s);
  else launch_conv_tm<T, 1>(p, s);
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

extern "C" int vm_causal_conv1d_fwd(const void* x, long long x_sb, long long x_sd, long long x_sl,
                                    const float* weight, const float* bias,
                                    const void* cs_in, int cs_in_dtype, long long csi_sb, long long csi_sd,
                                    void* cs_out, int cs_out_dtype, long long cso_sb, long long cso_sd,
                                    void* out, long long o_sb, long long o_sd, long long o_sl,
                                    int out_len, int batch, int dim, int seqlen, int width, int silu,
                                    int dtype, vm_stream_t stream) {
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
  p.x_sl = x_sl; p.o_sl = o_sl;
  p.batch = batch; p.dim = dim; p.seqlen = seqlen; p.width = width; p.out_len = out_len;
  p.silu = silu; p.csi_dtype = cs_in_dtype; p.cso_dtype = cs_out_dtype;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (x_sd == 1 && o_sd == 1 && dim > 1) {  // token-major
    if (dtype == VM_DTYPE_BF16) dispatch_conv_tm<bf16_t>(p, s);
    else dispatch_conv_tm<float>(p, s);
    return vmhost::launch_status("vm_causal_conv1d_fwd");
  }
  if (x_sl != 1 || o_sl != 1) {
    vmhost::set_error("vm_causal_conv1d_fwd: x/out need a unit channel stride or a unit step "
                      "stride");
    return VM_E_INVALID;
  }
  const long long m = dtype == VM_DTYPE_BF16 ? 8 : 4;
  p.vec = vmhost::aligned16(x) && vmhost::aligned16(out) && x_sb % m == 0 && x_sd % m == 0 &&
          o_sb % m == 0 && o_sd % m == 0;
  const int nchunk = out_len > 0 ? (out_len + 7) / 8 : 1;
  const long long total = 1LL * batch * dim * nchunk;
  dim3 grid(static_cast<unsigned>((total + 255) / 256));
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
