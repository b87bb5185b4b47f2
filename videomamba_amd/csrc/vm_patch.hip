// Tubelet patch embed: Conv3d with kernel = stride = (kt, P, P) as an implicit GEMM,
// fused with the bias, the spatial and the temporal positional embedding adds.
// Replaces PatchEmbed.forward + the pos-embed adds of models/videomamba/videomamba.py
// (:359-368, :806-815).  The reference materialises the conv output, the +spatial and
// the +temporal sums in the model dtype; the epilogue rounds at the same three points.
//
//   tok[m, n] = sum_k video[gather(m, k)] * weight[n, k],  m = (b, t, gh, gw),
//   k = (ci, kt_, kh, kw) in the weight's (C, Cin, kt, P, P) order.
//
// bf16 path: v_mfma_f32_16x16x32_bf16, operands loaded straight into fragments (with
// P % 8 == 0 the 8 consecutive k of a lane are 8 contiguous pixels of one patch row:
// one 16-byte load), block tile 64 tokens x 64 channels (2x2 waves of 32x32).
// Other shapes / fp32: a scalar implicit-GEMM kernel (same math, fp32 accumulate).

#include "vm_common.h"

namespace vm {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct PatchParams {
  const void* video; const void* w; const float* bias; const void* spos; const void* tpos;
  void* out;
  long long out_sb;
  int row0, batch, cin, frames, height, width, kt, patch, embed;
  int tt, gh, gw, K, M;  // derived: temporal tokens, grid, reduction length, tokens
};

template <typename T>
__device__ __forceinline__ void patch_store(const PatchParams& p, int m, int n, float acc) {
  const int hw = p.gh * p.gw;
  const int per_b = p.tt * hw;
  const int b = m / per_b;
  const int rem = m - b * per_b;
  const int t = rem / hw;
  const int s = rem - t * hw;
  float v = round_to<T>(acc + p.bias[n]);
  v = round_to<T>(v + to_f32(static_cast<const T*>(p.spos)[(long long)s * p.embed + n]));
  v = v + to_f32(static_cast<const T*>(p.tpos)[(long long)t * p.embed + n]);
  static_cast<T*>(p.out)[b * p.out_sb + (long long)(p.row0 + rem) * p.embed + n] = from_f32<T>(v);
}

__device__ __forceinline__ long long token_base(const PatchParams& p, int m) {
  const int hw = p.gh * p.gw;
  const int per_b = p.tt * hw;
  const int b = m / per_b;
  const int rem = m - b * per_b;
  const int t = rem / hw;
  const int s = rem - t * hw;
  const int gy = s / p.gw;
  const int gx = s - gy * p.gw;
  return ((long long)b * p.cin * p.frames + (long long)t * p.kt) * p.height * p.width +
         (long long)gy * p.patch * p.width + (long long)gx * p.patch;
}

__device__ __forceinline__ long long k_offset(const PatchParams& p, int k) {
  const int pp = p.patch * p.patch;
  const int per_c = p.kt * pp;
  const int ci = k / per_c;
  const int r1 = k - ci * per_c;
  const int kz = r1 / pp;
  const int r2 = r1 - kz * pp;
  const int ky = r2 / p.patch;
  const int kx = r2 - ky * p.patch;
  return ((long long)ci * p.frames + kz) * p.height * p.width + (long long)ky * p.width + kx;
}

__global__ __launch_bounds__(256) void patch_mfma_kernel(const PatchParams p) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 64 + (wave & 1) * 32;
  const int n0 = blockIdx.y * 64 + (wave >> 1) * 32;
  const int r = lane & 15;
  const int kg = lane >> 4;
  const bf16_t* vid = static_cast<const bf16_t*>(p.video);
  const bf16_t* wt = static_cast<const bf16_t*>(p.w);

  long long abase[2];
  bool mval[2], nval[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + i * 16 + r;
    mval[i] = m < p.M;
    abase[i] = token_base(p, mval[i] ? m : 0);
    nval[i] = (n0 + i * 16 + r) < p.embed;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16x8 zero = {};
  for (int kk = 0; kk < p.K; kk += 32) {
    const int k = kk + kg * 8;
    const bool kval = k < p.K;
    const long long koff = k_offset(p, kval ? k : 0);
    bf16x8 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      a[i] = (kval && mval[i]) ? *reinterpret_cast<const bf16x8*>(vid + abase[i] + koff) : zero;
      const int n = n0 + i * 16 + r;
      b[i] = (kval && nval[i]) ? *reinterpret_cast<const bf16x8*>(wt + (long long)n * p.K + k) : zero;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + i * 16 + kg * 4 + e;
        const int n = n0 + j * 16 + r;
        if (m < p.M && n < p.embed) patch_store<bf16_t>(p, m, n, acc[i][j][e]);
      }
}

template <typename T>
__global__ __launch_bounds__(256) void patch_generic_kernel(const PatchParams p) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)p.M * p.embed) return;
  const int m = static_cast<int>(gid / p.embed);
  const int n = static_cast<int>(gid - (long long)m * p.embed);
  const T* vid = static_cast<const T*>(p.video);
  const T* wt = static_cast<const T*>(p.w) + (long long)n * p.K;
  const long long base = token_base(p, m);
  float acc = 0.0f;
  for (int k = 0; k < p.K; ++k) acc = fmaf(to_f32(vid[base + k_offset(p, k)]), to_f32(wt[k]), acc);
  patch_store<T>(p, m, n, acc);
}

}  // namespace vm

using namespace vm;

extern "C" int vm_patch_embed_fwd(const void* video, const void* weight, const float* bias,
                                  const void* spos, const void* tpos, void* out, long long out_sb,
                                  int row0, int batch, int cin, int frames, int height, int width,
                                  int kt, int patch, int embed, int dtype, vm_stream_t stream) {
  if (!video || !weight || !bias || !spos || !tpos || !out) {
    vmhost::set_error("vm_patch_embed_fwd: null required pointer");
    return VM_E_INVALID;
  }
  if (batch < 0 || cin < 1 || kt < 1 || patch < 1 || embed < 1 || frames % kt != 0 ||
      height < patch || width < patch || !vmhost::dtype_ok(dtype)) {
    vmhost::set_error("vm_patch_embed_fwd: bad shape/dtype");
    return VM_E_INVALID;
  }
  PatchParams p{};
  p.video = video; p.w = weight; p.bias = bias; p.spos = spos; p.tpos = tpos; p.out = out;
  p.out_sb = out_sb; p.row0 = row0; p.batch = batch; p.cin = cin; p.frames = frames;
  p.height = height; p.width = width; p.kt = kt; p.patch = patch; p.embed = embed;
  p.tt = frames / kt; p.gh = height / patch; p.gw = width / patch;
  p.K = cin * kt * patch * patch;
  const long long M = 1LL * batch * p.tt * p.gh * p.gw;
  if (M == 0) return VM_OK;
  if (M > 0x7fffffffLL) {
    vmhost::set_error("vm_patch_embed_fwd: too many tokens");
    return VM_E_INVALID;
  }
  p.M = static_cast<int>(M);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool mfma_ok = dtype == VM_DTYPE_BF16 && patch % 8 == 0 && width % 8 == 0 &&
                       p.K % 8 == 0 && vmhost::aligned16(video) && vmhost::aligned16(weight);
  if (mfma_ok) {
    dim3 grid((p.M + 63) / 64, (embed + 63) / 64);
    hipLaunchKernelGGL(patch_mfma_kernel, grid, dim3(256), 0, s, p);
  } else {
    const long long total = M * embed;
    dim3 grid(static_cast<unsigned>((total + 255) / 256));
    if (dtype == VM_DTYPE_BF16) hipLaunchKernelGGL(patch_generic_kernel<bf16_t>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(patch_generic_kernel<float>, grid, dim3(256), 0, s, p);
  }
  return vmhost::launch_status("vm_patch_embed_fwd");
}
