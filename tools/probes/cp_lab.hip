// conv_proj lab (tools only): prices the pieces of vm::conv_proj_kernel and vm::dt_proj_kernel
// at the bench shape (B clips x Lp=3144 rows, D=1152, R=36, e=68 -> e_pad 80, bf16) by
// timing the library kernel with pieces removed (EXP bits, see vm_conv_proj.hip), plus a
// copy kernel with the same row pattern (x = first D of each 2D-wide xz row -> u rows).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I videomamba_amd/csrc \
//         tools/probes/cp_lab.hip -o tools/probes/cp_lab
//   ./tools/probes/cp_lab [B]
#include "../../videomamba_amd/csrc/vm_conv_proj.hip"

#include <stdio.h>
#include <string.h>
#include <vector>

// host helpers the included library source refers to (defined in vm_api.hip there)
namespace vmhost {
void set_error(const char*, ...) {}
int launch_status(const char*) { return hipGetLastError() == hipSuccess ? 0 : 1; }
}  // namespace vmhost

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

// x rows (pitch 2D) -> u rows (pitch D), 16 B per lane
__global__ __launch_bounds__(256) void copy_rows(const uint4* __restrict__ x, uint4* __restrict__ u,
                                                 long long rows, int dq) {
  const long long n = rows * dq;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long r = i / dq, q = i - r * dq;
    u[i] = x[r * 2 * dq + q];
  }
}

// row-structured copies, no division: one 16-B piece per lane, rows of dq pieces;
// in_pitch / out_pitch in pieces.  MODE 0 copy, 1 read only (xor-reduce, one store per
// thread), 2 write only.
template <int MODE, int DQ>
__global__ __launch_bounds__(256) void rows_kernel(const uint4* __restrict__ x, uint4* __restrict__ u,
                                                   int rows, int in_pitch, int out_pitch) {
  const unsigned n = static_cast<unsigned>(rows) * DQ;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    const unsigned r = i / DQ, q = i - r * DQ;  // constant divisor: mul + shift
    if (MODE == 2) {
      u[(long long)r * out_pitch + q] = make_uint4(r, q, 0, 0);
    } else {
      const uint4 v = x[(long long)r * in_pitch + q];
      if (MODE == 0) u[(long long)r * out_pitch + q] = v;
      else { acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w; }
    }
  }
  if (MODE == 1 && (acc.x == 0x12345678u)) u[threadIdx.x] = acc;
}

// write-only variants over n bytes: W = bytes per lane per store (4, 8, 16); NT = 1
// nontemporal builtin, 2..5 buffer-store aux = NT - 2
template <int W, int NT>
__global__ __launch_bounds__(256) void wr_kernel(uint8_t* __restrict__ u, unsigned long long n) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(u, 0, 0x7fffffff, 0x00020000);
  for (unsigned long long i = (blockIdx.x * 256ull + threadIdx.x) * W; i < n;
       i += (unsigned long long)gridDim.x * 256 * W) {
    if constexpr (W == 16) {
      const uint4 v = make_uint4((uint32_t)i, 1, 2, 3);
      typedef __attribute__((ext_vector_type(4))) unsigned int v4u;
      if constexpr (NT == 1) __builtin_nontemporal_store(v4u{(uint32_t)i, 1, 2, 3}, reinterpret_cast<v4u*>(u + i));
      else if constexpr (NT >= 2) {
        // buffer stores need 32-bit offsets: per-block base instead
        typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
        const unsigned long long base = i & ~0xfffffffull;
        const auto rb = __builtin_amdgcn_make_buffer_rsrc(u + base, 0, 0x7fffffff, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{(uint32_t)i, 1, 2, 3}, rb, (int)(i - base), 0, NT - 2);
      } else *reinterpret_cast<uint4*>(u + i) = v;
    } else if constexpr (W == 8) {
      const uint2 v = make_uint2((uint32_t)i, 1);
      typedef __attribute__((ext_vector_type(2))) unsigned int v2u;
      if constexpr (NT == 1) __builtin_nontemporal_store(v2u{(uint32_t)i, 1}, reinterpret_cast<v2u*>(u + i));
      else *reinterpret_cast<uint2*>(u + i) = v;
    } else {
      if constexpr (NT == 1) __builtin_nontemporal_store((uint32_t)i, reinterpret_cast<uint32_t*>(u + i));
      else *reinterpret_cast<uint32_t*>(u + i) = (uint32_t)i;
    }
  }
  (void)rs;
}

// conv_proj's traffic shape without its math: a workgroup owns 64 rows and sweeps 64-channel
// chunks (CHUNKED: thread = 8 channels x 2 rows per chunk, 128-B segments of 64 rows), or
// walks its 64 rows in row order (full 2304-B rows, 16 B per lane).
template <bool CHUNKED>
__global__ __launch_bounds__(256) void shape_copy(const bf16_t* __restrict__ xz, bf16_t* __restrict__ u,
                                                  int rows, int D) {
  const int tid = threadIdx.x, row0 = blockIdx.x * 64;
  if (CHUNKED) {
    const int cg = tid & 7, tg = tid >> 3;
    const int ra = row0 + 2 * tg;
    for (int c0 = 0; c0 < D; c0 += 64) {
      const int c = c0 + cg * 8;
      if (ra < rows) {
        const uint4 a = *reinterpret_cast<const uint4*>(xz + (long long)ra * 2 * D + c);
        const uint4 b = *reinterpret_cast<const uint4*>(xz + (long long)(ra + 1) * 2 * D + c);
        *reinterpret_cast<uint4*>(u + (long long)ra * D + c) = a;
        *reinterpret_cast<uint4*>(u + (long long)(ra + 1) * D + c) = b;
      }
    }
  } else {
    const int dq = D / 8;
    for (int i = tid; i < 64 * dq; i += 256) {
      const int lr = i / dq, q = i - lr * dq;
      const int r = row0 + lr;
      if (r < rows)
        *reinterpret_cast<uint4*>(u + (long long)r * D + q * 8) =
            *reinterpret_cast<const uint4*>(xz + (long long)r * 2 * D + q * 8);
    }
  }
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 336;
  const int D = 1152, L = 3137, Lp = 3144, R = 36, E = 68, EP = 80, RP = 64, W = 4;
  const long long rows = (long long)B * Lp;
  std::vector<uint16_t> h(rows * 2 * D);
  uint32_t s = 12345;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = 0x3c00 + ((s >> 16) & 0x3ff) - 0x200 * ((s >> 27) & 1); }
  bf16_t *xz, *wx, *wdt, *u, *xd, *dt;
  float *cw, *cb;
  CK(hipMalloc(&xz, rows * 2 * D * 2)); CK(hipMalloc(&u, rows * D * 2));
  CK(hipMalloc(&dt, rows * D * 2)); CK(hipMalloc(&xd, rows * E * 2));
  CK(hipMalloc(&wx, EP * D * 2)); CK(hipMalloc(&wdt, D * RP * 2));
  CK(hipMalloc(&cw, D * W * 4)); CK(hipMalloc(&cb, D * 4));
  CK(hipMemcpy(xz, h.data(), rows * 2 * D * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(wx, h.data(), EP * D * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(wdt, h.data() + 7, D * RP * 2, hipMemcpyHostToDevice));
  std::vector<float> f(D * W, 0.1f);
  CK(hipMemcpy(cw, f.data(), D * W * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(cb, f.data(), D * 4, hipMemcpyHostToDevice));

  ConvProjParams p{};
  p.xz = xz; p.cw = cw; p.cb = cb; p.csi = nullptr; p.cso = nullptr; p.wx = wx; p.wdt = wdt;
  p.u = u; p.xdbl = xd; p.dt = dt;
  p.xz_sb = (long long)Lp * 2 * D; p.xz_sl = 2 * D; p.u_sb = (long long)Lp * D; p.u_sl = D;
  p.xd_sb = (long long)Lp * E; p.xd_sl = E; p.dt_sb = (long long)Lp * D; p.dt_sl = D;
  p.batch = B; p.dim = D; p.seqlen = L; p.lp = Lp; p.rows = (int)rows; p.e = E; p.e_pad = EP;
  p.r = R; p.r_pad = RP; p.width = W;
  const dim3 grid((p.rows + kCPTok - 1) / kCPTok);
  const size_t lds = (size_t)D * 5 * sizeof(float);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    printf("%-34s B=%d %9.1f us  %7.1f GB/s\n", name, B, us, bytes / us * 1e-3);
    fflush(stdout);
  };
  const double cp_bytes = (double)rows * (2.0 * D * 2 + E * 2);  // x in, u out, x_dbl out
  if (argc > 2 && strcmp(argv[2], "only") == 0) {  // PMC runs: the library kernels alone
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL((conv_proj_kernel<false, 5, 0>), grid, dim3(256), lds, 0, p);
      hipLaunchKernelGGL((dt_proj_kernel<16, 4>), grid, dim3(256), 0, 0, p);
    }
    CK(hipDeviceSynchronize());
    return 0;
  }
  const double dt_bytes = (double)rows * (R * 2 + D * 2);
  timeit("copy x->u (same rows)", rows * 2.0 * D * 2, [&] {
    hipLaunchKernelGGL(copy_rows, dim3(4096), dim3(256), 0, 0, (const uint4*)xz, (uint4*)u, rows, D / 8);
  });
  const int dq = D / 8;  // 144 pieces per x row
  const int g2 = 256 * 16;
  timeit("rows copy, x half-rows -> u", rows * 2.0 * D * 2, [&] {
    hipLaunchKernelGGL((rows_kernel<0, 144>), dim3(g2), dim3(256), 0, 0, (const uint4*)xz, (uint4*)u, (int)rows, 2 * dq, dq);
  });
  timeit("rows copy, contiguous -> u", rows * 2.0 * D * 2, [&] {
    hipLaunchKernelGGL((rows_kernel<0, 144>), dim3(g2), dim3(256), 0, 0, (const uint4*)dt, (uint4*)u, (int)rows, dq, dq);
  });
  timeit("rows read, x half-rows", rows * 1.0 * D * 2, [&] {
    hipLaunchKernelGGL((rows_kernel<1, 144>), dim3(g2), dim3(256), 0, 0, (const uint4*)xz, (uint4*)u, (int)rows, 2 * dq, dq);
  });
  timeit("rows read, contiguous", rows * 1.0 * D * 2, [&] {
    hipLaunchKernelGGL((rows_kernel<1, 144>), dim3(g2), dim3(256), 0, 0, (const uint4*)dt, (uint4*)u, (int)rows, dq, dq);
  });
  timeit("rows write, contiguous", rows * 1.0 * D * 2, [&] {
    hipLaunchKernelGGL((rows_kernel<2, 144>), dim3(g2), dim3(256), 0, 0, (const uint4*)dt, (uint4*)u, (int)rows, dq, dq);
  });
  timeit("full xz read (both halves)", rows * 2.0 * D * 2, [&] {
    hipLaunchKernelGGL((rows_kernel<1, 144>), dim3(g2), dim3(256), 0, 0, (const uint4*)xz, (uint4*)u, (int)rows * 2, dq, dq);
  });
  timeit("shape copy, 64-row WG, chunked", rows * 2.0 * D * 2, [&] {
    hipLaunchKernelGGL((shape_copy<true>), grid, dim3(256), 0, 0, xz, u, (int)rows, D); });
  timeit("shape copy, 64-row WG, row order", rows * 2.0 * D * 2, [&] {
    hipLaunchKernelGGL((shape_copy<false>), grid, dim3(256), 0, 0, xz, u, (int)rows, D); });
  const unsigned long long wn = rows * 1ull * D * 2;
#define WR(NAME, W, NT, G) timeit(NAME, (double)wn, [&] { \
    hipLaunchKernelGGL((wr_kernel<W, NT>), dim3(G), dim3(256), 0, 0, (uint8_t*)u, wn); })
  WR("write x16 plain g4096", 16, 0, 4096);
  WR("write x16 plain g16384", 16, 0, 16384);
  WR("write x16 nontemporal", 16, 1, 4096);
  WR("write x16 buffer aux0", 16, 2, 4096);
  WR("write x16 buffer aux1 (sc0)", 16, 3, 4096);
  WR("write x16 buffer aux2 (nt)", 16, 4, 4096);
  WR("write x16 buffer aux3", 16, 5, 4096);
  WR("write x8 plain", 8, 0, 4096);
  WR("write x8 nontemporal", 8, 1, 4096);
  WR("write x4 plain", 4, 0, 4096);
  WR("write x4 nontemporal", 4, 1, 4096);
#define RUN(NAME, X) timeit(NAME, cp_bytes, [&] { \
    hipLaunchKernelGGL((conv_proj_kernel<false, 5, X>), grid, dim3(256), lds, 0, p); })
  RUN("conv_proj (library)", 0);
  RUN("  - W_x staging loads", 1);
  RUN("  - x_proj MFMA", 2);
  RUN("  - u stores", 4);
  RUN("  - window loads", 8);
  RUN("  - loop barriers", 16);
  RUN("  - all memory in loop", 13);
  {  // with the streaming conv state in and out (the bench's stateful chunk)
    bf16_t *csi, *cso;
    CK(hipMalloc(&csi, (size_t)B * D * 4 * 2)); CK(hipMalloc(&cso, (size_t)B * D * 4 * 2));
    CK(hipMemset(csi, 0, (size_t)B * D * 4 * 2));
    ConvProjParams q = p;
    q.csi = csi; q.cso = cso; q.csi_sb = q.cso_sb = (long long)D * 4; q.csi_sd = q.cso_sd = 4;
    q.csi_dtype = q.cso_dtype = VM_DTYPE_BF16;
    timeit("conv_proj (library), conv state in+out", cp_bytes, [&] {
      hipLaunchKernelGGL((conv_proj_kernel<false, 5, 0>), grid, dim3(256), lds, 0, q);
      hipLaunchKernelGGL(conv_state_out_kernel, dim3((D + 255) / 256, B), dim3(256), 0, 0, q); });
    q.csi = nullptr;
    timeit("conv_proj (library), conv state out", cp_bytes, [&] {
      hipLaunchKernelGGL((conv_proj_kernel<false, 5, 0>), grid, dim3(256), lds, 0, q);
      hipLaunchKernelGGL(conv_state_out_kernel, dim3((D + 255) / 256, B), dim3(256), 0, 0, q); });
  }
  for (int rep = 0; rep < 2; ++rep) {
    timeit("split: conv_proj + dt_proj (library)", cp_bytes + dt_bytes, [&] {
      hipLaunchKernelGGL((conv_proj_kernel<false, 5, 0>), grid, dim3(256), lds, 0, p);
      hipLaunchKernelGGL((dt_proj_kernel<16, 4>), grid, dim3(256), 0, 0, p); });
    timeit("fused: conv_proj<DT> (half-tile dt)", cp_bytes + dt_bytes, [&] {
      hipLaunchKernelGGL((conv_proj_kernel<true, 5, 0>), grid, dim3(256), lds, 0, p); });
  }
  {  // fused dt must equal the split kernels' dt bit for bit
    std::vector<uint16_t> r1(rows * D), r2(rows * D);
    hipLaunchKernelGGL((conv_proj_kernel<false, 5, 0>), grid, dim3(256), lds, 0, p);
    hipLaunchKernelGGL((dt_proj_kernel<16, 4>), grid, dim3(256), 0, 0, p);
    CK(hipMemcpy(r1.data(), dt, rows * D * 2, hipMemcpyDeviceToHost));
    CK(hipMemset(dt, 0, rows * D * 2));
    hipLaunchKernelGGL((conv_proj_kernel<true, 5, 0>), grid, dim3(256), lds, 0, p);
    CK(hipMemcpy(r2.data(), dt, rows * D * 2, hipMemcpyDeviceToHost));
    long long diff = 0;
    for (long long i = 0; i < rows * D; ++i) diff += r1[i] != r2[i];
    printf("fused vs split dt: %lld differing elements of %lld\n", diff, rows * D);
  }
  for (int rep = 0; rep < 2; ++rep) {
    timeit("dt_proj 16 B stores, 4 waves", dt_bytes, [&] {
      hipLaunchKernelGGL((dt_proj_kernel<16, 4>), grid, dim3(256), 0, 0, p); });
    timeit("dt_proj (library: 8 B stores, 4 waves)", dt_bytes, [&] {
      hipLaunchKernelGGL((dt_proj_kernel<8, 4>), grid, dim3(256), 0, 0, p); });
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
