// Issue-rate probe for the selective-scan step mix on gfx950 (tools only, not product).
// Per iteration and lane: 16 states x { t = dl*A[n]; a = exp2(t); b = du*B[n];
// h[n] = a*h[n] + b; y += h[n]*C[n] } — the channel-per-lane scan step — compiled by
// hipcc, in registers, at 1..4 waves per SIMD.  Variants isolate the exp stream and the
// FMA stream, and test whether independent transcendental and FMA streams overlap.
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITERS = 2048;

template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out, float s0, float s1) {
  float A[16], Bv[16], Cv[16], h[16];
#pragma unroll
  for (int n = 0; n < 16; ++n) {
    A[n] = -(n + 1) * 0.01f * s0;
    Bv[n] = 0.5f + n * s1;
    Cv[n] = 0.25f - n * s1;
    h[n] = threadIdx.x * 1e-4f;
  }
  float dl = 0.1f + threadIdx.x * 1e-5f, du = 0.2f, y = 0.0f, e = 0.0f;
  for (int it = 0; it < ITERS; ++it) {
    if (MODE == 0) {  // full step
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        const float a = __builtin_amdgcn_exp2f(dl * A[n]);
        h[n] = fmaf(a, h[n], du * Bv[n]);
        y = fmaf(h[n], Cv[n], y);
      }
    } else if (MODE == 1) {  // exps only (16, independent)
#pragma unroll
      for (int n = 0; n < 16; ++n) h[n] += __builtin_amdgcn_exp2f(dl * A[n]);
    } else if (MODE == 2) {  // the step without the exp (a := t)
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        const float a = dl * A[n];
        h[n] = fmaf(a, h[n], du * Bv[n]);
        y = fmaf(h[n], Cv[n], y);
      }
    } else if (MODE == 3) {  // full step, two y chains
      float y1 = 0.0f;
#pragma unroll
      for (int n = 0; n < 16; n += 2) {
        const float a0 = __builtin_amdgcn_exp2f(dl * A[n]);
        const float a1 = __builtin_amdgcn_exp2f(dl * A[n + 1]);
        h[n] = fmaf(a0, h[n], du * Bv[n]);
        h[n + 1] = fmaf(a1, h[n + 1], du * Bv[n + 1]);
        y = fmaf(h[n], Cv[n], y);
        y1 = fmaf(h[n + 1], Cv[n + 1], y1);
      }
      y += y1;
    } else if (MODE == 4) {  // 16 independent exps + 48 independent fmas per iteration
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(Bv[n]));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(h[n]) : "v"(dl), "v"(du));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(Cv[n]) : "v"(dl), "v"(du));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(A[n]) : "v"(dl), "v"(du));
      }
    } else if (MODE == 5) {  // 64 independent fmas (no exps)
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(Bv[n]) : "v"(dl), "v"(du));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(h[n]) : "v"(dl), "v"(du));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(Cv[n]) : "v"(dl), "v"(du));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(A[n]) : "v"(dl), "v"(du));
      }
    }
    dl = fmaf(dl, 0.9999f, 1e-6f);
    du = fmaf(du, 0.9999f, 1e-6f);
  }
  float s = y + e;
#pragma unroll
  for (int n = 0; n < 16; ++n) s += h[n] + A[n] + Bv[n] + Cv[n];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
float run(int waves_per_simd, float* buf, int cus) {
  dim3 grid(cus * waves_per_simd);  // 256-thread blocks: one wave per SIMD each
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<MODE><<<grid, 256>>>(buf, 1.0f, 0.001f);
  hipEventRecord(e0);
  probe<MODE><<<grid, 256>>>(buf, 1.0f, 0.001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  float* buf;
  hipMalloc(&buf, sizeof(float) * cus * 8 * 256);
  const char* names[] = {"step(16 exp+64 valu)", "exp only (16)", "step w/o exp (64)",
                         "step, 2 y-chains", "indep 16exp+48fma", "indep 64 fma"};
  printf("CUs=%d clock(kHz)=%d  (cycles assume 2.4 GHz)\n", cus, prop.clockRate);
  for (int w : {1, 2, 3, 4}) {
    const float t[6] = {run<0>(w, buf, cus), run<1>(w, buf, cus), run<2>(w, buf, cus),
                        run<3>(w, buf, cus), run<4>(w, buf, cus), run<5>(w, buf, cus)};
    for (int m = 0; m < 6; ++m) {
      const double cycles = t[m] * 1e-3 * 2.4e9;
      printf("waves/SIMD=%d %-22s cycles per wave-iteration per SIMD = %7.1f\n", w, names[m],
             cycles / (ITERS * (double)w));
    }
  }
  return 0;
}
