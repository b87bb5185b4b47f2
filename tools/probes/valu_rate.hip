// VALU issue-rate probe for gfx950: cycles per wave64 instruction per SIMD for
// independent v_fma_f32 / v_pk_fma_f32 / v_exp_f32 / v_mul_f32 streams, at 1..8 waves
// per SIMD.  Standalone executable (tools only, not part of the product).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out, float a, float b) {
  float x[16];
  f2 y[8];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 1e-3f + i;
#pragma unroll
  for (int i = 0; i < 8; ++i) y[i] = f2{x[2 * i], x[2 * i + 1]};
  const f2 a2 = {a, a}, b2 = {b, b};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (MODE == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
      if (MODE == 2) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
      if (MODE == 3) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
      if (MODE == 4) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
      }
    }
    if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(y[i]) : "v"(a2), "v"(b2));
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(y[i]) : "v"(a2), "v"(b2));
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += x[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += y[i].x + y[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
float run(int waves_per_simd, float* buf, int cus) {
  // 256-thread blocks = 1 wave per SIMD; blocks per CU = waves_per_simd
  dim3 grid(cus * waves_per_simd);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  probe<MODE><<<grid, 256>>>(buf, 0.999f, 0.001f);
  hipEventRecord(e0);
  probe<MODE><<<grid, 256>>>(buf, 0.999f, 0.001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0);
  int cus = prop.multiProcessorCount;
  float* buf; hipMalloc(&buf, sizeof(float) * cus * 8 * 256);
  const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_exp_f32", "v_mul_f32", "exp+fma"};
  // instruction count per wave per iteration (VALU wave-instructions)
  const double inst[] = {16, 16, 16, 16, 32};
  printf("CUs=%d clock(kHz)=%d\n", cus, prop.clockRate);
  for (int w : {1, 2, 4, 8}) {
    float t[5] = {run<0>(w, buf, cus), run<1>(w, buf, cus), run<2>(w, buf, cus), run<3>(w, buf, cus), run<4>(w, buf, cus)};
    for (int m = 0; m < 5; ++m) {
      double cycles = t[m] * 1e-3 * 2.4e9;  // assume 2.4 GHz
      double per = cycles / (ITERS * inst[m] * w);
      printf("waves/SIMD=%d %-14s %.3f ms  cycles/wave-instr/SIMD=%.2f\n", w, names[m], t[m], per);
    }
  }
  return 0;
}
