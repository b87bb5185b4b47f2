// Packed-f32 issue-rate probe for gfx950 (tools only, not product): does one
// v_pk_fma_f32 / v_pk_mul_f32 (two f32 FMAs per lane) issue as fast as one v_fma_f32,
// and what does the channel-per-lane scan step cost when its four per-state VALU ops are
// packed over state pairs?  Cycles come from s_memtime inside the kernel (shader clock),
// so DVFS does not skew them.  1..4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 2048;

template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out, long long* cyc, float s0, float s1) {
  float x[16];
  f2 y[8], A[8], Bv[8], Cv[8], h[8];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 1e-3f + i;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    y[i] = f2{x[2 * i], x[2 * i + 1]};
    A[i] = f2{-(2 * i + 1) * 0.01f * s0, -(2 * i + 2) * 0.01f * s0};
    Bv[i] = f2{0.5f + 2 * i * s1, 0.5f + (2 * i + 1) * s1};
    Cv[i] = f2{0.25f - 2 * i * s1, 0.25f - (2 * i + 1) * s1};
    h[i] = f2{threadIdx.x * 1e-4f, threadIdx.x * 2e-4f};
  }
  const f2 a2 = {s0, s0}, b2 = {s1, s1};
  float dl = 0.1f + threadIdx.x * 1e-5f, du = 0.2f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
    if (MODE == 0) {  // 16 independent v_fma_f32
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(s0), "v"(s1));
    } else if (MODE == 1) {  // 16 independent v_pk_fma_f32 (32 FMAs)
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(y[i]) : "v"(a2), "v"(b2));
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(h[i]) : "v"(a2), "v"(b2));
    } else if (MODE == 2) {  // 16 independent v_pk_mul_f32
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(y[i]) : "v"(a2));
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(h[i]) : "v"(a2));
    } else if (MODE == 3) {  // 16 independent v_exp_f32
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
    } else if (MODE == 4) {  // 16 exp interleaved with 16 pk_fma
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(x[2 * i]));
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(y[i]) : "v"(a2), "v"(b2));
        asm volatile("v_exp_f32 %0, %0" : "+v"(x[2 * i + 1]));
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(h[i]) : "v"(a2), "v"(b2));
      }
    } else if (MODE == 5) {  // scalar scan step (compiled)
      float y0 = 0.f, y1 = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float a0 = __builtin_amdgcn_exp2f(dl * A[i].x);
        const float a1 = __builtin_amdgcn_exp2f(dl * A[i].y);
        h[i].x = fmaf(a0, h[i].x, du * Bv[i].x);
        h[i].y = fmaf(a1, h[i].y, du * Bv[i].y);
        y0 = fmaf(h[i].x, Cv[i].x, y0);
        y1 = fmaf(h[i].y, Cv[i].y, y1);
      }
      x[0] += y0 + y1;
    } else if (MODE == 6) {  // packed scan step: pk_mul(dl*A), 2 exp, pk_mul(du*B), pk_fma h, pk_fma y
      f2 yy = {0.f, 0.f};
      const f2 dl2 = {dl, dl}, du2 = {du, du};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f2 t = dl2 * A[i];
        f2 a;
        a.x = __builtin_amdgcn_exp2f(t.x);
        a.y = __builtin_amdgcn_exp2f(t.y);
        h[i] = __builtin_elementwise_fma(a, h[i], du2 * Bv[i]);
        yy = __builtin_elementwise_fma(h[i], Cv[i], yy);
      }
      x[0] += yy.x + yy.y;
    }
    dl = fmaf(dl, 0.9999f, 1e-6f);
    du = fmaf(du, 0.9999f, 1e-6f);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += x[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += y[i].x + y[i].y + h[i].x + h[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

template <int MODE>
void run(int w, float* buf, long long* cyc, int cus, double* ms_out, double* cyc_out) {
  dim3 grid(cus * w);  // 256-thread blocks: one wave per SIMD each
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<MODE><<<grid, 256>>>(buf, cyc, 1.0f, 0.001f);
  hipEventRecord(e0);
  probe<MODE><<<grid, 256>>>(buf, cyc, 1.0f, 0.001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long c;
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  *ms_out = ms;
  *cyc_out = (double)c;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  float* buf;
  long long* cyc;
  hipMalloc(&buf, sizeof(float) * cus * 8 * 256);
  hipMalloc(&cyc, sizeof(long long));
  const char* names[] = {"16 v_fma_f32", "16 v_pk_fma_f32", "16 v_pk_mul_f32", "16 v_exp_f32",
                         "16 exp + 16 pk_fma", "scan step scalar", "scan step packed"};
  printf("CUs=%d; cycles = s_memtime delta of wave 0 / ITERS (per wave-iteration; with w waves "
         "per SIMD the SIMD cost per wave-iteration is cycles/w)\n", cus);
  for (int w : {1, 2, 4}) {
    double ms[7], c[7];
    run<0>(w, buf, cyc, cus, &ms[0], &c[0]);
    run<1>(w, buf, cyc, cus, &ms[1], &c[1]);
    run<2>(w, buf, cyc, cus, &ms[2], &c[2]);
    run<3>(w, buf, cyc, cus, &ms[3], &c[3]);
    run<4>(w, buf, cyc, cus, &ms[4], &c[4]);
    run<5>(w, buf, cyc, cus, &ms[5], &c[5]);
    run<6>(w, buf, cyc, cus, &ms[6], &c[6]);
    for (int m = 0; m < 7; ++m)
      printf("waves/SIMD=%d %-20s %.3f ms  wave0 cycles/iter=%7.1f  SIMD cycles/wave-iter=%7.1f  clk=%.2f GHz\n",
             w, names[m], ms[m], c[m] / ITERS, c[m] / ITERS / w, c[m] / (ms[m] * 1e6));
  }
  return 0;
}
