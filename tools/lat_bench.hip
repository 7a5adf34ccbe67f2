// tools/lat_bench.hip -- latency calibration for a lone wave on gfx950 (tools only): s_memtime cycles per operation of
// dependent chains (f32 add, f64 fma, IEEE f32 divide, IEEE sqrt, glibc sinf/cosf restatement, LDS round trip).
#include "../nascargymnasium_amd/csrc/nascar_device.h"
using namespace nascar;
#define N 256
__global__ void __launch_bounds__(64) lat_kernel(float x0, double y0, unsigned long long* out, float* sink) {
  __shared__ float lds[64];
  const int lane = threadIdx.x;
  float x = x0 + lane * 1e-7f; double y = y0 + lane * 1e-9;
  unsigned long long t0, t1;
  int k = 0;
#define MEASURE(...) \
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); t0 = __builtin_amdgcn_s_memtime(); \
  __VA_ARGS__; asm volatile("" :: "v"(x)); t1 = __builtin_amdgcn_s_memtime(); if (lane == 0) out[k] = t1 - t0; ++k;
  MEASURE(for (int i = 0; i < N; ++i) { asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(x0)); })            // 0 dep add
  MEASURE(float a = x, b = x + 1, c = x + 2, d = x + 3;
          for (int i = 0; i < N / 4; ++i) { asm volatile("v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4"
                                                       : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x0)); } x = a + b + c + d;)  // 1 indep add
  MEASURE(for (int i = 0; i < N / 4; ++i) { x = fdiv_cr(1.0f, x + 1.5f); })                                          // 2 div
  MEASURE(for (int i = 0; i < N / 4; ++i) { x = fsqrt_cr(x + 1.5f); })                                               // 3 sqrt
  MEASURE(for (int i = 0; i < N / 4; ++i) { float s, c; glibc_sincosf(x + 0.5f, &s, &c); x = s + c; })              // 4 sincos
  MEASURE(for (int i = 0; i < N; ++i) { asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(y) : "v"(y0)); } x += (float)y;)  // 5 dep f64 fma
  MEASURE(for (int i = 0; i < N / 4; ++i) { lds[lane] = x; __builtin_amdgcn_s_waitcnt(0xc07f); x = lds[lane ^ 1] + 1.0f; })  // 6 lds
  MEASURE(for (int i = 0; i < N; ++i) { asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(x0)); })            // 7 dep mul
  MEASURE(for (int i = 0; i < N / 4; ++i) { x = (x > 0.5f) ? x * 0.5f : x + 0.7f; })                                 // 8 select chain
  if (lane == 0) sink[0] = x;
}
extern "C" int lat_bench(unsigned long long* out, float* sink) {
  hipLaunchKernelGGL(lat_kernel, dim3(1), dim3(64), 0, 0, 1.25f, 1.0000001, out, sink);
  hipLaunchKernelGGL(lat_kernel, dim3(1), dim3(64), 0, 0, 1.25f, 1.0000001, out, sink);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
