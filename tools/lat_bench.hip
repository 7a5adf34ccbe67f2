// tools/lat_bench.hip -- latency calibration for a lone wave on gfx950 (tools only): s_memtime cycles per operation of
// dependent chains (f32 add, f64 fma, IEEE f32 divide, IEEE sqrt, glibc sinf/cosf restatement, LDS round trip).
#include "../nascargymnasium_amd/csrc/nascar_device.h"
using namespace nascar;
#define N 256
__global__ void __launch_bounds__(64) lat_kernel(float x0, double y0, unsigned long long* out, float* sink, int flat_lds) {
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
  // 9: the same LDS round trip through a generic (flat) pointer, as the Box2D step's contact records are reached
  float* gp = flat_lds ? (float*)lds : sink + 64;
  asm volatile("" : "+v"(gp));
  MEASURE(for (int i = 0; i < N / 4; ++i) { gp[lane] = x; x = gp[lane ^ 1] + 1.0f; })
  // 10: flat LDS round trips while a global store is outstanding (one store to sink per iteration)
  MEASURE(for (int i = 0; i < N / 4; ++i) { sink[128 + lane] = x; gp[lane] = x; x = gp[lane ^ 1] + 1.0f; })
  // 11: LDS round trips with a global store outstanding (ds ops do not wait for it)
  MEASURE(for (int i = 0; i < N / 4; ++i) { sink[128 + lane] = x; lds[lane] = x; __builtin_amdgcn_s_waitcnt(0xc07f); x = lds[lane ^ 1] + 1.0f; })
  // 12: f64 divide, 13: f64 sqrt (dependent)
  MEASURE(for (int i = 0; i < N / 4; ++i) { y = 1.0 / (y + 1.5); } x += (float)y;)
  MEASURE(for (int i = 0; i < N / 4; ++i) { y = sqrt(y + 1.5); } x += (float)y;)
  // 14: global load round trip (L2-warm, dependent)
  MEASURE(for (int i = 0; i < N / 4; ++i) { x = sink[64 + (((int)x) & 3)] + x; })
  if (lane == 0) sink[0] = x;
}
extern "C" int lat_bench(unsigned long long* out, float* sink) {
  hipLaunchKernelGGL(lat_kernel, dim3(1), dim3(64), 0, 0, 1.25f, 1.0000001, out, sink, 1);
  hipLaunchKernelGGL(lat_kernel, dim3(1), dim3(64), 0, 0, 1.25f, 1.0000001, out, sink, 1);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
