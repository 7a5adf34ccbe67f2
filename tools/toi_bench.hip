// tools/toi_bench.hip -- micro-benchmark of one b2TimeOfImpact job (nascar_device.h toi_alpha) on captured inputs.
// Not product code: tools/toi_bench.py builds it (with the variant's -D flags), feeds it the jobs a
// -DNASCAR_TOI_CAPTURE profile build recorded at the bench's steady state, and reports s_memtime cycles per call
// and the alphas (bit-compared across variants).
#include "../nascargymnasium_amd/csrc/nascar_device.h"
using namespace nascar;

struct TCap { float4 s0, s1, w0, w1; };

// one wave per workgroup; round it: lanes 0 .. lanes-1 take jobs it * lanes + lane (lanes = 1: a lone TOI chain as in
// the slowest wave's scans).  Every workgroup runs the same jobs (blocks > 1: co-resident competing waves); workgroup 0
// writes the alphas and the cycles of each round.
__global__ void __launch_bounds__(64) toi_bench_kernel(const TCap* jobs, int n, int lanes, float* alpha,
                                                       unsigned long long* cyc, int* det) {
  const int lane = threadIdx.x;
  const int rounds = (n + lanes - 1) / lanes;
  for (int it = 0; it < rounds; ++it) {
    const int j = it * lanes + lane;
    const bool act = lane < lanes && j < n;
    TCap t = act ? jobs[j] : jobs[0];
    LWall w;
    w.px = t.w0.x; w.py = t.w0.y; w.qs = t.w0.z; w.qc = t.w0.w;
    w.hx = t.w1.x; w.hy = t.w1.y; w.ang = t.w1.z; w.key = __float_as_int(t.w1.w);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    float a = 1.0f;
#ifdef NASCAR_PROFILE   // detail build: outer / root / GJK iterations, GJK and separation-function cycles per job
    int it3[3] = {0, 0, 0}; unsigned long long cy2[2] = {0ull, 0ull};
    if (act) a = toi_alpha(t.s0, t.s1, w, it3, cy2);
#else
    if (act) a = toi_alpha(t.s0, t.s1, w);
#endif
    asm volatile("" :: "v"(a));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0) {
      if (act) alpha[j] = a;
      if (lane == 0) cyc[it] = t1 - t0;
#ifdef NASCAR_PROFILE
      if (act && det) {
        det[5 * j] = it3[0]; det[5 * j + 1] = it3[1]; det[5 * j + 2] = it3[2];
        det[5 * j + 3] = (int)cy2[0]; det[5 * j + 4] = (int)cy2[1];
      }
#endif
    }
  }
}

extern "C" int toi_bench(const void* jobs, int n, int lanes, int blocks, float* alpha, unsigned long long* cyc, int* det) {
  hipLaunchKernelGGL(toi_bench_kernel, dim3(blocks), dim3(64), 0, 0, (const TCap*)jobs, n, lanes, alpha, cyc, det);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
