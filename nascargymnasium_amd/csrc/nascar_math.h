// nascar_math.h -- device math that reproduces the reference's numerics on gfx950.
//
// * b2Rot::Set (Box2D, float32) calls glibc sinf/cosf on the reference host.
//   dev_sinf/dev_cosf below re-implement glibc's (>= 2.28) sinf/cosf
//   algorithm -- the __sincosf_table polynomials, reduce_fast / reduce_large --
//   evaluated in double with the fused multiply-adds of glibc's x86-64 FMA
//   variant.  Verified bit-identical to glibc 2.35 sinf/cosf over all 4.28e9
//   finite floats in the build container (DESIGN.md "Numerics").
// * Python float64 arithmetic: plain IEEE double ops, no contraction
//   (#pragma clang fp contract(off) + -ffp-contract=off).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace nascar {

// Correctly rounded float32 sqrt / divide (what x86 sqrtss / divss give Box2D).
// On gfx950 `sqrtf` and `/` lower to the IEEE sequences (v_sqrt + fma fix-up,
// v_div_scale/fmas/fixup); `__fsqrt_rn` lowers to a bare v_sqrt_f32 (~1 ulp),
// which broke parity -- never use it here.
__device__ __forceinline__ float fsqrt_cr(float x) { return sqrtf(x); }
__device__ __forceinline__ float fdiv_cr(float a, float b) { return a / b; }

// glibc's __sincosf_table (sysdeps/ieee754/flt-32/s_sincosf.h) as immediates: its second row is the first with
// every cosine coefficient negated (sine coefficients equal), and negating all coefficients of a fused
// multiply-add chain negates its result exactly, so the row choice becomes a final sign flip.  No table
// loads are left on the chain (a lane-dependent row index had turned them into per-lane memory loads).
#define SC_HPI_INV 0x1.45f306dc9c883p+23
#define SC_HPI 0x1.921fb54442d18p+0
#define SC_C0 0x1p0
#define SC_C1 (-0x1.ffffffd0c621cp-2)
#define SC_S1 (-0x1.555545995a603p-3)
#define SC_C2 0x1.55553e1068f19p-5
#define SC_S2 0x1.1107605230bc4p-7
#define SC_C3 (-0x1.6c087e89a359dp-10)
#define SC_S3 (-0x1.994eb3774cf24p-13)
#define SC_C4 0x1.99343027bf8c3p-16

__host__ __device__ __forceinline__ uint32_t f_as_u(float f) {
  union { float f; uint32_t u; } v; v.f = f; return v.u;
}
__host__ __device__ __forceinline__ uint32_t top12(float x) { return (f_as_u(x) >> 20) & 0x7ff; }

// glibc sinf_poly (FMA variant): the sine polynomial for even n, the cosine polynomial (negated for the
// second table row, neg != 0) for odd n
__host__ __device__ __forceinline__ float sc_poly(double x, double x2, int n, int neg) {
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = fma(x2, SC_S3, SC_S2);
    double x7 = x3 * x2;
    double s = fma(x3, SC_S1, x);
    return (float)fma(x7, s1, s);
  }
  double x4 = x2 * x2;
  double c2 = fma(x2, SC_C4, SC_C3);
  double c1 = fma(x2, SC_C1, SC_C0);
  double x6 = x4 * x2;
  double c = fma(x4, SC_C2, c1);
  float r = (float)fma(x6, c2, c);
  return neg ? -r : r;
}
__host__ __device__ __forceinline__ double reduce_fast(double x, int* np) {
  double r = x * SC_HPI_INV;
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return fma(-(double)n, SC_HPI, x);
}
#define SC_INV_PIO4 {0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529, \
                     0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0, \
                     0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041}
__device__ __constant__ const uint32_t kInvPio4[24] = SC_INV_PIO4;   // glibc __inv_pio4
static const uint32_t kInvPio4Host[24] = SC_INV_PIO4;
__host__ __device__ __forceinline__ uint32_t inv_pio4(int i) {
#ifdef __HIP_DEVICE_COMPILE__
  return kInvPio4[i];
#else
  return kInvPio4Host[i];
#endif
}
// |y| >= 120: rare (wound-up angles).  Out of line on the device: inlined into every b2Rot::Set it was ~15 KB of
// model_kernel's code for a path almost never taken.
#ifndef SINCOS_LARGE_INLINE
#define SINCOS_LARGE_INLINE 0
#endif
#if defined(__HIP_DEVICE_COMPILE__) && !SINCOS_LARGE_INLINE
__attribute__((noinline))
#endif
__host__ __device__ inline double reduce_large(uint32_t xi, int* np) {
  const int k = (xi >> 26) & 15;
  int shift = (xi >> 23) & 7;
  uint64_t n, res0, res1, res2;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  res0 = xi * inv_pio4(k);
  res1 = (uint64_t)xi * inv_pio4(k + 4);
  res2 = (uint64_t)xi * inv_pio4(k + 8);
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  n = (res0 + (1ULL << 61)) >> 62;
  res0 -= n << 62;
  double x = (double)(int64_t)res0;
  *np = (int)n;
  return x * 0x1.921FB54442D18p-62;
}
// glibc sinf and cosf (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c; FMA variant) of the same argument in one
// pass: both share the range reduction, and each result is bit-identical to the separate call (the same
// operations on the same values).  b2Rot::Set calls sinf then cosf.
#ifndef SINCOS_NOINLINE
#define SINCOS_NOINLINE 0   // A/B: one out-of-line copy of b2Rot::Set's sincosf instead of one per call site
#endif
#ifndef SINCOS_V2
#define SINCOS_V2 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && SINCOS_NOINLINE
__attribute__((noinline))
#endif
__host__ __device__ inline void glibc_sincosf(float y, float* sp, float* cp) {
#if SINCOS_V2
  // One straight-line path for |y| < 120 (the only rare branch is glibc's reduce_large): glibc's |y| < pi/4 path is
  // reduce_fast's n = 0 case (x - 0 * pi/2 == x exactly, sign +1, first table row), and both polynomials are
  // evaluated side by side and assigned by the quadrant's parity (glibc evaluates the same two polynomials on the
  // same values), so the dependent chain is one polynomial deep instead of two plus branches.  |y| < 2^-12 returns
  // (y, 1) as glibc does (also keeping sin(-0) = -0).  Bit-identical to the host glibc over all 2^32 floats
  // (tests/test_rays_cpu.py::test_glibc_sincosf_restatement_matches_host_libm: every 61st pattern by default,
  // every pattern with NASCAR_SINCOS_STRIDE=1: 4 278 190 080 finite floats, 0 mismatches, 26 s on 8 threads).
  const uint32_t t = top12(y);
  if (t >= top12(120.0f)) {
    uint32_t xi = f_as_u(y);
    int sign = xi >> 31, n = 0;
    const double x = reduce_large(xi, &n);
    const double sgn = ((n + sign + 1) & 2) ? -1.0 : 1.0;
    const int row = (n + sign) & 2;
    const double xs = x * sgn, x2 = x * x;
    *sp = sc_poly(xs, x2, n, row);
    *cp = sc_poly(xs, x2, n ^ 1, row);
    return;
  }
  int n = 0;
  const double x = reduce_fast((double)y, &n);
  const double xs = ((n + 1) & 2) ? -x : x, x2 = x * x;   // x * sgn, sgn = {1, -1, -1, 1}[n & 3]
  const float ps = sc_poly(xs, x2, 0, 0), pc = sc_poly(xs, x2, 1, n & 2);
  const bool odd = n & 1, tiny = t < top12(0x1p-12f);
  *sp = tiny ? y : (odd ? pc : ps);
  *cp = tiny ? 1.0f : (odd ? ps : pc);
#else
  double x = y;
  int n = 0, row = 0;
  double sgn = 1.0;
  const float pio4 = 0x1.921FB6p-1f;
  if (top12(y) < top12(pio4)) {
    if (top12(y) < top12(0x1p-12f)) { *sp = y; *cp = 1.0f; return; }
    double x2 = x * x;
    *sp = sc_poly(x, x2, 0, 0);
    *cp = sc_poly(x, x2, 1, 0);
    return;
  } else if (top12(y) < top12(120.0f)) {
    x = reduce_fast(x, &n);
    sgn = ((n + 1) & 2) ? -1.0 : 1.0;   // {1, -1, -1, 1}[n & 3]
    row = n & 2;
  } else {
    uint32_t xi = f_as_u(y);
    int sign = xi >> 31;
    x = reduce_large(xi, &n);
    sgn = ((n + sign + 1) & 2) ? -1.0 : 1.0;
    row = (n + sign) & 2;
  }
  const double xs = x * sgn, x2 = x * x;
  *sp = sc_poly(xs, x2, n, row);
  *cp = sc_poly(xs, x2, n ^ 1, row);
#endif
}

// Python float64 helpers
__device__ __forceinline__ double pymin(double a, double b) { return b < a ? b : a; }
__device__ __forceinline__ double pymax(double a, double b) { return b > a ? b : a; }
__device__ __forceinline__ double npclip(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
// Python `x ** 2` / `x ** 0.5` (glibc pow on the reference host).  x*x and the
// correctly-rounded sqrt differ from glibc pow only in rare near-tie cases (see
// DESIGN.md "Numerics"); none reaches a float32 output in the parity suite.
__device__ __forceinline__ double P2(double x) { return x * x; }
__device__ __forceinline__ double PH(double x) { return sqrt(x); }

}  // namespace nascar
