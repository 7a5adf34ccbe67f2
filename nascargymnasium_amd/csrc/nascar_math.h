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

struct SinCosTable {
  double sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4;
};

__device__ __constant__ const SinCosTable kSC[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 0x1p0, -0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, -0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16}};

__device__ __constant__ const uint32_t kInvPio4[24] = {
    0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};

__device__ __forceinline__ uint32_t f_as_u(float f) { return __float_as_uint(f); }
__device__ __forceinline__ uint32_t top12(float x) { return (f_as_u(x) >> 20) & 0x7ff; }

__device__ __forceinline__ float sc_poly(double x, double x2, const SinCosTable* p, int n) {
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = __fma_rn(x2, p->s3, p->s2);
    double x7 = x3 * x2;
    double s = __fma_rn(x3, p->s1, x);
    return (float)__fma_rn(x7, s1, s);
  } else {
    double x4 = x2 * x2;
    double c2 = __fma_rn(x2, p->c4, p->c3);
    double c1 = __fma_rn(x2, p->c1, p->c0);
    double x6 = x4 * x2;
    double c = __fma_rn(x4, p->c2, c1);
    return (float)__fma_rn(x6, c2, c);
  }
}
__device__ __forceinline__ double reduce_fast(double x, const SinCosTable* p, int* np) {
  double r = x * p->hpi_inv;
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return __fma_rn(-(double)n, p->hpi, x);
}
__device__ __forceinline__ double reduce_large(uint32_t xi, int* np) {
  const uint32_t* arr = &kInvPio4[(xi >> 26) & 15];
  int shift = (xi >> 23) & 7;
  uint64_t n, res0, res1, res2;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  res0 = xi * arr[0];
  res1 = (uint64_t)xi * arr[4];
  res2 = (uint64_t)xi * arr[8];
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  n = (res0 + (1ULL << 61)) >> 62;
  res0 -= n << 62;
  double x = (double)(int64_t)res0;
  *np = (int)n;
  return x * 0x1.921FB54442D18p-62;
}
// glibc sinf (sysdeps/ieee754/flt-32/s_sinf.c), FMA variant
__device__ inline float dev_sinf(float y) {
  double x = y, s;
  int n;
  const SinCosTable* p = &kSC[0];
  const float pio4 = 0x1.921FB6p-1f;
  if (top12(y) < top12(pio4)) {
    double x2 = x * x;
    if (top12(y) < top12(0x1p-12f)) return y;
    return sc_poly(x, x2, p, 0);
  } else if (top12(y) < top12(120.0f)) {
    x = reduce_fast(x, p, &n);
    s = p->sign[n & 3];
    if (n & 2) p = &kSC[1];
    return sc_poly(x * s, x * x, p, n);
  } else {
    uint32_t xi = f_as_u(y);
    int sign = xi >> 31;
    x = reduce_large(xi, &n);
    s = p->sign[(n + sign) & 3];
    if ((n + sign) & 2) p = &kSC[1];
    return sc_poly(x * s, x * x, p, n);
  }
}
// glibc cosf (sysdeps/ieee754/flt-32/s_cosf.c), FMA variant
__device__ inline float dev_cosf(float y) {
  double x = y, s;
  int n;
  const SinCosTable* p = &kSC[0];
  const float pio4 = 0x1.921FB6p-1f;
  if (top12(y) < top12(pio4)) {
    double x2 = x * x;
    if (top12(y) < top12(0x1p-12f)) return 1.0f;
    return sc_poly(x, x2, p, 1);
  } else if (top12(y) < top12(120.0f)) {
    x = reduce_fast(x, p, &n);
    s = p->sign[n & 3];
    if (n & 2) p = &kSC[1];
    return sc_poly(x * s, x * x, p, n ^ 1);
  } else {
    uint32_t xi = f_as_u(y);
    int sign = xi >> 31;
    x = reduce_large(xi, &n);
    s = p->sign[(n + sign) & 3];
    if ((n + sign) & 2) p = &kSC[1];
    return sc_poly(x * s, x * x, p, n ^ 1);
  }
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
