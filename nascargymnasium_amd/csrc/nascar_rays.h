// nascar_rays.h -- DistanceSensor ray end points (src/distance_sensor.py:95-103) without one f64
// sincos per ray.  Shared by the sensor kernel and a host harness (tests/test_rays_cpu.py compiles
// this header with g++ and checks it against glibc on random poses).
#pragma once
#include <math.h>

#pragma clang fp contract(off)

// cos / sin of k_i = math.radians(22.5 * i), i = 0..15 (f64, glibc 2.35 cos / sin of the f64 k_i)
#define NASCAR_RAY_CS_INIT { \
  {0x1.0000000000000p+0, 0x0.0p+0},                 {0x1.d906bcf328d46p-1, 0x1.87de2a6aea963p-2}, \
  {0x1.6a09e667f3bcdp-1, 0x1.6a09e667f3bccp-1},     {0x1.87de2a6aea964p-2, 0x1.d906bcf328d46p-1}, \
  {0x1.1a62633145c07p-54, 0x1.0000000000000p+0},    {-0x1.87de2a6aea962p-2, 0x1.d906bcf328d46p-1}, \
  {-0x1.6a09e667f3bccp-1, 0x1.6a09e667f3bcdp-1},    {-0x1.d906bcf328d46p-1, 0x1.87de2a6aea965p-2}, \
  {-0x1.0000000000000p+0, 0x1.1a62633145c07p-53},   {-0x1.d906bcf328d47p-1, -0x1.87de2a6aea961p-2}, \
  {-0x1.6a09e667f3bcep-1, -0x1.6a09e667f3bccp-1},   {-0x1.87de2a6aea95ep-2, -0x1.d906bcf328d47p-1}, \
  {-0x1.a79394c9e8a0ap-53, -0x1.0000000000000p+0},  {0x1.87de2a6aea967p-2, -0x1.d906bcf328d45p-1}, \
  {0x1.6a09e667f3bcbp-1, -0x1.6a09e667f3bcep-1},    {0x1.d906bcf328d47p-1, -0x1.87de2a6aea95fp-2}}

// f32 value of a f64 known only to lie within +-b of xa: true when every value of that interval
// rounds to the same float (round-to-nearest is monotonic, so the two end points decide)
__host__ __device__ inline bool f32_stable(double xa, double b, float& out) {
  const float lo = (float)(xa - b), hi = (float)(xa + b);
  out = (float)xa;
  return lo == hi;
}

// Ray i's end point (float)(px + cos(sa) * 250), (float)(py + sin(sa) * 250) with
// sa = -radians(22.5 i) + ang, as the reference computes it in Python floats before b2Vec2.
// The caller's cos/sin(ang) (c0, s0) are rotated by k_i (angle addition) and corrected to first
// order for the rounding error of sa (TwoSum: ang - k == sa + err exactly).  That puts cos/sin(sa)
// within 2e-15 of any libm value that is within 1 ulp; the f32 end point is taken from it only when
// the whole +-bound interval rounds to one float, otherwise (probability ~1e-8 per coordinate) from a
// direct f64 sincos(sa).  Returns 1 when the fallback was taken.  dx, dy: the f64 direction (cull only).
// the rare direct evaluation, out of line: inlined, its f64 sincos constants were hoisted out of the sensor
// kernel's ray loop and spilled to scratch (a reload per ray, 20 B of spill stores per lane)
__host__ __device__ __attribute__((noinline)) inline void ray_end_direct(double px, double py, double sa, float& fx,
                                                                         float& fy) {
  double ey, ex;
  sincos(sa, &ey, &ex);
  fx = (float)(px + ex * 250.0);
  fy = (float)(py + ey * 250.0);
}
// (ck, sk) = cs[i]: the ray offset's cos / sin from the table, passed in so a caller can request it early
__host__ __device__ inline int ray_end_f32_k(double px, double py, double ang, double c0, double s0, int i, double ck,
                                             double sk, double& dx, double& dy, float& fx, float& fy) {
  const double k = (double)i * (360.0 / 16) * (3.141592653589793 / 180.0);
  const double sa = -k + ang;
  const double bb = sa - ang;
  const double err = (ang - (sa - bb)) + (-k - bb);
  const double cd = c0 * ck + s0 * sk, sd = s0 * ck - c0 * sk;   // cos, sin(ang - k)
  dx = cd + sd * err;                                           // cos(ang - k - err)
  dy = sd - cd * err;
  const double xa = px + dx * 250.0, ya = py + dy * 250.0;
  // |cos error| <= 2e-15 (rotation ~1e-15 worst case + libm 1 ulp) x 250, plus the roundings of *250, +p
  const double bx = 6e-13 + fabs(xa) * 4.5e-16, by = 6e-13 + fabs(ya) * 4.5e-16;
  const bool okx = f32_stable(xa, bx, fx), oky = f32_stable(ya, by, fy);
  if (okx && oky) return 0;
  ray_end_direct(px, py, sa, fx, fy);
  return 1;
}
__host__ __device__ inline int ray_end_f32(double px, double py, double ang, double c0, double s0, int i,
                                           const double (*cs)[2], double& dx, double& dy, float& fx, float& fy) {
  return ray_end_f32_k(px, py, ang, c0, s0, i, cs[i][0], cs[i][1], dx, dy, fx, fy);
}
