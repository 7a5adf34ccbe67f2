// Host harness for nascar_rays.h (test infrastructure): random car poses, every ray's f32 end point
// from ray_end_f32 vs the direct Python-float evaluation (glibc sincos of sa, src/distance_sensor.py:95-103).
// Prints "<cases> <mismatches> <fallbacks>".
#define __host__
#define __device__
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include "../../nascargymnasium_amd/csrc/nascar_rays.h"

static uint64_t s = 0x9E3779B97F4A7C15ull;
static double urand() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (double)(s >> 11) * 0x1p-53; }

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  static const double cs[16][2] = NASCAR_RAY_CS_INIT;
  long bad = 0, fb = 0, cases = 0;
  for (long t = 0; t < n; ++t) {
    // positions as f32 Box2D values widened to double; angles from small to wound-up (|ang| < 400 rad)
    const double px = (float)((urand() - 0.5) * 1200.0), py = (float)((urand() - 0.5) * 900.0);
    const int kind = t & 3;
    double ang = kind == 0 ? (urand() - 0.5) * 6.5 : kind == 1 ? (urand() - 0.5) * 800.0
               : kind == 2 ? (float)((urand() - 0.5) * 0.01) : (float)((urand() - 0.5) * 6.5);
    if (t % 97 == 0) ang = (double)(t % 16) * 22.5 * (3.141592653589793 / 180.0);   // sa == 0 exactly
    double s0, c0;
    sincos(ang, &s0, &c0);
    for (int i = 0; i < 16; ++i) {
      double dx, dy;
      float fx, fy;
      fb += ray_end_f32(px, py, ang, c0, s0, i, cs, dx, dy, fx, fy);
      const double sa = -((double)i * (360.0 / 16) * (3.141592653589793 / 180.0)) + ang;
      double ey, ex;
      sincos(sa, &ey, &ex);
      const float gx = (float)(px + ex * 250.0), gy = (float)(py + ey * 250.0);
      if (gx != fx || gy != fy) ++bad;
      ++cases;
    }
  }
  printf("%ld %ld %ld\n", cases, bad, fb);
  return bad != 0;
}
