// Host check of nascar_math.h glibc_sincosf (the device restatement of glibc sinf/cosf used by b2Rot::Set)
// against the host glibc: every stride-th float bit pattern, split over threads.
//   sincosf_harness <stride> <threads>   ->  prints "<checked> <mismatches>"
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include "../../nascargymnasium_amd/csrc/nascar_math.h"

int main(int argc, char** argv) {
  const uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 10) : 97;
  const int T = argc > 2 ? atoi(argv[2]) : 8;
  std::atomic<uint64_t> checked{0}, bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back([&, t] {
    uint64_t c = 0, b = 0;
    for (uint64_t u = (uint64_t)t * stride; u < (1ull << 32); u += stride * T) {
      float x; uint32_t v = (uint32_t)u; memcpy(&x, &v, 4);
      if (!std::isfinite(x)) continue;
      float s, co; nascar::glibc_sincosf(x, &s, &co);
      float rs = sinf(x), rc = cosf(x);
      if (memcmp(&s, &rs, 4) || memcmp(&co, &rc, 4)) { if (b < 5) fprintf(stderr, "x=%a %a/%a %a/%a\n", x, s, rs, co, rc); ++b; }
      ++c;
    }
    checked += c; bad += b;
  });
  for (auto& x : th) x.join();
  printf("%llu %llu\n", (unsigned long long)checked.load(), (unsigned long long)bad.load());
  return 0;
}
