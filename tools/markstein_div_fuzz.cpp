// Host fuzz: fl(a / S) against Markstein's q0 = fl(a y), fl(q0 + fma(-q0, S, a) y), y = fl(1 / S)
// (csrc/seed.hip seg_block_kernel).  g++ -O2 -o /tmp/mk tools/markstein_div_fuzz.cpp && /tmp/mk
#include <cstdio>
#include <cmath>
#include <cstring>
#include <random>
#include <cstdint>
static inline double mk(double a, double S, double y) {
  const double q0 = a * y;
  const double r = std::fma(-q0, S, a);
  return std::fma(r, y, q0);
}
int main() {
  std::mt19937_64 g(7);
  long long n = 0, bad = 0;
  auto rnd_sig = [&](int mode) -> double {
    uint64_t m = g() & 0xFFFFFFFFFFFFFull;
    if (mode == 1) m = 0xFFFFFFFFFFFFFull - (g() & 0xFF);
    if (mode == 2) m = g() & 0xFF;
    if (mode == 3) m = (g() & 1) ? 0x8000000000000ull ^ (g() & 0xFFF) : 0x7FFFFFFFFFFFFull - (g() & 0xFFF);
    uint64_t bits = (1023ull << 52) | m;
    double x; memcpy(&x, &bits, 8); return x;  // [1, 2)
  };
  for (long long it = 0; it < 40000000; ++it) {
    const double S = std::ldexp(rnd_sig((int)(it % 4)), (int)(g() % 200) - 60);
    const double y = 1.0 / S;
    for (int t = 0; t < 8; ++t) {
      double a;
      int mode = (int)(g() % 4);
      a = std::ldexp(rnd_sig(mode), -(int)(g() % 120)) * S;  // a <= ~S
      a = std::nextafter(a, (g() & 1) ? 0.0 : INFINITY);
      if (a > S) a = S;
      if (g() % 16 == 0) a = S;
      if (!(a >= std::ldexp(1.0, -960))) continue;
      const double q1 = a / S, q2 = mk(a, S, y);
      ++n;
      if (q1 != q2 && bad++ < 10) printf("a=%a S=%a div=%a mk=%a\n", a, S, q1, q2);
    }
  }
  printf("cases %lld mismatches %lld\n", n, bad);
}
