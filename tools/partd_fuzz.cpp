// Host fuzz: csrc/seed.hip part_add (int64 run counts) vs partd_add (fp64 integer counts + parity bits).
// g++ -O2 -o /tmp/pd tools/partd_fuzz.cpp && /tmp/pd
#include <cstdio>
#include <cmath>
#include <cstring>
#include <cstdint>
#include <random>
constexpr int kNoE = -100000; constexpr long long kD52 = 1ll << 52;
struct Part { long long d0, d1; int e, st; };
static void part_add(Part& P, double p, int e) {
  if (P.st == 0) P = Part{0, 0, e, 1};
  if (P.st != 1) return;
  if (P.e != e) { P.st = 2; return; }
  const double f = std::ldexp(p, 52 - e);
  if (!(f < 4503599627370496.0)) { P.st = 2; return; }
  const double fl = std::floor(f); const double frac = f - fl;
  const long long k = (long long)fl; const long long up = frac > 0.5 ? 1 : 0; const bool tie = frac == 0.5;
  P.d0 += k + up + ((tie && ((P.d0 ^ k) & 1)) ? 1 : 0);
  P.d1 += k + up + ((tie && ((1 ^ P.d1 ^ k) & 1)) ? 1 : 0);
  if (P.d0 >= kD52 || P.d1 >= kD52) P.st = 2;
}
struct PartD { double d0, d1; int p0, p1; int e, st; };
static long long bits(double x) { long long b; memcpy(&b, &x, 8); return b; }
static void partd_add(PartD& P, double p, int e) {
  if (P.st == 0) P = PartD{0.0, 0.0, 0, 0, e, 1};
  if (P.st != 1) return;
  if (P.e != e) { P.st = 2; return; }
  const double f = std::ldexp(p, 52 - e);
  if (!(f < 4503599627370496.0)) { P.st = 2; return; }
  const double fl = std::floor(f); const double frac = f - fl;
  const int kp = (int)(bits(fl + 4503599627370496.0) & 1);
  const int up = frac > 0.5 ? 1 : 0; const int tie = frac == 0.5 ? 1 : 0;
  const int i0 = up | (tie & (P.p0 ^ kp)); const int i1 = up | (tie & (1 ^ P.p1 ^ kp));
  P.d0 = (P.d0 + fl) + (double)i0; P.d1 = (P.d1 + fl) + (double)i1;
  P.p0 ^= kp ^ i0; P.p1 ^= kp ^ i1;
  if (P.d0 >= 4503599627370496.0 || P.d1 >= 4503599627370496.0) P.st = 2;
}
int main() {
  std::mt19937_64 g(3); long long bad = 0, n = 0;
  for (int it = 0; it < 3000000; ++it) {
    const int e = (int)(g() % 60) - 50;
    Part P{0, 0, kNoE, 0}; PartD Q{0, 0, 0, 0, kNoE, 0};
    const int len = 1 + (int)(g() % 40);
    const int mode = (int)(g() % 4);
    for (int i = 0; i < len; ++i) {
      double p;
      if (mode == 0) p = std::ldexp((double)(g() >> 11), -53) * std::ldexp(1.0, e - (int)(g() % 30));
      else if (mode == 1) p = std::ldexp((double)(g() % 4096) + 0.5 * (g() & 1), e - 52);   // ties
      else if (mode == 2) p = std::ldexp((double)(g() >> 11), -53) * std::ldexp(1.0, e + 1 - (int)(g() % 3));
      else p = std::ldexp((double)((g() >> 12) | 1), e - 52 - 52 + (int)(g() % 60));
      int ee = (g() % 50 == 0) ? e + 1 : e;
      part_add(P, p, ee); partd_add(Q, p, ee); ++n;
      const bool same = P.st == Q.st && P.e == Q.e && (P.st != 1 || (P.d0 == (long long)Q.d0 && P.d1 == (long long)Q.d1));
      if (!same && bad++ < 10) printf("mismatch it=%d i=%d st %d/%d d0 %lld/%.0f d1 %lld/%.0f\n", it, i, P.st, Q.st, P.d0, Q.d0, P.d1, Q.d1);
    }
  }
  printf("adds %lld mismatches %lld\n", n, bad);
}
