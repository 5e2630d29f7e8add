// Host fuzz: f64sum.hip xfer_pre, integer (significand shifts) vs fp64 (ldexp/floor) form.
// g++ -O2 -o /tmp/fz tools/xfer_pre_fuzz.cpp && /tmp/fz
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <cstring>
#include <random>
constexpr int kENone = -100000;
template <int MB, int kMinE>
void pre_int(double x, int e, long long& q, int& r) {
  unsigned long long bits; memcpy(&bits, &x, 8); bits &= 0x7FFFFFFFFFFFFFFFull;
  const int er = (int)(bits >> 52);
  const unsigned long long mx = er ? ((bits & 0xFFFFFFFFFFFFFull) | (1ull << 52)) : bits;
  const int sh = e - MB - ((er ? er : 1) - 1075);
  const int sc = sh < 0 ? 0 : (sh > 63 ? 63 : sh);
  const long long qi = (long long)(mx >> sc);
  const unsigned long long rem = mx & ((1ull << sc) - 1ull);
  const unsigned long long half = sc ? (1ull << (sc - 1)) : 0ull;
  const bool bad = e == kENone || e < kMinE || !(x >= 0.0) || er == 0x7FF ||
                   (sh < 0 && mx != 0) || !(qi < (1ll << (MB + 1)));
  q = qi; r = (sc > 0 && rem > half ? 1 : 0) | (sc > 0 && rem == half ? 2 : 0) | (bad ? 4 : 0);
}
template <int MB, int kMinE>
void pre_fp(double x, int e, long long& q, int& r) {
  const double y = std::ldexp(x, MB - (e < -2000 ? -2000 : e));
  const double qf = std::floor(y);
  const double fr = y - qf;
  const bool bad = e == kENone || e < kMinE || !(x >= 0.0) || !(y < (double)(1ll << (MB + 1)));
  const double hf = std::floor(std::ldexp(qf, -32));
  const unsigned hi = bad ? 0u : (unsigned)hf;
  const unsigned lo = bad ? 0u : (unsigned)std::fma(hf, -4294967296.0, qf);
  q = (long long)(((unsigned long long)hi << 32) | lo);
  r = (fr > 0.5 ? 1 : 0) | (fr == 0.5 ? 2 : 0) | (bad ? 4 : 0);
}
int main() {
  std::mt19937_64 g(1);
  long long bad = 0, n = 0;
  auto chk = [&](double x, int e) {
    long long q1, q2; int r1, r2;
    pre_int<52, -1022>(x, e, q1, r1); pre_fp<52, -1022>(x, e, q2, r2);
    ++n;
    bool same = (r1 & 4) ? (r2 & 4) : (r1 == r2 && q1 == q2);
    if (!same && bad++ < 10) printf("D x=%a e=%d int q=%lld r=%d fp q=%lld r=%d\n", x, e, q1, r1, q2, r2);
    float xf = (float)x; double xd = xf;
    pre_int<23, -126>(xd, e, q1, r1); pre_fp<23, -126>(xd, e, q2, r2);
    same = (r1 & 4) ? (r2 & 4) : (r1 == r2 && q1 == q2);
    if (!same && bad++ < 10) printf("F x=%a e=%d int q=%lld r=%d fp q=%lld r=%d\n", xd, e, q1, r1, q2, r2);
  };
  std::uniform_int_distribution<int> ed(-1100, 1100), sd(-60, 60);
  for (long long i = 0; i < 20000000; ++i) {
    unsigned long long b = g();
    double x; memcpy(&x, &b, 8);
    int ex; std::frexp(std::fabs(x), &ex);
    int e = (i & 1) ? ed(g) : ex - 1 + sd(g);   // near the value's own binade
    if (i % 7 == 0) x = std::fabs(x);
    if (i % 11 == 0) { x = std::ldexp((double)(g() >> 11), -(int)(g() % 80)); e = (int)(g() % 40) - 20; }
    if (i % 13 == 0) { x = std::ldexp((double)(g() % 1024) + 0.5, (int)(g() % 20) - 10); e = (int)(g() % 30) - 10; }
    if (i % 17 == 0) e = kENone;
    if (i % 19 == 0) x = (g() & 1) ? -0.0 : 0.0;
    if (i % 23 == 0) x = std::ldexp(1.0, -1074) * (double)(g() % 5000);
    chk(x, e);
  }
  chk(INFINITY, 3); chk(NAN, 3); chk(1.0, 1023); chk(1e308, -1022); chk(5e-324, 1023); chk(0.75, -1); chk(0.75, 52);
  printf("cases %lld mismatches %lld\n", n, bad);
}
