// plan32.h — the screen32 plan (fp16 fragments, MFMA C operand, certified
// threshold) built identically on the host (build_plan32,
// screen32.hip) and on the device (plan32_kernel, and ll_finalize right after
// it moves the centroids, loop.hip): the same fp64 operations in the same
// order and one correctly rounded fp16 conversion (f64_to_f16), so both give
// the same bits.
#pragma once
#include "cdr_internal.h"

namespace cdr {

typedef _Float16 plan_h8 __attribute__((ext_vector_type(8)));

// Plan buffer layout (host upload and device plan alike):
//   frag [MT][2][64] h8 | cinit [MT][16][64] f32 | C copy k x d f64 |
//   thr0, D (f32; device plan) | prune block (16-byte aligned):
//   c32 [64][kPrStr] f32 | E [64] f32 | h [64] f32  (screen32p, plan32_prune)
constexpr int kPrStr = 20;  // c32 row stride in floats (16-byte aligned rows)
constexpr size_t kPrBytes = sizeof(float) * (64 * kPrStr + 64 + 64);
struct Plan32Layout {
  size_t cinit, cent, thr, prune, all;
};
__host__ __device__ inline Plan32Layout plan32_layout(int MT, int k, int d) {
  Plan32Layout L;
  L.cinit = (size_t)MT * 2 * 64 * sizeof(plan_h8);
  L.cent = L.cinit + (size_t)MT * 16 * 64 * sizeof(float);
  L.thr = L.cent + sizeof(double) * (size_t)k * d;
  L.prune = (L.thr + 16 + 15) / 16 * 16;
  L.all = L.prune + kPrBytes;
  return L;
}

// Drift-bound buffer (Ctx::bnd, kept by ll_finalize32):
//   W [64] int64 (2^-40 units) | wup [64] f32 | wdn [64] f32   (4-byte words)
//   G [64] int64 (the 2-byte words' per-centroid base: W_j at the last rebase)
//   T [64] u32   the next screen's code thresholds (base G, exponent E0 new)
//   wdg [64] f32 W_j - G_j (new base) rounded down, for the words written now
//   dG [64] f32  G_j(new) - G_j(old) rounded up (0 unless this step rebases)
//   hdr [4] int32: base set, E0 old, E0 new, rebase (zh_rebase_kernel: old -> new)
constexpr size_t kBndWup = 512, kBndWdn = 768, kBndG = 1024, kBndT = 1536, kBndWdg = 1792,
                 kBndDG = 2048, kBndHdr = 2304, kBndBytes = 2320;

// 2-byte bound words (screen32bs): code << 6 | label.  The
// code is a truncated 10-bit float (4 exponent bits from 2^E0, 6 mantissa
// bits) of v = Z - G_label, Z the 4-byte word's value; truncation rounds
// down, so G + dec(code) <= Z.  Code 0: no bound (always fails); 1023: a
// padding row (always kept); real points are clamped to 1022.
constexpr unsigned kZ16Pad = 1023u << 6;
__host__ __device__ inline int zb16_code(float v, int e0) {  // -1: v <= 0 (or NaN)
  if (!(v > 0.0f)) return -1;
  return (int)(__builtin_bit_cast(unsigned, v) >> 17) - ((127 + e0) << 6);
}
__host__ __device__ inline float zb16_dec(int code, int e0) {  // 1 <= code <= 1022
  return __builtin_bit_cast(float, (unsigned)(code + ((127 + e0) << 6)) << 17);
}
// the test threshold of a centroid: a word passes iff code > T, i.e. when
// dec(code) > v >= W_j(t) - G_j (v rounded up)
__host__ __device__ inline unsigned zb16_thr(float v, int e0) {
  if (v != v) return 1022u;
  const int c = zb16_code(v, e0);
  return (unsigned)(c < 0 ? 0 : (c > 1022 ? 1022 : c));
}

// Bound on ||fp16(xhat32) - xhat|| over the point set (screen32p): xhat32 =
// fma(x, 2^sigma, -mu 2^sigma) errs by <= 2^-24 |xhat| (0 when exact) and the
// fp16 rounding by <= 2^-11 |xhat32| + 2^-25 per feature; with dev_f >=
// |xhat_f| (plan32_point_side: xxmax = sum dev_f^2)
// ||h - xhat|| <= (2^-11 + 2^-23) sqrt(xxmax) + 2^-25 sqrt(16).
__host__ __device__ inline double plan32_prune_dn(double xxmax) {
  return ((ldexp(1.0, -11) + ldexp(1.0, -23)) * sqrt(xxmax) + ldexp(1.0, -23)) *
         (1.0 + ldexp(1.0, -20));
}

// From the rounding error e2 = ||c32 - v||^2 and n2 = ||v||^2 of one centroid
// (v = (C - mu) 2^sigma in fp64, within 2^-52 ||v|| of the exact chat):
// ec >= ||c32 - chat||; E >= (dn + ec)(1 + 2^-20) as fp32.
__host__ __device__ inline double plan32_prune_ec(double e2, double n2) {
  return (sqrt(e2) + ldexp(sqrt(n2), -52)) * (1.0 + ldexp(1.0, -40)) + ldexp(1.0, -80);
}
__host__ __device__ inline float plan32_prune_E(double dn, double ec) {
  return (float)((dn + ec) * (1.0 + ldexp(1.0, -20)));
}
// h_r from the smallest squared fp64 distance smin of c32_r to another c32_j
// (exact differences of floats, <= 18 roundings): a lower bound of
// min_j ||chat_r - chat_j|| rounded down into fp32; +inf when k = 1.
__host__ __device__ inline float plan32_prune_h(double smin, double ec_r, double ecmax) {
  if (!(smin < INFINITY)) return INFINITY;
  const double lo = sqrt(smin) * (1.0 - ldexp(1.0, -44)) - ec_r - ecmax;
  return lo > 0.0 ? (float)(lo * (1.0 - ldexp(1.0, -22))) : 0.0f;
}

// Certification constants from the centroid side (ccmax =
// max ||chat||^2, l1c = max ||chat||_1) and the point side.  Shared by the
// host plan (build_plan32) and the device plan (plan32_kernel): the same
// fp64 operations in the same order, so both give the same bits.
__host__ __device__ inline void plan32_bounds(double ccmax, double l1c, double xxmax, double l1x,
                                              int QH, double& D, float& thr0) {
  const double u = ldexp(1.0, -24);
  const int nmfma = QH == 2 ? 3 : 2;
  const double N = 16.0 * nmfma + 1.0;
  // fp32 accumulation inside the MFMA chain, order unknown, each addition
  // erring by at most 2u (no assumption on internal extra precision)
  const double gamma = 2.0 * u * N / (1.0 - 2.0 * u * N);
  // D >= max ||xhat||^2 + margin so that every screen value stays >= 0
  const double E0 = gamma * (2.0 * ccmax + 2.0 * xxmax + 4.0) + 2.4 * ldexp(1.0, -22) *
                    (ccmax + xxmax) + u * (ccmax + 2.0 * xxmax + 4.0) +
                    ldexp(1.0, -24) * (l1c + l1x) + ldexp(1.0, -40);
  D = xxmax + 4.0 * E0 + ldexp(1.0, -20);
  const double sum_abs = (ccmax + D) * (1.0 + u) + (1.0 + ldexp(1.0, -9)) * (ccmax + xxmax);
  const double E = gamma * sum_abs + 2.4 * ldexp(1.0, -22) * (ccmax + xxmax) + u * (ccmax + D) +
                   ldexp(1.0, -24) * (l1c + l1x) + ldexp(1.0, -46) * (ccmax + D);
  // reference slack: the fp64 distances and roots must not tie or flip
  const double Wmax = (sqrt(ccmax) + sqrt(xxmax)) * (sqrt(ccmax) + sqrt(xxmax));
  const double slack = ldexp(Wmax + 1.0, -38);
  thr0 = (float)((2.0 * E + slack) * 1.001);
}

// Fragments of one lane of 32-centroid tile m: A1 = -2 chi, A3 = -2 clo (the
// lane-half quad layout of screen32), and its 16 C-operand values.
__host__ __device__ inline void plan32_lane(const double* ch, const double* cc, double D, int k,
                                            int d, int QH, int m, int lane, plan_h8& A1, plan_h8& A3,
                                            float* cin16) {
  const int h = lane >> 5;
  const int j = 32 * m + (lane & 31);  // A row
  for (int i = 0; i < 8; ++i) {
    A1[i] = (_Float16)0.0f;
    A3[i] = (_Float16)0.0f;
  }
  for (int uq = 0; uq < QH; ++uq) {
    const int q = QH * h + uq;
    for (int i = 0; i < 4; ++i) {
      const int f = 4 * q + i;
      if (j >= k || f >= d) continue;
      const double v = ch[(size_t)j * d + f];
      const _Float16 hi = f64_to_f16(v);
      const _Float16 lo = f64_to_f16(v - (double)hi);
      const _Float16 m2hi = f64_to_f16(-2.0 * (double)hi);
      const _Float16 m2lo = f64_to_f16(-2.0 * (double)lo);
      if (QH == 1) {  // H = [hi(q0), lo(q0)]
        A1[i] = m2hi;
        A1[4 + i] = m2hi;
        A3[i] = m2lo;
      } else {  // H = [hi(q0), hi(q1)], L = [lo(q0), lo(q1)]
        A1[4 * uq + i] = m2hi;
        A3[4 * uq + i] = m2lo;
      }
    }
  }
  for (int i = 0; i < 16; ++i) {
    const int row = 32 * m + 8 * (i >> 2) + 4 * h + (i & 3);
    cin16[i] = row < k ? (float)(cc[row] + D) : 1.0e30f;
  }
}

// One workgroup (>= 256 threads) builds the plan of centroids C (k x d fp64)
// into the plan buffer, laid out as the host upload:
//   frag [MT][2][64] h8 | cinit [MT][16][64] f32 | C copy k x d f64 | thr0 f32.
// The fp16 range guard failing (or a NaN) stops the loop (state[0] = 0) with
// reason 3 (kLLHostPlan): the host then takes that step on the host-plan
// path.  k <= 64, d <= 16 (screen32 shapes).  Every thread must call it.
// Parallel form of build_plan32: the row sums run in the host's order (one
// thread per row), the fp16 halves one thread per element, the maxima by
// wave shuffles (max is exact), the bounds on one lane.
__device__ inline void plan32_build(const double* __restrict__ C, int k, int d, int QH, int MT,
                                    const double* __restrict__ mu, double sc, double xxmax,
                                    double l1x, long long* __restrict__ state,
                                    unsigned char* __restrict__ plan) {
  __shared__ _Float16 m2h[64 * 16], m2l[64 * 16];  // -2 hi, -2 lo of every element
  __shared__ double cc[64];
  __shared__ double sD;
  __shared__ int ok;
  const int t = threadIdx.x;
  double s = 0.0, l1 = 0.0, ca = 0.0;
  if (t < k) {
    for (int f = 0; f < d; ++f) {
      const double v = (C[(size_t)t * d + f] - mu[f]) * sc;
      s += v * v;
      l1 += fabs(v);
      ca = fmax(ca, fabs(v));
    }
    cc[t] = s;
  }
  for (int e = t; e < k * d; e += blockDim.x) {
    const int f = e % d;
    const double v = (C[e] - mu[f]) * sc;
    const _Float16 hi = f64_to_f16(v);
    const _Float16 lo = f64_to_f16(v - (double)hi);
    m2h[e] = f64_to_f16(-2.0 * (double)hi);
    m2l[e] = f64_to_f16(-2.0 * (double)lo);
  }
  if (t < 64) {  // wave 0 holds every row (k <= 64)
    double ccmax = s, l1c = l1, cabs = ca;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      ccmax = fmax(ccmax, __shfl_xor(ccmax, o));
      l1c = fmax(l1c, __shfl_xor(l1c, o));
      cabs = fmax(cabs, __shfl_xor(cabs, o));
    }
    if (t == 0) {
      ok = cabs <= 1024.0;
      if (!ok) {
        state[0] = 0;
        state[2] = 3;  // kLLHostPlan
      } else {
        double D;
        float thr0;
        plan32_bounds(ccmax, l1c, xxmax, l1x, QH, D, thr0);
        sD = D;
        const size_t b_all = (size_t)MT * 2 * 64 * sizeof(plan_h8) +
                             (size_t)MT * 16 * 64 * sizeof(float) + sizeof(double) * (size_t)k * d;
        *reinterpret_cast<float*>(plan + b_all) = thr0;
        reinterpret_cast<float*>(plan + b_all)[1] = (float)D;  // (the hi-only screen's bound)
      }
    }
  }
  __syncthreads();
  if (!ok) return;
  const size_t b_frag = (size_t)MT * 2 * 64 * sizeof(plan_h8);
  const size_t b_cinit = (size_t)MT * 16 * 64 * sizeof(float);
  plan_h8* frag = reinterpret_cast<plan_h8*>(plan);
  float* cinit = reinterpret_cast<float*>(plan + b_frag);
  double* cent = reinterpret_cast<double*>(plan + b_frag + b_cinit);
  for (int idx = t; idx < MT * 64; idx += blockDim.x) {  // the layout of plan32_lane
    const int m = idx >> 6, lane = idx & 63;
    const int h = lane >> 5, j = 32 * m + (lane & 31);
    plan_h8 A1, A3;
    for (int i = 0; i < 8; ++i) {
      A1[i] = (_Float16)0.0f;
      A3[i] = (_Float16)0.0f;
    }
    for (int uq = 0; uq < QH; ++uq)
      for (int i = 0; i < 4; ++i) {
        const int f = 4 * (QH * h + uq) + i;
        if (j >= k || f >= d) continue;
        const _Float16 a = m2h[j * d + f], b = m2l[j * d + f];
        if (QH == 1) {
          A1[i] = a;
          A1[4 + i] = a;
          A3[i] = b;
        } else {
          A1[4 * uq + i] = a;
          A3[4 * uq + i] = b;
        }
      }
    frag[(m * 2 + 0) * 64 + lane] = A1;
    frag[(m * 2 + 1) * 64 + lane] = A3;
  }
  for (int idx = t; idx < MT * 16 * 64; idx += blockDim.x) {
    const int lane = idx & 63, mi = idx >> 6, m = mi >> 4, i = mi & 15;
    const int row = 32 * m + 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3);
    cinit[idx] = row < k ? (float)(cc[row] + sD) : 1.0e30f;
  }
  for (int i = t; i < k * d; i += blockDim.x) cent[i] = C[i];
  // prune block (screen32p): fp32 centroids, their bounds, nearest-centroid
  // distances (the host's build_plan32 computes the same quantities)
  const Plan32Layout L = plan32_layout(MT, k, d);
  float* pc = reinterpret_cast<float*>(plan + L.prune);
  float* pE = pc + 64 * kPrStr;
  float* ph = pE + 64;
  __shared__ float c32[64 * 16];
  __shared__ double pec[64];
  __shared__ unsigned long long smin_b[64], ecmax_b;
  if (t == 0) ecmax_b = 0ull;
  for (int e = t; e < 64 * kPrStr; e += blockDim.x) {
    const int j = e / kPrStr, f = e - j * kPrStr;
    float cf = 0.0f;
    if (j < k && f < d) cf = (float)((C[(size_t)j * d + f] - mu[f]) * sc);
    pc[e] = cf;
    if (f < 16) c32[j * 16 + f] = cf;
  }
  if (t < 64) smin_b[t] = __double_as_longlong(INFINITY);
  __syncthreads();
  if (t < 64) {
    double e2 = 0.0, n2 = 0.0;
    if (t < k)
      for (int f = 0; f < d; ++f) {
        const double v = (C[(size_t)t * d + f] - mu[f]) * sc;
        const double r = (double)c32[t * 16 + f] - v;  // exact
        e2 += r * r;
        n2 += v * v;
      }
    const double ec = plan32_prune_ec(e2, n2);
    pec[t] = ec;
    pE[t] = plan32_prune_E(plan32_prune_dn(xxmax), ec);
    if (t < k) atomicMax(&ecmax_b, (unsigned long long)__double_as_longlong(ec));
  }
  {  // row r = t % 64, columns j = t / 64 + G i: the smallest squared distance
    const int r = t & 63, G = blockDim.x >> 6;
    double sm = INFINITY;
    if (r < k)
      for (int j = t >> 6; j < k; j += G) {
        if (j == r) continue;
        double s2 = 0.0;
        for (int f = 0; f < 16; ++f) {
          const double df = (double)c32[r * 16 + f] - (double)c32[j * 16 + f];
          s2 += df * df;
        }
        sm = fmin(sm, s2);
      }
    atomicMin(&smin_b[r], (unsigned long long)__double_as_longlong(sm));  // >= 0: bits order
  }
  __syncthreads();
  if (t < 64)
    ph[t] = t < k ? plan32_prune_h(__longlong_as_double(smin_b[t]), pec[t],
                                   __longlong_as_double(ecmax_b))
                  : INFINITY;
}

}  // namespace cdr
