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
}

}  // namespace cdr
