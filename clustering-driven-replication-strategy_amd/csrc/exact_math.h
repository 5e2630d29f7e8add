// exact_math.h — device functions that reproduce NumPy's float64 reduction
// orders bit for bit.  The whole library is compiled with -ffp-contract=off,
// so `a * b + c` below is a rounded multiply followed by a rounded add, as in
// NumPy; fused operations are written explicitly (fma/fmaf) where wanted.
//
// pw_d: np.add.reduce over a contiguous run of m <= 128 float64 values, i.e.
// numpy/_core/src/umath/loops_utils.h.src pairwise_sum for n <= PW_BLOCKSIZE:
//   m < 8  : ((0 + s0) + s1) + ...                     (sequential)
//   m >= 8 : r[j] = s[j]; r[j] += s[8i + j] (i = 1..);
//            ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)); then the m % 8 tail in order.
// This is the order np.linalg.norm(X[:, None, :] - C[None], axis=2) sums the
// squared differences in (reference src/kmeans_plusplus.py:15 and :33); the
// oracle checks it against NumPy itself (tests/test_oracle.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cdr {

// Squared Euclidean distance in NumPy order.  `xv(f)` returns feature f of
// the point, `cv(f)` of the centroid; R is the arithmetic (double, or float
// for the reference's float32 runs: every difference, square and sum rounded
// to fp32 as NumPy does on float32 arrays).  Requires d <= 128.
template <typename XF, typename CF, typename R = double>
__device__ __forceinline__ R np_sqdist(XF xv, CF cv, int d) {
  if (d < 8) {
    R res = 0.0;
    for (int f = 0; f < d; ++f) {
      const R t = (R)xv(f) - (R)cv(f);
      res = res + t * t;
    }
    return res;
  }
  R r0, r1, r2, r3, r4, r5, r6, r7;
  {
    R t;
    t = (R)xv(0) - (R)cv(0); r0 = t * t;
    t = (R)xv(1) - (R)cv(1); r1 = t * t;
    t = (R)xv(2) - (R)cv(2); r2 = t * t;
    t = (R)xv(3) - (R)cv(3); r3 = t * t;
    t = (R)xv(4) - (R)cv(4); r4 = t * t;
    t = (R)xv(5) - (R)cv(5); r5 = t * t;
    t = (R)xv(6) - (R)cv(6); r6 = t * t;
    t = (R)xv(7) - (R)cv(7); r7 = t * t;
  }
  const int dd = d - (d & 7);
  for (int f = 8; f < dd; f += 8) {
    R t;
    t = (R)xv(f + 0) - (R)cv(f + 0); r0 = r0 + t * t;
    t = (R)xv(f + 1) - (R)cv(f + 1); r1 = r1 + t * t;
    t = (R)xv(f + 2) - (R)cv(f + 2); r2 = r2 + t * t;
    t = (R)xv(f + 3) - (R)cv(f + 3); r3 = r3 + t * t;
    t = (R)xv(f + 4) - (R)cv(f + 4); r4 = r4 + t * t;
    t = (R)xv(f + 5) - (R)cv(f + 5); r5 = r5 + t * t;
    t = (R)xv(f + 6) - (R)cv(f + 6); r6 = r6 + t * t;
    t = (R)xv(f + 7) - (R)cv(f + 7); r7 = r7 + t * t;
  }
  R res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (int f = dd; f < d; ++f) {
    const R t = (R)xv(f) - (R)cv(f);
    res = res + t * t;
  }
  return res;
}

// Leaf of NumPy's pairwise_sum over a[0..m), m <= 128 (same orders as above).
template <typename AF, typename R = double>
__device__ __forceinline__ R np_pw_leaf(AF a, int m) {
  if (m < 8) {
    R res = 0.0;
    for (int i = 0; i < m; ++i) res = res + (R)a(i);
    return res;
  }
  R r0 = a(0), r1 = a(1), r2 = a(2), r3 = a(3), r4 = a(4), r5 = a(5), r6 = a(6), r7 = a(7);
  const int mm = m - (m & 7);
  for (int i = 8; i < mm; i += 8) {
    r0 = r0 + (R)a(i + 0); r1 = r1 + (R)a(i + 1); r2 = r2 + (R)a(i + 2); r3 = r3 + (R)a(i + 3);
    r4 = r4 + (R)a(i + 4); r5 = r5 + (R)a(i + 5); r6 = r6 + (R)a(i + 6); r7 = r7 + (R)a(i + 7);
  }
  R res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (int i = mm; i < m; ++i) res = res + (R)a(i);
  return res;
}

// Full pairwise_sum over a[0..n) for any n (recursion split n2 = n/2 - (n/2)%8,
// leaves <= 128), evaluated by one thread with an explicit stack.
template <typename AF, typename R = double>
__device__ R np_pairwise(AF a, int64_t n) {
  if (n <= 128) return np_pw_leaf<AF, R>(a, (int)n);
  struct Frame {
    int64_t off, n;
    int state;  // 0 = not split yet, 1 = left pending, 2 = right pending
    R left;
  };
  Frame st[48];
  int sp = 0;
  st[0] = {0, n, 0, (R)0.0};
  R ret = 0.0;
  bool have_ret = false;
  while (sp >= 0) {
    Frame& fr = st[sp];
    if (have_ret) {
      if (fr.state == 1) {
        fr.left = ret;
        fr.state = 2;
        have_ret = false;
        int64_t n2 = fr.n / 2;
        n2 -= n2 % 8;
        st[sp + 1] = {fr.off + n2, fr.n - n2, 0, (R)0.0};
        ++sp;
      } else {  // state 2: both halves done
        ret = fr.left + ret;
        --sp;
      }
      continue;
    }
    if (fr.n <= 128) {
      const int64_t off = fr.off;
      auto leaf = [&](int i) { return a(off + i); };
      ret = np_pw_leaf<decltype(leaf), R>(leaf, (int)fr.n);
      have_ret = true;
      --sp;
      continue;
    }
    int64_t n2 = fr.n / 2;
    n2 -= n2 % 8;
    fr.state = 1;
    st[sp + 1] = {fr.off, n2, 0, (R)0.0};
    ++sp;
  }
  return ret;
}

// np.argmin of the fp64 NumPy-order norms (src/kmeans_plusplus.py:33-34):
// the first index of the smallest correctly rounded root; a root is taken
// only for a smaller square (sqrt is monotone).
template <typename XF>
__device__ __forceinline__ int exact_argmin(XF xv, const double* __restrict__ C, int k,
                                            int d) {
  double Rb = INFINITY, rb = INFINITY;
  int jb = 0;
  for (int j = 0; j < k; ++j) {
    const double* cj = C + (size_t)j * d;
    const double R = np_sqdist(xv, [&](int f) { return cj[f]; }, d);
    if (R < Rb) {
      const double r = sqrt(R);
      if (r < rb) {
        rb = r;
        Rb = R;
        jb = j;
      }
    }
  }
  return jb;
}

}  // namespace cdr
