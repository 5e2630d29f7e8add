// seed.hip — k-means++ D^2 seeding (reference src/kmeans_plusplus.py:3-22).
//
// Per step i (one new centre c):
//   dist_sq = min(dist_sq, norm(X - c)**2)        :14-17  (running min is exact:
//                                                         min is order free)
//   total   = dist_sq.sum()                        :18     NumPy add.reduce: 8192-
//             element chunks, pairwise inside each chunk, chunks added left to right
//   idx     = rng.choice(n, p=dist_sq/total)       :19     = searchsorted(cumsum(p) /
//             cumsum(p)[-1], rng.random(), 'right') (one draw; u comes from host)
//
// The cumulative sum is where a parallel scan would change the rounding.  We
// emulate NumPy's strictly sequential fp64 accumulation exactly:
//   while the running value c stays inside one binade [2^e, 2^(e+1)), every
//   fl(c + p) lands on the grid g = 2^(e-52), so c/g = N is an integer and
//   N' = N + rne(p/g) — independent of N except for exact ties, where round-
//   half-even looks at the parity of N.  A run of elements is therefore a
//   *transfer* (D0, D1): the increment of N when N enters even / odd.  Two
//   transfers compose as D_q = L_q + R_{q ^ (L_q & 1)} (associative), so
//   blocks are reduced in parallel; a single wave then walks the blocks,
//   applying whole blocks inside a binade and walking element by element only
//   across the ~log2(c_last/c_first) binade crossings.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "cdr_internal.h"
#include "exact_math.h"

namespace cdr {

struct Xfer {
  long long d0, d1;
  int e;      // binade exponent the transfer was computed for
  int valid;  // 0: some element would leave the binade / overflow
  long long pad;
};

constexpr int kSub = 128;  // elements per lane in a block (8192 = 64 x 128)

__global__ void fill_inf(double* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = INFINITY;
}

// Pairwise tree skeleton of NumPy's pairwise_sum with leaves produced by a
// functor leaf(off, m) (m <= 128) — same recursion as np_pairwise.
template <typename LF>
__device__ double pw_tree(int64_t n, LF leaf) {
  if (n <= 128) return leaf((int64_t)0, (int)n);
  struct Frame {
    int64_t off, n;
    int state;
    double left;
  };
  Frame st[48];
  int sp = 0;
  st[0] = {0, n, 0, 0.0};
  double ret = 0.0;
  bool have = false;
  while (sp >= 0) {
    Frame& fr = st[sp];
    if (have) {
      if (fr.state == 1) {
        fr.left = ret;
        fr.state = 2;
        have = false;
        int64_t n2 = fr.n / 2;
        n2 -= n2 % 8;
        st[sp + 1] = {fr.off + n2, fr.n - n2, 0, 0.0};
        ++sp;
      } else {
        ret = fr.left + ret;
        --sp;
      }
      continue;
    }
    if (fr.n <= 128) {
      ret = leaf(fr.off, (int)fr.n);
      have = true;
      --sp;
      continue;
    }
    int64_t n2 = fr.n / 2;
    n2 -= n2 % 8;
    fr.state = 1;
    st[sp + 1] = {fr.off, n2, 0, 0.0};
    ++sp;
  }
  return ret;
}

// One workgroup (256 threads) per 8192-point block.  The block is handled in
// two halves of 4096 (pw(8192) = pw(4096) + pw(4096)); each half's values sit
// in LDS (one pad slot per 16).
//
// Full blocks (TAIL = false): the 32 pairwise leaves of 128 of a half are
// summed by 8 threads each — thread (leaf L, j) adds NumPy's accumulator r_j
// = a(j) + a(j + 8) + ... sequentially, shfl_xor 1, 2, 4 forms
// ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), shfl_xor 8, 16, 32 and
// then a 4-wave LDS step combine the leaves in the balanced tree of
// pw(4096).
// TAIL = true: the one partial block (m < 8192) at b_off; its pairwise tree
// is enumerated by one thread (a stack: scratch memory, kept out of the
// full-block kernel).
// D > 0 (float points, d == D <= 16): each thread takes 4 points per
// iteration with all their 16-byte feature-quad loads and dmin loads issued
// before any arithmetic, and the NumPy-order distance unrolled for that d.
// Exact pruning of the running minimum (the k-means++ D^2 step,
// src/kmeans_plusplus.py:14-17): the point's nearest centre so far, c_a =
// near[i], is at distance r with dmin = fl(r^2); if the new centre is at
// least 2 r (1 + 2^-30) from c_a, the triangle inequality puts it at least
// r (1 + 2^-30) from the point, so its computed squared distance (NumPy
// order, relative error < 2^-45 at d <= 128) is >= dmin and min(dmin, .)
// leaves dmin unchanged bit for bit: the point is not read at all.
// ccd[j] = ||c_j - c_new|| (fp64, relative error < 2^-48).  dmin = +inf (no
// centre yet) never prunes.
__device__ __forceinline__ bool seed_prunable(double ccd_a, double dmin_old) {
  return ccd_a >= 2.0 * sqrt(dmin_old) * (1.0 + 0x1p-30);
}

// ccd[j] = ||cents[j] - cen|| for the j < count centres so far.
__global__ void seed_ccd_kernel(const double* __restrict__ cents, int count, int d,
                                const double* __restrict__ cen, double* __restrict__ ccd) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < count; j += gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int f = 0; f < d; ++f) {
      const double t = cents[(size_t)j * d + f] - cen[f];
      s += t * t;
    }
    ccd[j] = sqrt(s);
  }
}

template <typename T, int D, bool TAIL>
__global__ __launch_bounds__(256) void seed_update_kernel(
    const T* __restrict__ X, int64_t n, int64_t n_pad, int d, const double* __restrict__ cen,
    double* __restrict__ dmin, double* __restrict__ blocksums, int64_t b_off,
    int32_t* __restrict__ near, const double* __restrict__ ccd, int cidx) {
  constexpr int kHalf = 4096;
  __shared__ double sdm[kHalf + kHalf / 16];
  __shared__ double swave[4];
  const int64_t b = blockIdx.x + b_off;
  const int64_t base = b * kSeedBlock;
  const int m = TAIL ? (int)(n - base) : kSeedBlock;
  auto spos = [](int q) { return q + (q >> 4); };
  double halves[2] = {0.0, 0.0};
  for (int h = 0; h < 2; ++h) {
    if constexpr (D > 0) {
      constexpr int Q = (D + 3) / 4;
      typedef float f4v __attribute__((ext_vector_type(4)));
      const f4v* X4 = reinterpret_cast<const f4v*>(X);
      double cr[D];
#pragma unroll
      for (int f = 0; f < D; ++f) cr[f] = cen[f];
      for (int q0 = threadIdx.x; q0 < kHalf; q0 += 4 * 256) {
        f4v xv[4][Q];
        double old[4];
        bool go[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int qi = h * kHalf + q0 + 256 * u;
          const int64_t i = base + qi;
          go[u] = false;
          if (!TAIL || qi < m) {
            old[u] = dmin[i];
            go[u] = cidx == 0 || !seed_prunable(ccd[near[i]], old[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t i = base + h * kHalf + q0 + 256 * u;
          if (go[u]) {
#pragma unroll
            for (int qq = 0; qq < Q; ++qq) xv[u][qq] = X4[(int64_t)qq * n_pad + i];
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int q = q0 + 256 * u;
          const int qi = h * kHalf + q;
          double v = 0.0;
          if (!TAIL || qi < m) {
            v = old[u];
            if (go[u]) {
              auto xf = [&](int f) { return (double)xv[u][f >> 2][f & 3]; };
              auto cf = [&](int f) { return cr[f]; };
              const double R = np_sqdist(xf, cf, D);
              const double r = sqrt(R);
              const double t = r * r;
              if (t < old[u]) {
                v = t;
                dmin[base + qi] = t;
                near[base + qi] = cidx;
              }
            }
          }
          sdm[spos(q)] = v;
        }
      }
    } else {
      for (int q = threadIdx.x; q < kHalf; q += blockDim.x) {
        const int qi = h * kHalf + q;
        const int64_t i = base + qi;
        double v = 0.0;
        if (!TAIL || qi < m) {
          const double old = dmin[i];
          v = old;
          if (cidx == 0 || !seed_prunable(ccd[near[i]], old)) {
            auto xv = [&](int f) { return (double)X[xidx(f, i, n_pad)]; };
            auto cv = [&](int f) { return cen[f]; };
            const double R = np_sqdist(xv, cv, d);
            const double r = sqrt(R);
            const double t = r * r;
            if (t < old) {
              v = t;
              dmin[i] = t;
              near[i] = cidx;
            }
          }
        }
        sdm[spos(q)] = v;
      }
    }
    __syncthreads();
    if constexpr (!TAIL) {
      const int t = threadIdx.x;
      const int L = t >> 3, j = t & 7;
      double r = sdm[spos(128 * L + j)];
#pragma unroll
      for (int i = 1; i < 16; ++i) r = r + sdm[spos(128 * L + j + 8 * i)];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) r = r + __shfl_xor(r, o);
      if ((t & 63) == 0) swave[t >> 6] = r;
      __syncthreads();
      if (t == 0) halves[h] = (swave[0] + swave[1]) + (swave[2] + swave[3]);
      __syncthreads();
    }
  }
  if constexpr (!TAIL) {
    if (threadIdx.x == 0) blocksums[b] = halves[0] + halves[1];
  } else {
    __shared__ double sleaf[160];
    __shared__ int soff[160], slen[160];
    __shared__ int sleaves;
    // partial (last) block: enumerate the pairwise leaves, sum them in
    // parallel from global memory, combine in tree order.
    __threadfence_block();
    __syncthreads();
    if (threadIdx.x == 0) {
      int cnt = 0;
      pw_tree((int64_t)m, [&](int64_t off, int len) {
        soff[cnt] = (int)off;
        slen[cnt] = len;
        ++cnt;
        return 0.0;
      });
      sleaves = cnt;  // <= 128 leaves of (64, 128] elements for m < 8192
    }
    __syncthreads();
    const int cnt = sleaves;
    if (threadIdx.x < cnt) {
      const int off = soff[threadIdx.x], len = slen[threadIdx.x];
      sleaf[threadIdx.x] = np_pw_leaf([&](int i) { return dmin[base + off + i]; }, len);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int cur = 0;
      blocksums[b] = pw_tree((int64_t)m, [&](int64_t, int) { return sleaf[cur++]; });
    }
  }
}

// ---- cumulative-sum emulation --------------------------------------------

__device__ __forceinline__ void compose(long long L0, long long L1, long long R0, long long R1,
                                        long long& o0, long long& o1) {
  o0 = L0 + ((L0 & 1) ? R1 : R0);
  o1 = L1 + ((L1 & 1) ? R0 : R1);
}

// Transfer of elements [lo, hi) (values v(i)) under binade exponent e.
template <typename V>
__device__ __forceinline__ void range_transfer_v(V v, double S, int64_t lo, int64_t hi, int e,
                                                 long long& D0, long long& D1, int& valid) {
  D0 = 0;
  D1 = 0;
  valid = 1;
  for (int64_t i = lo; i < hi; ++i) {
    const double p = v(i) / S;
    const double f = ldexp(p, 52 - e);
    if (!(f < 4503599627370496.0)) {  // >= 2^52 (or NaN): leaves the binade
      valid = 0;
      continue;
    }
    const double fl = floor(f);
    const double frac = f - fl;
    const long long k = (long long)fl;
    const long long up = frac > 0.5 ? 1 : 0;
    const bool tie = frac == 0.5;
    // incoming parity q = 0
    {
      const long long par = (D0 ^ k) & 1;  // parity of N + fl with N even + D0
      D0 += k + up + ((tie && par) ? 1 : 0);
    }
    {
      const long long par = (1 ^ D1 ^ k) & 1;
      D1 += k + up + ((tie && par) ? 1 : 0);
    }
  }
  if (D0 >= (1ll << 52) || D1 >= (1ll << 52)) valid = 0;
}

__device__ void range_transfer(const double* __restrict__ dmin, double S, int64_t lo,
                               int64_t hi, int e, long long& D0, long long& D1, int& valid) {
  range_transfer_v([&](int64_t i) { return dmin[i]; }, S, lo, hi, e, D0, D1, valid);
}

__device__ __forceinline__ bool binade_of(double c, int& e, long long& N) {
  const unsigned long long bits = __double_as_longlong(c);
  const int ef = (int)((bits >> 52) & 0x7FF);
  if (ef == 0 || ef >= 2046 || (bits >> 63)) return false;  // zero/subnormal/huge/neg
  e = ef - 1023;
  N = (long long)((bits & 0xFFFFFFFFFFFFFull) | (1ull << 52));
  return true;
}
__device__ __forceinline__ double from_binade(int e, long long N) {
  const unsigned long long bits =
      ((unsigned long long)(e + 1023) << 52) | ((unsigned long long)N & 0xFFFFFFFFFFFFFull);
  return __longlong_as_double(bits);
}

// Per-block transfers under the guessed binade of the block's start.  One
// wave per 8192-element block, in 8 passes of 1024: the pass is loaded
// coalesced (16 B per lane per load) into LDS with one pad slot per 16
// elements, then lane l walks elements [16 l, 16 l + 16) of the pass from LDS
// (conflict-free ds_read_b64), the 64 lane transfers are composed in order and
// the pass transfer is composed onto the block's.
constexpr int kPass = 1024;
constexpr int kPassPad = kPass + kPass / 16;

__global__ __launch_bounds__(256) void xfer_kernel(const double* __restrict__ dmin, int64_t n,
                                                   double S, const double* __restrict__ approx,
                                                   int64_t nblocks, Xfer* __restrict__ out) {
  __shared__ double sbuf[4][kPassPad];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t b = (int64_t)blockIdx.x * 4 + w;
  const bool live = b < nblocks;
  double* sb = sbuf[w];
  int e = 0;
  long long Ndummy;
  const bool okg = live && binade_of(approx[b], e, Ndummy);
  const int64_t base = b * kSeedBlock;
  long long T0 = 0, T1 = 0;
  int tv = okg ? 1 : 0;
  for (int ps = 0; ps < kSeedBlock / kPass; ++ps) {
    const int64_t pb = base + (int64_t)ps * kPass;
    const bool act = okg && pb < n;  // wave-uniform
    if (act) {
      // dmin is allocated to n_pad (a multiple of the block): whole passes load
      const double2* src = reinterpret_cast<const double2*>(dmin + pb);
#pragma unroll
      for (int j = 0; j < kPass / 128; ++j) {
        const double2 v = src[j * 64 + lane];
        const int el = j * 128 + 2 * lane;
        const int pos = el + (el >> 4);
        sb[pos] = v.x;
        sb[pos + 1] = v.y;
      }
    }
    __syncthreads();
    if (act) {
      const int64_t lo = pb + (int64_t)lane * 16;
      const int64_t hi = (lo + 16) < n ? (lo + 16) : n;
      long long D0 = 0, D1 = 0;
      int valid = 1;
      const double* sl = sb + lane * 17;
      if (lo < hi)
        range_transfer_v([&](int64_t i) { return sl[i - lo]; }, S, lo, hi, e, D0, D1, valid);
      // ordered reduction over lanes: lane l absorbs lane l+o
      for (int o = 1; o < 64; o <<= 1) {
        const long long r0 = __shfl_down(D0, o), r1 = __shfl_down(D1, o);
        const int rv = __shfl_down(valid, o);
        if ((lane & (2 * o - 1)) == 0 && lane + o < 64) {
          long long n0, n1;
          compose(D0, D1, r0, r1, n0, n1);
          D0 = n0;
          D1 = n1;
          valid &= rv;
        }
      }
      long long n0, n1;
      compose(T0, T1, D0, D1, n0, n1);
      tv &= valid;
      // saturate: keeps the composition of later passes from overflowing
      if (n0 >= (1ll << 52) || n1 >= (1ll << 52)) {
        tv = 0;
        n0 = n1 = 0;
      }
      T0 = n0;
      T1 = n1;
    }
    __syncthreads();
  }
  if (live && lane == 0) out[b] = Xfer{T0, T1, e, tv, 0};
}

// approx[b] = c_in + sum_{b' < b} blocksums[b'] / S   (guesses only)
__global__ __launch_bounds__(1024) void approx_prefix_kernel(const double* __restrict__ bs,
                                                             int64_t nb, double S, double c_in,
                                                             double* __restrict__ approx) {
  __shared__ double part[1024];
  const int t = threadIdx.x;
  const int64_t per = (nb + 1023) / 1024;
  const int64_t lo = t * per, hi = (lo + per) < nb ? (lo + per) : nb;
  double s = 0.0;
  for (int64_t i = lo; i < hi; ++i) s += bs[i] / S;
  part[t] = s;
  __syncthreads();
  if (t == 0) {
    double acc = c_in;
    for (int i = 0; i < 1024; ++i) {
      const double v = part[i];
      part[i] = acc;
      acc += v;
    }
  }
  __syncthreads();
  double acc = part[t];
  for (int64_t i = lo; i < hi; ++i) {
    approx[i] = acc;
    acc += bs[i] / S;
  }
}

// Wave-parallel exact walk of elements [lo, hi) starting from running value c.
// If `search`, stops at the first element m with fl(c_m / c_last) > u and
// returns its index in *found (else *found stays -1).  Returns the running
// value after the last element processed.  Executed by all 64 lanes of a
// single-wave workgroup (it synchronises the workgroup).
//
// The range is taken in segments of 4096: p = fl(dmin / S) of the segment is
// staged in LDS (coalesced loads, one pad slot per 64 so that lane l's
// sub-chunk [64 l, 64 l + 64) reads conflict-free), then sub-chunk transfers
// are applied in bulk while they stay in the binade and the sub-chunk that
// leaves it is walked element by element.
constexpr int kSeg = 4096;
constexpr int kSegSub = kSeg / 64;

__device__ double fine_walk(const double* __restrict__ dmin, double S, int64_t lo, int64_t hi,
                            double c, bool search, double c_last, double u, int64_t* found) {
  __shared__ double sp[kSeg + kSeg / kSegSub];
  const int lane = threadIdx.x & 63;
  for (int64_t s0 = lo; s0 < hi; s0 += kSeg) {
    const int m = (int)((hi - s0) < kSeg ? (hi - s0) : kSeg);
    __syncthreads();  // the previous segment's reads are done
    if (m == kSeg && (s0 & 1) == 0) {
      // whole segment: 32 independent 16-byte loads per lane in flight
      // (a rolled load/divide/store loop would pay the full HBM latency per
      // element pair)
      const double2* src = reinterpret_cast<const double2*>(dmin + s0);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double2 v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = src[(h * 16 + j) * 64 + lane];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int i = ((h * 16 + j) * 64 + lane) * 2;
          sp[i + i / kSegSub] = v[j].x / S;
          sp[i + 1 + (i + 1) / kSegSub] = v[j].y / S;
        }
      }
    } else {
      for (int i0 = 0; i0 < m; i0 += 64 * 8) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = i0 + j * 64 + lane;
          v[j] = i < m ? dmin[s0 + i] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = i0 + j * 64 + lane;
          if (i < m) sp[i + i / kSegSub] = v[j] / S;
        }
      }
    }
    __syncthreads();
    auto pv = [&](int i) { return sp[i + i / kSegSub]; };
    int pos = 0;
    while (pos < m) {
      int e;
      long long N;
      const bool inb = binade_of(c, e, N);
      int L = 0;  // sub-chunks applied in bulk
      if (inb) {
        const int slo = pos + lane * kSegSub;
        const int shi = (slo + kSegSub) < m ? (slo + kSegSub) : m;
        long long D0 = 0, D1 = 0;
        int valid = 1;
        if (slo < m)
          range_transfer_v([&](int64_t i) { return pv((int)i); }, 1.0, slo, shi, e, D0, D1,
                           valid);
        else
          valid = 0;
        // inclusive ordered prefix over lanes
        for (int o = 1; o < 64; o <<= 1) {
          const long long l0 = __shfl_up(D0, o), l1 = __shfl_up(D1, o);
          const int lv = __shfl_up(valid, o);
          if (lane >= o) {
            long long n0, n1;
            compose(l0, l1, D0, D1, n0, n1);
            D0 = n0;
            D1 = n1;
            valid &= lv;
          }
        }
        const long long Dq = (N & 1) ? D1 : D0;
        const long long Nend = N + Dq;
        bool ok = valid && slo < m && Dq < (1ll << 52) && Nend < (1ll << 53);
        bool hit = false;
        if (ok && search) hit = (from_binade(e, Nend) / c_last) > u;
        const unsigned long long okm = __ballot(ok && !hit);
        // number of leading lanes that are ok and not yet past the target
        L = (okm == ~0ull) ? 64 : __builtin_ctzll(~okm);
        if (L > 0) {
          const long long DL = __shfl(Dq, L - 1);
          c = from_binade(e, N + DL);
          pos += L * kSegSub;
          if (pos > m) pos = m;
        }
        if (pos >= m) break;
        if (L == 64) continue;  // every sub-chunk applied: next bulk round
      }
      // element-wise over (at most) one sub-chunk; lane 0 computes, broadcasts
      const int ehi = (pos + kSegSub) < m ? (pos + kSegSub) : m;
      double cc = c;
      int hitidx = -1;
      if (lane == 0) {
        for (int i = pos; i < ehi; ++i) {
          cc = cc + pv(i);
          if (search && (cc / c_last) > u) {
            hitidx = i;
            break;
          }
        }
      }
      cc = __shfl(cc, 0);
      hitidx = __shfl(hitidx, 0);
      c = cc;
      if (hitidx >= 0) {
        *found = s0 + hitidx;
        return c;
      }
      pos = ehi;
    }
  }
  return c;
}

// Single wave: exact running value through every block, cend[b] = value after
// block b.  Each round takes the next 64 blocks: the leading run of blocks
// whose transfers apply in the current binade is applied at once (an ordered
// prefix of the transfers), the first block that does not is done alone
// (its transfer if it applies from the new value, else an element walk), and
// the next round starts after it.
constexpr int kXWin = 1024;  // block transfers staged in LDS per window (32 KB)

__global__ __launch_bounds__(64) void walk_kernel(const double* __restrict__ dmin, int64_t n,
                                                  double S, const Xfer* __restrict__ xf,
                                                  int64_t nblocks, double c_in,
                                                  double* __restrict__ cend,
                                                  double* __restrict__ c_out,
                                                  long long* __restrict__ stats) {
  __shared__ Xfer sx[kXWin];
  const int lane = threadIdx.x;
  double c = c_in;
  int64_t dummy = -1;
  int64_t b0 = 0;
  int64_t win0 = -1;  // first block of the staged window
  long long st_rounds = 0, st_single = 0, st_fine = 0, st_fcyc = 0;
  const long long st_t0 = stats ? (long long)clock64() : 0;
  while (b0 < nblocks) {
    const int nb = (int)((nblocks - b0) < 64 ? (nblocks - b0) : 64);
    if (win0 < 0 || b0 + nb > win0 + kXWin) {
      // restage [b0, b0 + kXWin): 16 independent loads per lane in flight
      __syncthreads();
      win0 = b0;
      Xfer v[kXWin / 64];
#pragma unroll
      for (int j = 0; j < kXWin / 64; ++j) {
        const int64_t bb = b0 + j * 64 + lane;
        v[j] = bb < nblocks ? xf[bb] : Xfer{0, 0, 0, 0, 0};
      }
#pragma unroll
      for (int j = 0; j < kXWin / 64; ++j) sx[j * 64 + lane] = v[j];
      __syncthreads();
    }
    const Xfer r = lane < nb ? sx[b0 - win0 + lane] : Xfer{0, 0, 0, 0, 0};
    int e;
    long long N;
    const bool inb = binade_of(c, e, N);
    // inclusive ordered prefix of the round's transfers
    long long D0 = r.d0, D1 = r.d1;
    int valid = (lane < nb) && r.valid && inb && r.e == e;
    for (int o = 1; o < 64; o <<= 1) {
      const long long l0 = __shfl_up(D0, o), l1 = __shfl_up(D1, o);
      const int lv = __shfl_up(valid, o);
      if (lane >= o) {
        long long n0, n1;
        compose(l0, l1, D0, D1, n0, n1);
        D0 = n0;
        D1 = n1;
        valid &= lv;
      }
    }
    const long long Dq = (N & 1) ? D1 : D0;
    const bool ok = inb && valid && Dq < (1ll << 52) && (N + Dq) < (1ll << 53);
    const unsigned long long okm = __ballot(ok);
    int L = (okm == ~0ull) ? 64 : __builtin_ctzll(~okm);
    if (L > nb) L = nb;
    if (L > 0) {
      if (lane < L) cend[b0 + lane] = from_binade(e, N + Dq);
      c = from_binade(e, N + __shfl(Dq, L - 1));
    }
    ++st_rounds;
    if (L == nb) {
      b0 += nb;
      continue;
    }
    ++st_single;
    // block bj alone
    const int64_t bj = b0 + L;
    const Xfer rj = sx[bj - win0];
    int ej;
    long long Nj;
    bool done = false;
    if (binade_of(c, ej, Nj) && rj.valid && rj.e == ej) {
      const long long Dj = (Nj & 1) ? rj.d1 : rj.d0;
      if (Dj < (1ll << 52) && Nj + Dj < (1ll << 53)) {
        c = from_binade(ej, Nj + Dj);
        done = true;
      }
    }
    if (!done) {
      const int64_t lo = bj * kSeedBlock;
      const int64_t hi = (lo + kSeedBlock) < n ? (lo + kSeedBlock) : n;
      const long long tf = stats ? (long long)clock64() : 0;
      c = fine_walk(dmin, S, lo, hi, c, false, 1.0, 0.0, &dummy);
      if (stats) st_fcyc += (long long)clock64() - tf;
      ++st_fine;
    }
    if (lane == 0) cend[bj] = c;
    b0 = bj + 1;
  }
  if (lane == 0) *c_out = c;
  if (stats && lane == 0) {
    stats[0] += st_rounds;
    stats[1] += st_single;
    stats[2] += st_fine;
    stats[3] += st_fcyc;
    stats[4] += (long long)clock64() - st_t0;
  }
}

// Single wave: first local index m with fl(c_m / c_last) > u (or -1).  The
// running values cend are non-decreasing, so hit(b) = fl(cend[b] / c_last) > u
// is monotone in b: a 64-ary search (64 probes per round) finds the first hit
// block, then an exact walk of that block finds the element.
__global__ __launch_bounds__(64) void search_kernel(const double* __restrict__ dmin, int64_t n,
                                                    double S, const double* __restrict__ cend,
                                                    int64_t nblocks, double c_in, double c_last,
                                                    double u, int64_t* __restrict__ result) {
  const int lane = threadIdx.x;
  // invariant: every block < lo misses, block hi hits (hi == nblocks: none)
  int64_t lo = 0, hi = nblocks;
  while (hi - lo > 0) {
    const int64_t span = hi - lo;
    const int64_t step = (span + 63) / 64;
    const int64_t pb = lo + (int64_t)lane * step;
    const bool probe = pb < hi;
    const bool hit = probe && (cend[pb] / c_last) > u;
    const unsigned long long m = __ballot(hit);
    const unsigned long long pm = __ballot(probe);
    if (step == 1) {
      if (m) hi = lo + __builtin_ctzll(m);
      break;
    }
    // first probing lane that hits: the answer is in (probe[j-1], probe[j]]
    if (m) {
      const int j = __builtin_ctzll(m);
      hi = lo + (int64_t)j * step;
      lo = j > 0 ? lo + (int64_t)(j - 1) * step + 1 : lo;
    } else {
      const int jl = 63 - __builtin_clzll(pm);  // last probe misses
      lo = lo + (int64_t)jl * step + 1;
    }
  }
  const int64_t bstar = hi < nblocks ? hi : -1;
  int64_t found = -1;
  if (bstar >= 0) {
    const double c0 = bstar == 0 ? c_in : cend[bstar - 1];
    const int64_t lo2 = bstar * kSeedBlock;
    const int64_t hi2 = (lo2 + kSeedBlock) < n ? (lo2 + kSeedBlock) : n;
    fine_walk(dmin, S, lo2, hi2, c0, true, c_last, u, &found);
  }
  if (lane == 0) *result = found;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static void check_points(const Ctx& c) {
  if (c.mode == 0) CDR_FAIL(CDR_ERR_STATE, "no points loaded");
  if (c.d > 128) CDR_FAIL(CDR_ERR_UNSUPPORTED, "d > 128 is not supported yet");
}

void seed_reset(Ctx& c) {
  check_points(c);
  c.dmin.ensure(sizeof(double) * c.n_pad);
  hipLaunchKernelGGL(fill_inf, dim3(1024), dim3(256), 0, c.stream, c.dmin.as<double>(), c.n_pad);
  HIP_CHECK(hipGetLastError());
  c.seed_near.ensure(sizeof(int32_t) * c.n_pad);
  HIP_CHECK(hipMemsetAsync(c.seed_near.p, 0, sizeof(int32_t) * c.n_pad, c.stream));
  c.seed_count = 0;
  c.seed_scanned = false;
}

// Append the new centre (device copy in seed_scalar) to the centre list and
// compute its distances to the earlier ones (the pruning table).
static void seed_track(Ctx& c) {
  const int d = c.d;
  const size_t need = sizeof(double) * (size_t)(c.seed_count + 1) * d;
  if (c.seed_cents.bytes < need) {
    DevBuf grown;
    grown.ensure(std::max(need, 2 * c.seed_cents.bytes));
    if (c.seed_count > 0)
      HIP_CHECK(hipMemcpyAsync(grown.p, c.seed_cents.p, sizeof(double) * (size_t)c.seed_count * d,
                               hipMemcpyDeviceToDevice, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    c.seed_cents.release();
    c.seed_cents = grown;
    grown.p = nullptr;
    grown.bytes = 0;
  }
  c.seed_ccd.ensure(sizeof(double) * (size_t)(c.seed_count + 1));
  if (c.seed_count > 0)
    hipLaunchKernelGGL(seed_ccd_kernel, dim3((c.seed_count + 255) / 256), dim3(256), 0, c.stream,
                       c.seed_cents.as<double>(), c.seed_count, d, c.seed_scalar.as<double>(),
                       c.seed_ccd.as<double>());
  HIP_CHECK(hipMemcpyAsync(c.seed_cents.as<double>() + (size_t)c.seed_count * d,
                           c.seed_scalar.p, sizeof(double) * d, hipMemcpyDeviceToDevice,
                           c.stream));
}

void seed_update(Ctx& c, const double* cen) {
  check_points(c);
  if (!c.dmin.p) seed_reset(c);
  const int64_t nb = c.nblocks();
  c.blocksums.ensure(sizeof(double) * (nb > 0 ? nb : 1));
  c.seed_scalar.ensure(sizeof(double) * (c.d + 8));
  HIP_CHECK(hipMemcpyAsync(c.seed_scalar.p, cen, sizeof(double) * c.d, hipMemcpyHostToDevice,
                           c.stream));
  if (!c.seed_near.p) {  // dmin from an earlier session without the tracking buffers
    c.seed_near.ensure(sizeof(int32_t) * c.n_pad);
    HIP_CHECK(hipMemsetAsync(c.seed_near.p, 0, sizeof(int32_t) * c.n_pad, c.stream));
  }
  seed_track(c);
  int32_t* near = c.seed_near.as<int32_t>();
  const double* ccd = c.seed_ccd.as<double>();
  const int cidx = c.seed_count;
  if (nb > 0) {
    typedef void (*SeedFn)(const float*, int64_t, int64_t, int, const double*, double*, double*,
                           int64_t, int32_t*, const double*, int);
#define CDR_SU(D_) seed_update_kernel<float, D_, false>
    static const SeedFn fns[17] = {CDR_SU(0),  CDR_SU(1),  CDR_SU(2),  CDR_SU(3),  CDR_SU(4),
                                   CDR_SU(5),  CDR_SU(6),  CDR_SU(7),  CDR_SU(8),  CDR_SU(9),
                                   CDR_SU(10), CDR_SU(11), CDR_SU(12), CDR_SU(13), CDR_SU(14),
                                   CDR_SU(15), CDR_SU(16)};
#undef CDR_SU
    const int64_t nfull = c.n / kSeedBlock;
    const bool f32 = c.mode == CDR_MODE_F32X;
    if (nfull > 0) {
      if (f32)
        hipLaunchKernelGGL(fns[c.d <= 16 ? c.d : 0], dim3(nfull), dim3(256), 0, c.stream,
                           c.x32.as<float>(), c.n, c.n_pad, c.d, c.seed_scalar.as<double>(),
                           c.dmin.as<double>(), c.blocksums.as<double>(), (int64_t)0, near, ccd,
                           cidx);
      else
        hipLaunchKernelGGL((seed_update_kernel<double, 0, false>), dim3(nfull), dim3(256), 0,
                           c.stream, c.x64.as<double>(), c.n, c.n_pad, c.d,
                           c.seed_scalar.as<double>(), c.dmin.as<double>(),
                           c.blocksums.as<double>(), (int64_t)0, near, ccd, cidx);
      HIP_CHECK(hipGetLastError());
    }
    if (nb > nfull) {
      if (f32)
        hipLaunchKernelGGL((seed_update_kernel<float, 0, true>), dim3(1), dim3(256), 0,
                           c.stream, c.x32.as<float>(), c.n, c.n_pad, c.d,
                           c.seed_scalar.as<double>(), c.dmin.as<double>(),
                           c.blocksums.as<double>(), nfull, near, ccd, cidx);
      else
        hipLaunchKernelGGL((seed_update_kernel<double, 0, true>), dim3(1), dim3(256), 0,
                           c.stream, c.x64.as<double>(), c.n, c.n_pad, c.d,
                           c.seed_scalar.as<double>(), c.dmin.as<double>(),
                           c.blocksums.as<double>(), nfull, near, ccd, cidx);
    }
    HIP_CHECK(hipGetLastError());
  }
  c.seed_count += 1;
  c.seed_scanned = false;
}

void seed_scan(Ctx& c, double total, double c_in, double* c_out) {
  check_points(c);
  const int64_t nb = c.nblocks();
  if (nb == 0) {
    *c_out = c_in;
    return;
  }
  c.xfer.ensure(sizeof(Xfer) * nb);
  c.cend.ensure(sizeof(double) * nb * 2);
  double* approx = c.cend.as<double>() + nb;
  hipLaunchKernelGGL(approx_prefix_kernel, dim3(1), dim3(1024), 0, c.stream,
                     c.blocksums.as<double>(), nb, total, c_in, approx);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(xfer_kernel, dim3((int)ceil_div(nb, 4)), dim3(256), 0, c.stream,
                     c.dmin.as<double>(), c.n, total, approx, nb, c.xfer.as<Xfer>());
  HIP_CHECK(hipGetLastError());
  c.seed_scalar.ensure(sizeof(double) * (c.d + 8));
  double* dres = c.seed_scalar.as<double>() + c.d;
  static const bool want_stats = std::getenv("CDR_SEED_STATS") != nullptr;
  long long* dstats = nullptr;
  if (want_stats) {
    static long long* ds = nullptr;
    if (!ds) {
      HIP_CHECK(hipMalloc(&ds, 8 * sizeof(long long)));
      HIP_CHECK(hipMemset(ds, 0, 8 * sizeof(long long)));
    }
    dstats = ds;
  }
  hipLaunchKernelGGL(walk_kernel, dim3(1), dim3(64), 0, c.stream, c.dmin.as<double>(), c.n,
                     total, c.xfer.as<Xfer>(), nb, c_in, c.cend.as<double>(), dres, dstats);
  if (want_stats) {
    long long hs[8];
    HIP_CHECK(hipMemcpyAsync(hs, dstats, sizeof(hs), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    fprintf(stderr,
            "seed walk stats (cumulative): rounds %lld single %lld fine %lld nb %lld "
            "fine_cycles %lld total_cycles %lld\n",
            hs[0], hs[1], hs[2], (long long)nb, hs[3], hs[4]);
  }
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(c_out, dres, sizeof(double), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.seed_c_in = c_in;
  c.seed_total = total;
  c.seed_scanned = true;
}

void seed_search(Ctx& c, double c_last, double u, int64_t* idx) {
  check_points(c);
  if (!c.seed_scanned) CDR_FAIL(CDR_ERR_STATE, "cdr_seed_search before cdr_seed_scan");
  const int64_t nb = c.nblocks();
  if (nb == 0) {
    *idx = -1;
    return;
  }
  c.seed_scalar.ensure(sizeof(double) * (c.d + 8));
  int64_t* dres = reinterpret_cast<int64_t*>(c.seed_scalar.as<double>() + c.d + 1);
  hipLaunchKernelGGL(search_kernel, dim3(1), dim3(64), 0, c.stream, c.dmin.as<double>(), c.n,
                     c.seed_total, c.cend.as<double>(), nb, c.seed_c_in, c_last, u, dres);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(idx, dres, sizeof(int64_t), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
}

}  // namespace cdr

using namespace cdr;

extern "C" {

int cdr_seed_reset(cdr_ctx* h) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_reset(h->c);
  CDR_CATCH
}

int cdr_seed_update(cdr_ctx* h, const double* c) {
  CDR_TRY
  if (!h || !c) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_update(h->c, c);
  CDR_CATCH
}

int cdr_seed_num_blocks(cdr_ctx* h, int64_t* nblocks) {
  CDR_TRY
  if (!h || !nblocks) CDR_FAIL(CDR_ERR_ARG, "null argument");
  *nblocks = h->c.nblocks();
  CDR_CATCH
}

int cdr_seed_block_sums(cdr_ctx* h, double* out) {
  CDR_TRY
  if (!h || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  const int64_t nb = c.nblocks();
  if (nb > 0) {
    HIP_CHECK(hipMemcpyAsync(out, c.blocksums.p, sizeof(double) * nb, hipMemcpyDeviceToHost,
                             c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
  }
  CDR_CATCH
}

int cdr_seed_scan(cdr_ctx* h, double total, double c_in, double* c_out) {
  CDR_TRY
  if (!h || !c_out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  if (!(total > 0.0) || std::isinf(total)) CDR_FAIL(CDR_ERR_NAN, "Probabilities contain NaN");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_scan(h->c, total, c_in, c_out);
  CDR_CATCH
}

int cdr_seed_search(cdr_ctx* h, double c_last, double u, int64_t* idx) {
  CDR_TRY
  if (!h || !idx) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_search(h->c, c_last, u, idx);
  CDR_CATCH
}

}  // extern "C"
