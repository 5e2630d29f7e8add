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
// in LDS with one pad slot per 128 (conflict-free leaf reads).
template <typename T>
__global__ __launch_bounds__(256) void seed_update_kernel(
    const T* __restrict__ X, int64_t n, int64_t n_pad, int d, const double* __restrict__ cen,
    double* __restrict__ dmin, double* __restrict__ blocksums) {
  __shared__ double sdm[4096 + 32];
  __shared__ double sleaf[160];
  __shared__ int soff[160], slen[160];
  __shared__ int sleaves;
  const int64_t b = blockIdx.x;
  const int64_t base = b * kSeedBlock;
  const int m = (int)((n - base) < kSeedBlock ? (n - base) : kSeedBlock);
  double halves[2] = {0.0, 0.0};
  for (int h = 0; h < 2; ++h) {
    for (int q = threadIdx.x; q < 4096; q += blockDim.x) {
      const int qi = h * 4096 + q;
      const int64_t i = base + qi;
      double v = 0.0;
      if (qi < m) {
        auto xv = [&](int f) { return (double)X[xidx(f, i, n_pad)]; };
        auto cv = [&](int f) { return cen[f]; };
        const double R = np_sqdist(xv, cv, d);
        const double r = sqrt(R);
        const double t = r * r;
        const double old = dmin[i];
        v = t < old ? t : old;
        dmin[i] = v;
      }
      sdm[q + (q >> 7)] = v;
    }
    __syncthreads();
    if (m == kSeedBlock && threadIdx.x < 32) {
      const int l = threadIdx.x;
      double s = np_pw_leaf([&](int i) { return sdm[129 * l + i]; }, 128);
      for (int o = 1; o < 32; o <<= 1) s = s + __shfl_xor(s, o);
      if (l == 0) halves[h] = s;
    }
    __syncthreads();
  }
  if (m == kSeedBlock) {
    if (threadIdx.x == 0) blocksums[b] = halves[0] + halves[1];
    return;
  }
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

// ---- cumulative-sum emulation --------------------------------------------

__device__ __forceinline__ void compose(long long L0, long long L1, long long R0, long long R1,
                                        long long& o0, long long& o1) {
  o0 = L0 + ((L0 & 1) ? R1 : R0);
  o1 = L1 + ((L1 & 1) ? R0 : R1);
}

// Transfer of elements [lo, hi) of dmin under binade exponent e.
__device__ void range_transfer(const double* __restrict__ dmin, double S, int64_t lo,
                               int64_t hi, int e, long long& D0, long long& D1, int& valid) {
  D0 = 0;
  D1 = 0;
  valid = 1;
  for (int64_t i = lo; i < hi; ++i) {
    const double p = dmin[i] / S;
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

// Per-block transfers under the guessed binade of the block's start.
__global__ __launch_bounds__(256) void xfer_kernel(const double* __restrict__ dmin, int64_t n,
                                                   double S, const double* __restrict__ approx,
                                                   int64_t nblocks, Xfer* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (b >= nblocks) return;
  const double ca = approx[b];
  int e = 0;
  long long Ndummy;
  const bool okg = binade_of(ca, e, Ndummy);
  const int64_t base = b * kSeedBlock;
  const int64_t lo = base + (int64_t)lane * kSub;
  int64_t hi = lo + kSub;
  if (hi > n) hi = n;
  long long D0 = 0, D1 = 0;
  int valid = okg ? 1 : 0;
  if (okg && lo < hi) range_transfer(dmin, S, lo, hi, e, D0, D1, valid);
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
  if (lane == 0) {
    if (D0 >= (1ll << 52) || D1 >= (1ll << 52)) valid = 0;
    out[b] = Xfer{D0, D1, e, valid, 0};
  }
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
// value after the last element processed.  Executed by all 64 lanes of a wave.
__device__ double fine_walk(const double* __restrict__ dmin, double S, int64_t lo, int64_t hi,
                            double c, bool search, double c_last, double u, int64_t* found) {
  const int lane = threadIdx.x & 63;
  int64_t pos = lo;
  while (pos < hi) {
    int e;
    long long N;
    const bool inb = binade_of(c, e, N);
    int L = 0;  // sub-chunks applied in bulk
    if (inb) {
      const int64_t slo = pos + (int64_t)lane * kSub;
      int64_t shi = slo + kSub;
      if (shi > hi) shi = hi;
      long long D0 = 0, D1 = 0;
      int valid = 1;
      if (slo < hi) range_transfer(dmin, S, slo, shi, e, D0, D1, valid);
      else valid = 0;
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
      bool ok = valid && slo < hi && Dq < (1ll << 52) && Nend < (1ll << 53);
      bool hit = false;
      if (ok && search) hit = (from_binade(e, Nend) / c_last) > u;
      const unsigned long long okm = __ballot(ok && !hit);
      // number of leading lanes that are ok and not yet past the target
      L = (okm == ~0ull) ? 64 : __builtin_ctzll(~okm);
      if (L > 0) {
        const long long DL = __shfl(Dq, L - 1);
        c = from_binade(e, N + DL);
        pos += (int64_t)L * kSub;
        if (pos > hi) pos = hi;
      }
      if (pos >= hi) break;
      if (L == 64) continue;  // every sub-chunk applied: next bulk round
    }
    // element-wise over (at most) one sub-chunk; lane 0 computes, broadcasts
    const int64_t ehi = (pos + kSub) < hi ? (pos + kSub) : hi;
    double cc = c;
    int64_t hitidx = -1;
    if (lane == 0) {
      for (int64_t i = pos; i < ehi; ++i) {
        cc = cc + dmin[i] / S;
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
      *found = hitidx;
      return c;
    }
    pos = ehi;
  }
  return c;
}

// Single wave: exact running value through every block, cend[b] = value after
// block b.  Whole 64-block chunks are applied at once when they stay inside
// one binade.
__global__ __launch_bounds__(64) void walk_kernel(const double* __restrict__ dmin, int64_t n,
                                                  double S, const Xfer* __restrict__ xf,
                                                  int64_t nblocks, double c_in,
                                                  double* __restrict__ cend,
                                                  double* __restrict__ c_out) {
  const int lane = threadIdx.x;
  double c = c_in;
  int64_t dummy = -1;
  for (int64_t b0 = 0; b0 < nblocks; b0 += 64) {
    const int64_t b = b0 + lane;
    const int nb = (int)((nblocks - b0) < 64 ? (nblocks - b0) : 64);
    Xfer r = (b < nblocks) ? xf[b] : Xfer{0, 0, 0, 0, 0};
    int e;
    long long N;
    const bool inb = binade_of(c, e, N);
    // bulk: inclusive prefix of the chunk's transfers
    long long D0 = r.d0, D1 = r.d1;
    int valid = (b < nblocks) && r.valid && inb && r.e == e;
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
    const unsigned long long okm = __ballot(ok || lane >= nb);
    if (okm == ~0ull) {
      if (lane < nb) cend[b] = from_binade(e, N + Dq);
      c = from_binade(e, N + __shfl(Dq, nb - 1));
      continue;
    }
    // block by block
    for (int j = 0; j < nb; ++j) {
      const int64_t bj = b0 + j;
      const Xfer rj = xf[bj];
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
        c = fine_walk(dmin, S, lo, hi, c, false, 1.0, 0.0, &dummy);
      }
      if (lane == 0) cend[bj] = c;
    }
  }
  if (lane == 0) *c_out = c;
}

// Single wave: first local index m with fl(c_m / c_last) > u (or -1).
__global__ __launch_bounds__(64) void search_kernel(const double* __restrict__ dmin, int64_t n,
                                                    double S, const double* __restrict__ cend,
                                                    int64_t nblocks, double c_in, double c_last,
                                                    double u, int64_t* __restrict__ result) {
  const int lane = threadIdx.x;
  int64_t bstar = -1;
  for (int64_t b0 = 0; b0 < nblocks && bstar < 0; b0 += 64) {
    const int64_t b = b0 + lane;
    const bool hit = b < nblocks && (cend[b] / c_last) > u;
    const unsigned long long m = __ballot(hit);
    if (m) bstar = b0 + __builtin_ctzll(m);
  }
  int64_t found = -1;
  if (bstar >= 0) {
    const double c0 = bstar == 0 ? c_in : cend[bstar - 1];
    const int64_t lo = bstar * kSeedBlock;
    const int64_t hi = (lo + kSeedBlock) < n ? (lo + kSeedBlock) : n;
    fine_walk(dmin, S, lo, hi, c0, true, c_last, u, &found);
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
  c.seed_scanned = false;
}

void seed_update(Ctx& c, const double* cen) {
  check_points(c);
  if (!c.dmin.p) seed_reset(c);
  const int64_t nb = c.nblocks();
  c.blocksums.ensure(sizeof(double) * (nb > 0 ? nb : 1));
  c.seed_scalar.ensure(sizeof(double) * (c.d + 8));
  HIP_CHECK(hipMemcpyAsync(c.seed_scalar.p, cen, sizeof(double) * c.d, hipMemcpyHostToDevice,
                           c.stream));
  if (nb > 0) {
    if (c.mode == CDR_MODE_F32X)
      hipLaunchKernelGGL(seed_update_kernel<float>, dim3(nb), dim3(256), 0, c.stream,
                         c.x32.as<float>(), c.n, c.n_pad, c.d, c.seed_scalar.as<double>(),
                         c.dmin.as<double>(), c.blocksums.as<double>());
    else
      hipLaunchKernelGGL(seed_update_kernel<double>, dim3(nb), dim3(256), 0, c.stream,
                         c.x64.as<double>(), c.n, c.n_pad, c.d, c.seed_scalar.as<double>(),
                         c.dmin.as<double>(), c.blocksums.as<double>());
    HIP_CHECK(hipGetLastError());
  }
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
  hipLaunchKernelGGL(walk_kernel, dim3(1), dim3(64), 0, c.stream, c.dmin.as<double>(), c.n,
                     total, c.xfer.as<Xfer>(), nb, c_in, c.cend.as<double>(), dres);
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
