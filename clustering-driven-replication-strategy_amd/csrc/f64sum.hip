// f64sum.hip — exact, parallel F64-mode centroid sums (src/kmeans_plusplus.py:
// 41, `X[labels == j].mean(axis=0)`): for d >= 2 NumPy adds the selected rows
// one after another, so sums[j][f] is the SEQUENTIAL fp64 sum of the column in
// row order.  Floating-point addition is not associative; this reproduces the
// sequential result bit for bit without a serial pass over n.
//
// While the running value s stays inside one binade [2^e, 2^(e+1)) it is
// m * g with g = 2^(e-52) and 2^52 <= m < 2^53, and adding x >= 0 gives
// m + q + (rounding of the fraction r of x / g: up when r > 1/2, down when
// r < 1/2, to even when r == 1/2).  Only the tie depends on m, through its
// parity, so a run of additions inside one binade is an integer transfer that
// depends only on the parity of m when the run starts: (D0, P0) for an even
// entry and (D1, P1) for an odd one (the same idea as the seeding cumsum,
// csrc/seed.hip).
//
//   A  f64_blocksum   per 256-row block: approximate per-(cluster, feature)
//                     sums (any order) and member counts
//   B  f64_predict_a/b/c  per (cluster, feature): running approximate prefix
//                     (group sums, group prefix, in-group prefix) -> the
//                     binade the exact running value is expected to be in
//                     when each block starts
//   C  f64_transfer   per (block, feature): the block's transfer for every
//                     cluster in its predicted binade (flagged when an addend
//                     is negative or not below the binade's top)
//   G  f64_group      per (cluster, feature) and group of 64 blocks: the
//                     group's composed transfer when all its blocks share one
//                     predicted binade
//   D  f64_walk       per (cluster, feature), sequential over the groups (one
//                     step each) and, where a group cannot be applied whole,
//                     its blocks: the exact running value; a block whose prediction missed,
//                     whose transfer is flagged or would leave the binade is
//                     re-added element by element in real fp64 (so the result
//                     is exact whatever the data; the prediction only decides
//                     how often that happens: about once per binade crossing,
//                     ~log2(n) times per sequence for non-negative data).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "cdr_internal.h"

namespace cdr {

namespace {

constexpr int kFB = 256;               // rows per block
constexpr int kFMaxK = 64;             // clusters handled here (LDS state)
constexpr int kENone = -100000;        // no prediction (no member before the block)

// The summed type T: double (F64 mode) or float (the reference's float32
// runs: the same algorithm on a 24-bit significand).  MB = significand bits
// after the point; binades below kMinE are subnormal (no fixed grid): those
// blocks are re-added element by element.
template <typename T>
struct SumTraits {
  static constexpr int MB = 52;
  static constexpr int kMinE = -1022;
};
template <>
struct SumTraits<float> {
  static constexpr int MB = 23;
  static constexpr int kMinE = -126;
};

struct Xfer {
  long long d0;  // grid steps added for an even entry
  int dd;        // d1 - d0
  int flags;     // bit0 P0, bit1 P1 (exit parities), bit2 invalid, bit3 members
};

template <typename T>
__global__ __launch_bounds__(kFB) void f64_blocksum(const T* __restrict__ X, int64_t n,
                                                    int64_t n_pad, int d, int k,
                                                    const int32_t* __restrict__ labels,
                                                    double* __restrict__ A,
                                                    unsigned* __restrict__ cnt) {
  extern __shared__ double sh[];
  double* tab = sh;                                   // [k][d]
  unsigned* c = reinterpret_cast<unsigned*>(sh + k * d);  // [k]
  const int64_t b = blockIdx.x;
  for (int i = threadIdx.x; i < k * d; i += kFB) tab[i] = 0.0;
  for (int i = threadIdx.x; i < k; i += kFB) c[i] = 0;
  __syncthreads();
  const int64_t row = b * kFB + threadIdx.x;
  if (row < n) {
    const int j = labels[row];
    atomicAdd(&c[j], 1u);
    for (int f = 0; f < d; ++f) atomicAdd(&tab[j * d + f], (double)X[xidx(f, row, n_pad)]);
  }
  __syncthreads();
  // sequence-major ([cluster * d + feature][block], [cluster][block]): the
  // later passes walk one sequence over the blocks with the lanes, so their
  // loads are contiguous
  const int64_t nbk = gridDim.x;
  for (int i = threadIdx.x; i < k * d; i += kFB) A[(int64_t)i * nbk + b] = tab[i];
  for (int i = threadIdx.x; i < k; i += kFB) cnt[(int64_t)i * nbk + b] = c[i];
}

// The predicted binade of each block's start: an exclusive prefix of the
// approximate block sums per (cluster, feature), any order (it only
// predicts), in three parallel passes over groups of 64 blocks: group sums
// (one wave per sequence and group), the groups' exclusive prefix (one wave
// per sequence), the blocks' prefix inside each group.
__device__ __forceinline__ int binade_e(double P) {
  if (!(P > 0.0) || !isfinite(P)) return kENone;
  int ex;
  frexp(P, &ex);  // P in [2^(ex-1), 2^ex)
  return ex - 1;
}
__global__ __launch_bounds__(256) void f64_predict_a(const double* __restrict__ A,
                                                     const unsigned* __restrict__ cnt,
                                                     int64_t nb, int d, int k, int64_t ng,
                                                     double* __restrict__ GS) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= (int64_t)k * d * ng) return;
  const int t = (int)(w / ng);
  const int64_t g = w % ng;
  const int j = t / d;
  const int64_t b = g * 64 + lane;
  double v = (b < nb && cnt[(int64_t)j * nb + b]) ? A[(int64_t)t * nb + b] : 0.0;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if (lane == 0) GS[w] = v;
}
__global__ __launch_bounds__(256) void f64_predict_b(double* __restrict__ GS, int kd,
                                                     int64_t ng) {
  const int t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (t >= kd) return;
  double* gs = GS + (int64_t)t * ng;
  double carry = 0.0;
  for (int64_t g0 = 0; g0 < ng; g0 += 64) {
    const int64_t g = g0 + lane;
    const double v = g < ng ? gs[g] : 0.0;
    double inc = v;
    for (int o = 1; o < 64; o <<= 1) {
      const double u = __shfl_up(inc, o);
      if (lane >= o) inc += u;
    }
    if (g < ng) gs[g] = carry + (inc - v);
    carry += __shfl(inc, 63);
  }
}
__global__ __launch_bounds__(256) void f64_predict_c(const double* __restrict__ A,
                                                     const unsigned* __restrict__ cnt,
                                                     int64_t nb, int d, int k, int64_t ng,
                                                     const double* __restrict__ GS,
                                                     int* __restrict__ E) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= (int64_t)k * d * ng) return;
  const int t = (int)(w / ng);
  const int64_t g = w % ng;
  const int j = t / d;
  const int64_t b = g * 64 + lane;
  const double v = (b < nb && cnt[(int64_t)j * nb + b]) ? A[(int64_t)t * nb + b] : 0.0;
  double inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const double u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (b < nb) E[(int64_t)t * nb + b] = binade_e(GS[w] + (inc - v));
}

// One thread per (block, feature); the per-cluster transfer states live in
// LDS ([thread][cluster]).
template <typename TA, typename S>
__global__ void f64_transfer(const S* __restrict__ X, int64_t n, int64_t n_pad, int d,
                             int k, int64_t nb, const int32_t* __restrict__ labels,
                             const int* __restrict__ E, Xfer* __restrict__ T) {
  extern __shared__ unsigned char smem[];
  const int nt = blockDim.x;
  long long* s0 = reinterpret_cast<long long*>(smem);   // [nt][k]
  int* sdd = reinterpret_cast<int*>(s0 + (size_t)nt * k);  // [nt][k]
  int* sfl = sdd + (size_t)nt * k;                        // [nt][k]
  int* se = sfl + (size_t)nt * k;                         // [nt][k]
  const int64_t t = (int64_t)blockIdx.x * nt + threadIdx.x;
  const bool live = t < nb * d;
  // the d threads of one block are neighbours: they share its label stream
  const int64_t b = live ? t / d : 0;
  const int f = live ? (int)(t % d) : 0;
  long long* m0 = s0 + (size_t)threadIdx.x * k;
  int* mdd = sdd + (size_t)threadIdx.x * k;
  int* mfl = sfl + (size_t)threadIdx.x * k;
  int* me = se + (size_t)threadIdx.x * k;
  if (!live) return;
  for (int j = 0; j < k; ++j) {
    m0[j] = 0;
    mdd[j] = 0;
    mfl[j] = 2;  // P0 = 0, P1 = 1
    me[j] = E[((int64_t)j * d + f) * nb + b];
  }
  const int64_t r0 = b * kFB, r1 = min(n, r0 + kFB);
  // rows in chunks of 16: the chunk's labels and values are loaded before
  // the (serial, LDS-dependent) updates, so the loop does not pay a memory
  // round trip per row
  constexpr int kCh = 16;
  for (int64_t rc = r0; rc < r1; rc += kCh) {
    int lj[kCh];
    double lx[kCh];
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      const int64_t row = rc + u;
      lj[u] = row < r1 ? labels[row] : -1;
      lx[u] = row < r1 ? (double)X[xidx(f, row, n_pad)] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
    const int j = lj[u];
    if (j < 0) continue;
    const double x = lx[u];
    int fl = mfl[j] | 8;
    const int e = me[j];
    if (e == kENone || e < SumTraits<TA>::kMinE || !(x >= 0.0)) {
      mfl[j] = fl | 4;
      continue;
    }
    const double y = ldexp(x, SumTraits<TA>::MB - e);  // exact: a power-of-two scaling
    if (!(y < (double)(1ll << (SumTraits<TA>::MB + 1)))) {  // x not below the binade's top
      mfl[j] = fl | 4;
      continue;
    }
    const double q = floor(y);
    const double r = y - q;
    const long long qi = (long long)q;
    const bool up = r > 0.5, tie = r == 0.5;
    // even-entry path
    const int p0 = fl & 1;
    const long long i0 = qi + (up ? 1 : (tie ? ((p0 + qi) & 1) : 0));
    // odd-entry path
    const int p1 = (fl >> 1) & 1;
    const long long i1 = qi + (up ? 1 : (tie ? ((p1 + qi) & 1) : 0));
    m0[j] += i0;
    mdd[j] += (int)(i1 - i0);
    fl = (fl & ~3) | (int)((p0 + i0) & 1) | ((int)((p1 + i1) & 1) << 1);
    mfl[j] = fl;
    }
  }
  for (int j = 0; j < k; ++j) {
    Xfer x;
    x.d0 = m0[j];
    x.dd = mdd[j];
    x.flags = mfl[j];
    T[((int64_t)j * d + f) * nb + b] = x;
  }
}

// Transfer composition: entering with parity p, A then B gives
// D_p = D^A_p + D^B_(P^A_p) and the exit parity P^B_(P^A_p).  Associative,
// so a run of blocks that stay in one binade is one transfer: as the
// addends are >= 0 the running value only grows, and when it is still in
// the binade after the whole run it was inside it after every block.
struct XferC {
  long long d0, d1;
  int p;  // bit0 P0, bit1 P1
};
__device__ __forceinline__ XferC xc_compose(const XferC& a, const XferC& b) {
  XferC r;
  const int a0 = a.p & 1, a1 = (a.p >> 1) & 1;
  r.d0 = a.d0 + (a0 ? b.d1 : b.d0);
  r.d1 = a.d1 + (a1 ? b.d1 : b.d0);
  r.p = ((b.p >> a0) & 1) | (((b.p >> a1) & 1) << 1);
  return r;
}

// Group transfers: one wave per (cluster, feature) and group of 64 blocks
// (all groups in parallel): when every non-empty block of the group is
// predicted in one binade with a usable transfer, their composition (the
// same 6-level shuffle tree as f64_walk's) so that the walk applies the
// whole group in one step.
struct GXfer {
  long long d0, d1;
  int e;
  int p;  // bit0 P0, bit1 P1, bit2 usable, bit3 any member
};
__global__ __launch_bounds__(256) void f64_group(const unsigned* __restrict__ cnt,
                                                 const int* __restrict__ E,
                                                 const Xfer* __restrict__ T, int64_t nb, int d,
                                                 int k, int64_t ng, GXfer* __restrict__ G) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int kd = k * d;
  if (w >= (int64_t)kd * ng) return;
  const int t = (int)(w / ng);
  const int64_t g = w % ng;
  const int j = t / d;
  const int64_t bl = g * 64 + lane;
  const bool in = bl < nb;
  const unsigned c = in ? cnt[(int64_t)j * nb + bl] : 0u;
  const int el = in ? E[(int64_t)t * nb + bl] : kENone;
  const Xfer xl = in ? T[(int64_t)t * nb + bl] : Xfer{0, 0, 4};
  const unsigned long long live = __ballot(c != 0);
  int e0 = kENone;
  if (live) e0 = __shfl(el, __ffsll((long long)live) - 1);
  const bool ok = c == 0 || (e0 != kENone && el == e0 && !(xl.flags & 4));
  const bool usable = live && __ballot(!ok) == 0ull;
  XferC x;
  const bool on = c != 0;
  x.d0 = on ? xl.d0 : 0;
  x.d1 = on ? xl.d0 + xl.dd : 0;
  x.p = on ? (xl.flags & 3) : 2;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    XferC y;
    y.d0 = __shfl_down(x.d0, o);
    y.d1 = __shfl_down(x.d1, o);
    y.p = __shfl_down(x.p, o);
    if ((lane & (2 * o - 1)) == 0 && lane + o < 64) x = xc_compose(x, y);
  }
  if (lane == 0)
    G[w] = GXfer{x.d0, x.d1, e0, (x.p & 3) | (usable ? 4 : 0) | (live ? 8 : 0)};
}

// One wave per (cluster, feature), the running value uniform across it.  The
// lanes load 64 blocks' (count, prediction, transfer) per round; the wave
// takes the longest run of blocks from the current one that are empty or
// predicted in the running value's binade with a valid transfer, composes
// their transfers with a 6-level shuffle tree (in block order) and applies
// the result at once.  A block that breaks a run (another binade, a flagged
// transfer, the first member of the sequence) or a run that would leave the
// binade is applied block by block, re-adding a block element by element in
// real fp64 whenever its transfer cannot be used.  (Stepping every block
// through the transfer one at a time cost 8 ms at 10M x 5, k = 16.)
template <typename TA, typename S>
__global__ __launch_bounds__(256) void f64_walk(const S* __restrict__ X, int64_t n,
                                                int64_t n_pad, int d, int k, int64_t nb,
                                                const int32_t* __restrict__ labels,
                                                const unsigned* __restrict__ cnt,
                                                const int* __restrict__ E,
                                                const Xfer* __restrict__ T,
                                                const GXfer* __restrict__ G, int64_t ng,
                                                double* __restrict__ sums,
                                                long long* __restrict__ walked,
                                                long long* __restrict__ prof) {
  const int t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (t >= k * d) return;
  const int j = t / d, f = t % d;
  constexpr int MB = SumTraits<TA>::MB, kMinE = SumTraits<TA>::kMinE;
  constexpr long long kTop = 1ll << (MB + 1);
  double s = 0.0;  // (a T value)
  bool any = false;  // NumPy's reduce starts from the first selected row
  long long nwalk = 0;
  long long pc_el = 0, pc_slow = 0, n_slow = 0;  // CDR_F64_PROF: cycles
  const long long pc0 = prof ? (long long)clock64() : 0;
  // one block by transfer or element by element (wave-uniform b)
  auto step_block = [&](int64_t b, int e, int flags, long long d0, int dd) {
    bool ok = false;
    if (!(flags & 4) && s > 0.0) {
      int ex;
      frexp(s, &ex);
      if (ex - 1 == e && e >= kMinE) {
        const long long m = (long long)ldexp(s, MB - e);  // exact: s is on the grid
        const long long m2 = m + ((m & 1) ? d0 + dd : d0);
        if (m2 < kTop) {
          s = ldexp((double)m2, e - MB);
          ok = true;
        }
      }
    }
    if (!ok) {  // element by element, in real fp64 (row order)
      ++nwalk;
      const long long pe0 = prof ? (long long)clock64() : 0;
      const int64_t r0 = b * kFB;
      for (int q = 0; q < kFB; q += 64) {
        const int64_t row = r0 + q + lane;
        const bool mine = row < n && labels[row] == j;
        const double x = mine ? (double)X[xidx(f, row, n_pad)] : 0.0;
        unsigned long long mk = __ballot(mine);
        while (mk) {
          const int l = __builtin_amdgcn_readfirstlane(__ffsll((long long)mk) - 1);
          mk &= mk - 1;
          const long long xb = __double_as_longlong(x);
          const double v = __longlong_as_double(
              (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane(
                               (int)(xb >> 32), l)
                           << 32) |
                          (unsigned)__builtin_amdgcn_readlane((int)xb, l)));
          s = any ? (double)((TA)s + (TA)v) : v;  // (TA arithmetic: one rounding)
          any = true;
        }
      }
      if (prof) pc_el += (long long)clock64() - pe0;
    }
  };
  // a group's (count, prediction, transfer) per lane
  auto fetch = [&](int64_t b0, unsigned& c, int& el, Xfer& xl) {
    const int64_t bl = b0 + lane;
    const bool in = bl < nb;
    c = in ? cnt[(int64_t)j * nb + bl] : 0u;
    el = in ? E[(int64_t)t * nb + bl] : kENone;
    xl = in ? T[(int64_t)t * nb + bl] : Xfer{0, 0, 4};
  };
  // Groups are read 64 at a time (one load per lane, the next 64 prefetched)
  // and taken from registers: a group that applies in one step costs no
  // memory round trip.  The per-block records are loaded only for a group
  // that does not (about one per binade crossing).
  const GXfer* Gt = G + (int64_t)t * ng;
  auto gfetch = [&](int64_t g0) {
    return g0 + lane < ng ? Gt[g0 + lane] : GXfer{0, 0, kENone, 0};
  };
  // The running value as (binade sE, grid count sN) while groups apply whole
  // (integer work on scalar registers: readlane, no LDS shuffles and no
  // double <-> integer conversions per group); s is refreshed from it before
  // a group is walked block by block, and it from s afterwards.
  int sE = kENone;
  long long sN = 0;
  auto to_int = [&]() {
    sE = kENone;
    if (s > 0.0) {
      int ex;
      frexp(s, &ex);
      if (ex - 1 >= kMinE) {
        sE = ex - 1;
        sN = (long long)ldexp(s, MB - sE);  // exact: s is on the grid
      }
    }
  };
  GXfer gnext = gfetch(0);
  for (int64_t g0 = 0; g0 < ng; g0 += 64) {
    const GXfer gl = gnext;
    if (g0 + 64 < ng) gnext = gfetch(g0 + 64);
    const unsigned long long gl_live = __ballot((gl.p & 8) != 0);
    unsigned long long todo = gl_live;
    while (todo) {
      const int gi = __builtin_amdgcn_readfirstlane(__ffsll((long long)todo) - 1);
      todo &= todo - 1;
      const int gp = __builtin_amdgcn_readlane(gl.p, gi);
      if ((gp & 4) && sE != kENone) {  // the whole group in one step
        const int ge = __builtin_amdgcn_readlane(gl.e, gi);
        if (sE == ge) {
          const long long gd =
              (sN & 1) ? (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane(
                                          (int)(gl.d1 >> 32), gi)
                                      << 32) |
                                     (unsigned)__builtin_amdgcn_readlane((int)gl.d1, gi))
                       : (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane(
                                          (int)(gl.d0 >> 32), gi)
                                      << 32) |
                                     (unsigned)__builtin_amdgcn_readlane((int)gl.d0, gi));
          const long long m2 = sN + gd;
          if (m2 < kTop) {
            sN = m2;
            continue;
          }
        }
      }
      if (sE != kENone) s = ldexp((double)sN, sE - MB);  // s from the integer state
      const long long ps0 = prof ? (long long)clock64() : 0;
      ++n_slow;
      const int64_t b0 = (g0 + gi) * 64;
      unsigned c;
      int el;
      Xfer xl;
      fetch(b0, c, el, xl);
      if (!c) xl = Xfer{0, 0, 4};
      const unsigned long long live = __ballot(c != 0);
      int i = 0;  // next block of this group (wave-uniform)
      while (i < 64) {
        const unsigned long long rest = live & (~0ull << i);
        if (!rest) break;
        i = __builtin_amdgcn_readfirstlane(__ffsll((long long)rest) - 1);  // skip empty blocks
        int es = kENone;
        if (s > 0.0) {
          int ex;
          frexp(s, &ex);
          if (ex - 1 >= kMinE) es = ex - 1;
        }
        // blocks i.. that are empty or can take a transfer in binade es
        const bool compat = c == 0 || (es != kENone && !(xl.flags & 4) && el == es);
        const unsigned long long brk = ~__ballot(compat) & (~0ull << i);
        const int r = __builtin_amdgcn_readfirstlane(brk ? __ffsll((long long)brk) - 1 : 64);  // run [i, r)
        if (r > i + 1) {
          // inclusive ordered prefix of the run's transfers (lanes outside it
          // are the identity), then the longest prefix that stays in the
          // binade is applied at once and the block that leaves it is
          // stepped alone: one scan per binade crossing, not one per block
          XferC x;
          const bool on = lane >= i && lane < r && c != 0;
          x.d0 = on ? xl.d0 : 0;
          x.d1 = on ? xl.d0 + xl.dd : 0;
          x.p = on ? (xl.flags & 3) : 2;  // identity: P0 = 0, P1 = 1
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            XferC y;
            y.d0 = __shfl_up(x.d0, o);
            y.d1 = __shfl_up(x.d1, o);
            y.p = __shfl_up(x.p, o);
            if (lane >= o) x = xc_compose(y, x);
          }
          const long long m = (long long)ldexp(s, MB - es);
          const long long mq = m + ((m & 1) ? x.d1 : x.d0);
          const bool inrun = lane >= i && lane < r;
          const unsigned long long bad = __ballot(inrun && !(mq < kTop));
          const int L = __builtin_amdgcn_readfirstlane(bad ? __ffsll((long long)bad) - 1 : r);
          if (L > i) {  // blocks i .. L-1 in one step
            const long long mL =
                (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane(
                                 (int)(mq >> 32), L - 1)
                             << 32) |
                            (unsigned)__builtin_amdgcn_readlane((int)mq, L - 1));
            s = ldexp((double)mL, es - MB);
            i = L;
            if (i >= r) continue;
          }
          // block L leaves the binade: stepped alone below
        }
        const int e = __builtin_amdgcn_readlane(el, i);
        const int flags = __builtin_amdgcn_readlane(xl.flags, i);
        const long long d0 = (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane(
                                             (int)(xl.d0 >> 32), i)
                                         << 32) |
                                        (unsigned)__builtin_amdgcn_readlane((int)xl.d0, i));
        const int dd = __builtin_amdgcn_readlane(xl.dd, i);
        step_block(b0 + i, e, flags, d0, dd);
        ++i;
      }
      to_int();
      if (prof) pc_slow += (long long)clock64() - ps0;
    }
  }
  if (sE != kENone) s = ldexp((double)sN, sE - MB);
  if (prof && lane == 0) {
    prof[4 * t] = (long long)clock64() - pc0;
    prof[4 * t + 1] = pc_slow;
    prof[4 * t + 2] = pc_el;
    prof[4 * t + 3] = n_slow;
  }

  if (lane == 0) {
    sums[(int64_t)j * d + f] = s;
    walked[t] = nwalk;
  }
}

}  // namespace

// sums (k, d) on the device, exact sequential row-order fp64 sums; returns
// false when the shape is not covered (d < 2, k > 64): the caller runs the
// serial kernel.
// TA: the summed (arithmetic) type; S: the storage type of X
template <typename TA, typename S>
static bool sums_parallel(Ctx& c, const S* X, int k, double* d_sums) {
  const int d = c.d;
  if (d < 2 || k < 1 || k > kFMaxK || c.n < 1) return false;
  const int64_t n = c.n, nb = ceil_div(n, kFB);
  const size_t kd = (size_t)k * d;
  c.f64x_A.ensure(sizeof(double) * nb * kd);
  c.f64x_cnt.ensure(sizeof(unsigned) * nb * k);
  c.f64x_E.ensure(sizeof(int) * nb * kd);
  c.f64x_T.ensure(sizeof(Xfer) * nb * kd);
  c.f64x_walk.ensure(sizeof(long long) * kd);
  hipLaunchKernelGGL(f64_blocksum<S>, dim3(nb), dim3(kFB), sizeof(double) * kd + 4 * k, c.stream,
                     X, n, c.n_pad, d, k, c.labels.as<int32_t>(),
                     c.f64x_A.as<double>(), c.f64x_cnt.as<unsigned>());
  HIP_CHECK(hipGetLastError());
  const int64_t ng = ceil_div(nb, (int64_t)64);
  c.f64x_GS.ensure(sizeof(double) * ng * kd);
  const dim3 gwaves((unsigned)ceil_div((int64_t)kd * ng, (int64_t)4));
  hipLaunchKernelGGL(f64_predict_a, gwaves, dim3(256), 0, c.stream, c.f64x_A.as<double>(),
                     c.f64x_cnt.as<unsigned>(), nb, d, k, ng, c.f64x_GS.as<double>());
  hipLaunchKernelGGL(f64_predict_b, dim3(ceil_div((int64_t)kd, 4)), dim3(256), 0, c.stream,
                     c.f64x_GS.as<double>(), (int)kd, ng);
  hipLaunchKernelGGL(f64_predict_c, gwaves, dim3(256), 0, c.stream, c.f64x_A.as<double>(),
                     c.f64x_cnt.as<unsigned>(), nb, d, k, ng, c.f64x_GS.as<double>(),
                     c.f64x_E.as<int>());
  HIP_CHECK(hipGetLastError());
  const int nt = std::max(32, std::min(256, 4096 / k)) & ~31;
  const size_t lds = (size_t)nt * k * (8 + 4 + 4 + 4);
  hipLaunchKernelGGL((f64_transfer<TA, S>), dim3(ceil_div(nb * d, nt)), dim3(nt), lds, c.stream,
                     X, n, c.n_pad, d, k, nb, c.labels.as<int32_t>(),
                     c.f64x_E.as<int>(), c.f64x_T.as<Xfer>());
  HIP_CHECK(hipGetLastError());
  c.f64x_G.ensure(sizeof(GXfer) * ng * kd);
  static const bool prof_on = std::getenv("CDR_F64_PROF") != nullptr;
  if (prof_on) c.f64x_prof.ensure(sizeof(long long) * 4 * kd);
  hipLaunchKernelGGL(f64_group, dim3(ceil_div((int64_t)kd * ng, (int64_t)4)), dim3(256), 0,
                     c.stream, c.f64x_cnt.as<unsigned>(), c.f64x_E.as<int>(),
                     c.f64x_T.as<Xfer>(), nb, d, k, ng, c.f64x_G.as<GXfer>());
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL((f64_walk<TA, S>), dim3(ceil_div((int64_t)kd, 4)), dim3(256), 0, c.stream,
                     X, n, c.n_pad, d, k, nb, c.labels.as<int32_t>(),
                     c.f64x_cnt.as<unsigned>(), c.f64x_E.as<int>(), c.f64x_T.as<Xfer>(),
                     c.f64x_G.as<GXfer>(), ng, d_sums, c.f64x_walk.as<long long>(),
                     prof_on ? c.f64x_prof.as<long long>() : nullptr);
  HIP_CHECK(hipGetLastError());
  if (prof_on) {
    std::vector<long long> h(4 * kd);
    HIP_CHECK(hipMemcpyAsync(h.data(), c.f64x_prof.p, 8 * h.size(), hipMemcpyDeviceToHost,
                             c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    long long mx[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < kd; ++i)
      for (int q = 0; q < 4; ++q) mx[q] = std::max(mx[q], h[4 * i + q]);
    fprintf(stderr, "f64_walk max cycles: total %lld slow-groups %lld element-walks %lld; slow groups %lld\n",
            mx[0], mx[1], mx[2], mx[3]);
  }
  HIP_CHECK(hipGetLastError());
  return true;
}

bool f64_sums_parallel(Ctx& c, int k, double* d_sums) {
  return sums_parallel<double, double>(c, c.x64.as<double>(), k, d_sums);
}
// The reference's float32 runs: sequential fp32 sums of fp32 points (X:
// F32X storage, or F64 storage holding fp32 values), returned as doubles.
bool f32_sums_parallel(Ctx& c, int k, double* d_sums) {
  if (c.mode == CDR_MODE_F32X) return sums_parallel<float, float>(c, c.x32.as<float>(), k, d_sums);
  return sums_parallel<float, double>(c, c.x64.as<double>(), k, d_sums);
}

}  // namespace cdr
