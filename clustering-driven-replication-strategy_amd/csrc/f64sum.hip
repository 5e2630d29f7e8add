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
#include <utility>
#include <vector>

#include "cdr_internal.h"
#include "exact_math.h"

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

// One element x >= 0 of a (cluster, feature) sequence added to a transfer
// state (m0: grid steps for an even entry, mdd: odd - even, mfl: bit0 P0,
// bit1 P1, bit2 invalid, bit3 members) under the predicted binade e.  With
// x = mx 2^ex (integer significand), y = x / 2^(e - MB) = mx 2^-sh: q =
// mx >> sh and the rounding of the fraction from the shifted-out bits — the
// same q and fraction as ldexp / floor in fp64, in integer instructions.
// Split in two so that a thread can run the part that does not depend on
// the state (xfer_pre: q, the rounding of the fraction, validity) for a whole
// chunk of rows as independent, branch-free work before the short serial
// updates (xfer_apply) — f64_transfer was bound by the dependent latency of
// the branchy combined form at two waves per SIMD.
struct XPre {
  long long q;
  int r;  // bit0 fraction above one half, bit1 exactly one half, bit2 invalid
};
template <typename TA>
__device__ __forceinline__ XPre xfer_pre(double x, int e) {
  // In fp64 instructions: y = x 2^(MB - e) is exact (a power-of-two scale;
  // where it would underflow, y < 2^-1022 and the answer is q = 0 below one
  // half either way), q = floor(y), and the fraction y - q is exact.  The
  // integer form (shifts and masks of the significand, ~70 instructions) was
  // a large part of f64_transfer's issue time (128 -> 121 us); both forms
  // agree on every (x, e) of a 2e7-case host fuzz (tools/xfer_pre_fuzz.cpp).
  constexpr int MB = SumTraits<TA>::MB;
  const double y = ldexp(x, MB - (e < -2000 ? -2000 : e));
  const double qf = floor(y);
  const double fr = y - qf;
  const bool bad = e == kENone || e < SumTraits<TA>::kMinE || !(x >= 0.0) ||
                   !(y < (double)(1ll << (MB + 1)));
  const double hf = floor(ldexp(qf, -32));
  const unsigned hi = bad ? 0u : (unsigned)hf;
  const unsigned lo = bad ? 0u : (unsigned)fma(hf, -4294967296.0, qf);
  return XPre{(long long)(((unsigned long long)hi << 32) | lo),
              (fr > 0.5 ? 1 : 0) | (fr == 0.5 ? 2 : 0) | (bad ? 4 : 0)};
}
__device__ __forceinline__ void xfer_apply(XPre p, long long& m0, int& mdd, int& mfl) {
  const int fl = mfl | 8;
  const int p0 = fl & 1, p1 = (fl >> 1) & 1;
  const long long i0 = p.q + ((p.r & 1) ? 1 : ((p.r & 2) ? ((p0 + p.q) & 1) : 0));
  const long long i1 = p.q + ((p.r & 1) ? 1 : ((p.r & 2) ? ((p1 + p.q) & 1) : 0));
  const bool bad = p.r & 4;
  m0 += bad ? 0 : i0;
  mdd += bad ? 0 : (int)(i1 - i0);
  mfl = bad ? (fl | 4) : ((fl & ~3) | (int)((p0 + i0) & 1) | ((int)((p1 + i1) & 1) << 1));
}

// One element x >= 0 of a (cluster, feature) sequence added to a transfer
// state (m0: grid steps for an even entry, mdd: odd - even, mfl: bit0 P0,
// bit1 P1, bit2 invalid, bit3 members) under the predicted binade e.  With
// x = mx 2^ex (integer significand), y = x / 2^(e - MB) = mx 2^-sh: q =
// mx >> sh and the rounding of the fraction from the shifted-out bits — the
// same q and fraction as ldexp / floor in fp64, in integer instructions.
template <typename TA>
__device__ __forceinline__ void xfer_add(double x, int e, long long& m0, int& mdd, int& mfl) {
  xfer_apply(xfer_pre<TA>(x, e), m0, mdd, mfl);
}

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
    for (int f = 0; f < d; ++f) atomicAdd(&tab[j * d + f], (double)X[xidx(X, f, row, n_pad)]);
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
// (GC: the clusters' member counts per group as well, from the waves of
// feature 0 - f64_predict_b adds them up; null: not wanted)
__global__ __launch_bounds__(256) void f64_predict_a(const double* __restrict__ A,
                                                     const unsigned* __restrict__ cnt,
                                                     int64_t nb, int d, int k, int64_t ng,
                                                     double* __restrict__ GS,
                                                     unsigned long long* __restrict__ GC) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= (int64_t)k * d * ng) return;
  const int t = (int)(w / ng);
  const int64_t g = w % ng;
  const int j = t / d;
  const int64_t b = g * 64 + lane;
  const unsigned cb = b < nb ? cnt[(int64_t)j * nb + b] : 0u;
  double v = cb ? A[(int64_t)t * nb + b] : 0.0;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if (lane == 0) GS[w] = v;
  if (GC && t % d == 0) {  // (wave-uniform)
    unsigned long long s = cb;
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) GC[(int64_t)j * ng + g] = s;
  }
}
// (GC non-null: the waves of feature 0 also write cluster t / d's member
// count, the sum of its group counts - the fused step's counts)
__global__ __launch_bounds__(256) void f64_predict_b(double* __restrict__ GS, int kd,
                                                     int64_t ng, const double* __restrict__ off,
                                                     const unsigned long long* __restrict__ GC,
                                                     int d,
                                                     unsigned long long* __restrict__ counts) {
  const int t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (t >= kd) return;
  if (GC && t % d == 0) {  // (wave-uniform)
    const unsigned long long* gc = GC + (int64_t)(t / d) * ng;
    unsigned long long s = 0;
    for (int64_t g = lane; g < ng; g += 64) s += gc[g];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) counts[t / d] = s;
  }
  double* gs = GS + (int64_t)t * ng;
  // a shard of sharded rows starts from the earlier shards' approximate sum
  double carry = off ? off[t] : 0.0;
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
                                                     int* __restrict__ E,
                                                     int* __restrict__ dE, int stamp) {
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
  if (b < nb) {
    const int e = binade_e(GS[w] + (inc - v));
    // (the transfer cache: a block whose prediction moved for any sequence
    // gets this step's stamp, so its transfers are formed again; every
    // writer of one block writes the same value)
    if (dE && E[(int64_t)t * nb + b] != e) dE[b] = stamp;
    E[(int64_t)t * nb + b] = e;
  }
}

// The transfer cache's work list: the blocks whose transfers are formed this
// step (all, or those whose labels changed in the assignment or whose binade
// predictions moved), compacted in any order into list with one atomic per
// workgroup (one per wave, on a single address, serialised to ~9 us per
// launch); counters[par] is this step's count, and the other counter is
// zeroed for the next step (the one that read it last has finished: stream
// order).
__global__ __launch_bounds__(256) void f64_dirty_list(const int* __restrict__ dlab,
                                                      const int* __restrict__ dE, int stamp,
                                                      int all, int64_t nb, int* __restrict__ list,
                                                      int* __restrict__ counters, int par) {
  __shared__ int wsum[4], wbase;
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool need = b < nb && (all || dlab[b] != 0 || dE[b] == stamp);
  const unsigned long long m = __ballot(need);
  if (lane == 0) wsum[w] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    wbase = tot ? atomicAdd(&counters[par], tot) : 0;
  }
  __syncthreads();
  int base = wbase;
  for (int q = 0; q < w; ++q) base += wsum[q];
  if (need) list[base + __popcll(m & ((1ull << lane) - 1ull))] = (int)b;
  if (b == 0) counters[par ^ 1] = 0;
}

// One block's transfers for every cluster, split over kTQ threads per (block,
// feature): thread q walks the rows [q R, (q + 1) R), R = kFB / kTQ, with its
// per-cluster states in LDS, cluster-major ([cluster][thread]): a lane's
// state for cluster j sits at j * nt + lane, so the lanes of a wave hit
// distinct banks whatever clusters their rows belong to.  The kTQ parts are
// then composed in row order with shuffles (xfer_join).  Each row's update
// is a serial LDS read-modify-write, so a wave's time is its rows' chain:
// with the whole block in one thread (256 rows) a launch could not go below
// one ~80 us chain however few blocks the transfer cache leaves.  Measured
// over the bench's F64 window (10M x 5, k = 16, steps 3-22, with the cache):
// 1, 2 and 4 parts 0.413-0.417 / 0.404-0.405 / 0.414-0.415 ms per step (more
// parts shorten the chains but add the per-thread setup and joins).
constexpr int kTQ = 2;
// a then b, both Xfer (d0: steps for an even entry, dd: odd - even, flags:
// bit0 P0, bit1 P1, bit2 invalid, bit3 members)
__device__ __forceinline__ void xfer_join(long long& d0, int& dd, int& fl, long long bd0, int bdd,
                                          int bfl) {
  const int p0 = fl & 1, p1 = (fl >> 1) & 1;
  const int q0 = bfl & 1, q1 = (bfl >> 1) & 1;
  d0 += bd0 + (p0 ? bdd : 0);
  dd += (p1 ? bdd : 0) - (p0 ? bdd : 0);
  fl = (p0 ? q1 : q0) | ((p1 ? q1 : q0) << 1) | ((fl | bfl) & 12);
}
// NTS: log2 of the workgroup size (the state rows' stride: shifts, not
// quarter-rate multiplies, in the per-row LDS addresses)
template <typename TA, typename S, int NTS>
__global__ __launch_bounds__(256) void f64_transfer(const S* __restrict__ X, int64_t n, int64_t n_pad, int d,
                             int k, int64_t nb, const int32_t* __restrict__ labels,
                             const int* __restrict__ E, Xfer* __restrict__ T,
                             const int* __restrict__ list, const int* __restrict__ lcount) {
  extern __shared__ unsigned char smem[];
  constexpr int nt = 1 << NTS;
  long long* s0 = reinterpret_cast<long long*>(smem);   // [k][nt]
  int* sdd = reinterpret_cast<int*>(s0 + (size_t)nt * k);  // [k][nt]
  int* sfl = sdd + (size_t)nt * k;                        // [k][nt]
  int* se = sfl + (size_t)nt * k;                         // [k][nt]
  const int64_t t = (int64_t)blockIdx.x * nt + threadIdx.x;
  // the d * kTQ threads of one block are neighbours (they share its label
  // stream), the kTQ parts of one (block, feature) in consecutive lanes.
  // (list: the transfer cache's blocks, lcount[0] of them; the others keep
  // the transfers they have)
  const int64_t item = t / (d * kTQ);
  const bool live = list ? item < (int64_t)lcount[0] : item < nb;
  const int64_t b = live ? (list ? (int64_t)list[item] : item) : 0;
  const int f = live ? (int)(t / kTQ % d) : 0;
  const int q = (int)(t % kTQ);
  long long* m0 = s0 + threadIdx.x;  // [j * nt]
  int* mdd = sdd + threadIdx.x;
  int* mfl = sfl + threadIdx.x;
  int* me = se + threadIdx.x;
  if (!live) return;  // (whole groups of kTQ lanes)
  for (int j = 0; j < k; ++j) {
    m0[j * nt] = 0;
    mdd[j * nt] = 0;
    mfl[j * nt] = 2;  // P0 = 0, P1 = 1
    me[j * nt] = E[((int64_t)j * d + f) * nb + b];
  }
  constexpr int kR = kFB / kTQ;
  const int64_t r0 = b * kFB + q * kR, r1 = min(n, r0 + kR);
  // rows in chunks of 16, the next chunk's labels and values loaded while
  // the current one goes through the (serial, LDS-dependent) updates: at two
  // waves per SIMD (LDS-bound) the memory latency is not hidden otherwise
  // (0.27 ms at 10M x 5, k = 16 with the loads of a chunk issued only at its start)
  constexpr int kCh = 16;
  static_assert(kR % kCh == 0, "whole chunks per part");
  int lj[kCh], nj[kCh];
  double lx[kCh], nx[kCh];
  auto load = [&](int64_t rc, int* jj, double* xx) {
    if (rc + kCh <= r1) {  // (all but the last chunk of the last block)
#pragma unroll
      for (int u = 0; u < kCh; ++u) {
        jj[u] = labels[rc + u];
        xx[u] = (double)X[xidx(X, f, rc + u, n_pad)];
      }
    } else {
#pragma unroll
      for (int u = 0; u < kCh; ++u) {
        const int64_t row = rc + u;
        jj[u] = row < r1 ? labels[row] : -1;
        xx[u] = row < r1 ? (double)X[xidx(X, f, row, n_pad)] : 0.0;
      }
    }
  };
  if (r0 < r1) load(r0, lj, lx);
  for (int64_t rc = r0; rc < r1; rc += kCh) {
    if (rc + kCh < r1) load(rc + kCh, nj, nx);
    // the chunk's binades (read-only), then its state-free parts, then the
    // serial state updates
    int le[kCh];
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      const int ev = me[(lj[u] < 0 ? 0 : lj[u]) * nt];
      le[u] = lj[u] >= 0 ? ev : kENone;
    }
    XPre pr[kCh];
#pragma unroll
    for (int u = 0; u < kCh; ++u) pr[u] = xfer_pre<TA>(lx[u], le[u]);
    // branch-free (a row past the end rewrites cluster 0's state unchanged),
    // the row's three state words read together before its writes
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      const bool live_row = lj[u] >= 0;
      const int o = (live_row ? lj[u] : 0) * nt;
      long long a = m0[o];
      int bq = mdd[o], c = mfl[o];
      const long long a0 = a;
      const int b0 = bq, c0 = c;
      xfer_apply(pr[u], a, bq, c);
      m0[o] = live_row ? a : a0;
      mdd[o] = live_row ? bq : b0;
      mfl[o] = live_row ? c : c0;
    }
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      lj[u] = nj[u];
      lx[u] = nx[u];
    }
  }
  // the parts in row order: lane q takes q + o's composition when q is a
  // multiple of 2o (a tree over the kTQ consecutive lanes), lane 0 writes
  for (int j = 0; j < k; ++j) {
    long long x0 = m0[j * nt];
    int xdd = mdd[j * nt], xfl = mfl[j * nt];
#pragma unroll
    for (int o = 1; o < kTQ; o <<= 1) {
      const long long y0 = __shfl_down(x0, o, kTQ);
      const int ydd = __shfl_down(xdd, o, kTQ);
      const int yfl = __shfl_down(xfl, o, kTQ);
      if ((q & (2 * o - 1)) == 0) xfer_join(x0, xdd, xfl, y0, ydd, yfl);
    }
    if (q == 0) T[((int64_t)j * d + f) * nb + b] = Xfer{x0, xdd, xfl};
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
                                                 int k, int64_t ng, GXfer* __restrict__ G,
                                                 const int* __restrict__ Eend) {
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
  // Eend (sharded programs, f64s_program): a block is usable only when the
  // predicted binade at its end (the next block's start; Eend[t] after the
  // last block) is its start binade too, so no crossing falls inside it
  const int eafter = !Eend ? e0 : (bl + 1 < nb ? E[(int64_t)t * nb + bl + 1] : Eend[t]);
  const bool ok = c == 0 || (e0 != kENone && el == e0 && !(xl.flags & 4) && eafter == e0);
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
                                                long long* __restrict__ prof,
                                                const double* __restrict__ entry) {
  const int t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (t >= k * d) return;
  const int j = t / d, f = t % d;
  constexpr int MB = SumTraits<TA>::MB, kMinE = SumTraits<TA>::kMinE;
  constexpr long long kTop = 1ll << (MB + 1);
  // (entry: a shard of sharded rows continues the earlier shards' exact
  // running values {s [k d], any [k d]}; else the sequence starts here)
  double s = entry ? entry[t] : 0.0;  // (a T value)
  bool any = entry ? entry[k * d + t] != 0.0 : false;  // NumPy's reduce starts from the first selected row
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
      // the block's labels and values all issued first (independent loads:
      // one memory round trip, not two per 64 rows)
      static_assert(kFB == 256, "four rows per lane");
      int lj[4];
      double lx[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = r0 + 64 * q + lane;
        lj[q] = row < n ? labels[row] : -1;
        lx[q] = row < n ? (double)X[xidx(X, f, row, n_pad)] : 0.0;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool mine = lj[q] == j;
        const double x = lx[q];
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
      // a run of whole groups in the running value's binade, composed in one
      // step: the ordered prefix of their transfers (a 6-level shuffle
      // tree), then the longest prefix that stays in the binade (the values
      // only grow, so staying there at the end means staying throughout).
      // Stepping them one at a time cost ~430 cycles per group
      if (sE != kENone) {
        const int i0 = __builtin_amdgcn_readfirstlane(__ffsll((long long)todo) - 1);
        const bool lv = (gl.p & 8) != 0;
        const bool okg = !lv || ((gl.p & 4) && gl.e == sE);
        const unsigned long long brk = ~__ballot(okg) & (~0ull << i0);
        const int r = __builtin_amdgcn_readfirstlane(brk ? __ffsll((long long)brk) - 1 : 64);
        if (r > i0 + 1) {
          const bool on = lane >= i0 && lane < r && lv;
          XferC x;
          x.d0 = on ? gl.d0 : 0;
          x.d1 = on ? gl.d1 : 0;
          x.p = on ? (gl.p & 3) : 2;  // identity: P0 = 0, P1 = 1
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            XferC y;
            y.d0 = __shfl_up(x.d0, o);
            y.d1 = __shfl_up(x.d1, o);
            y.p = __shfl_up(x.p, o);
            if (lane >= o) x = xc_compose(y, x);
          }
          const long long mq = sN + ((sN & 1) ? x.d1 : x.d0);
          const bool inrun = lane >= i0 && lane < r;
          const unsigned long long bad = __ballot(inrun && !(mq < kTop));
          const int L = __builtin_amdgcn_readfirstlane(bad ? __ffsll((long long)bad) - 1 : r);
          if (L > i0) {  // groups i0 .. L-1 at once
            sN = (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane(
                                  (int)(mq >> 32), L - 1)
                              << 32) |
                             (unsigned)__builtin_amdgcn_readlane((int)mq, L - 1));
            todo &= L >= 64 ? 0ull : (~0ull << L);
            continue;
          }
        }
      }
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
    if (entry) sums[k * d + t] = any ? 1.0 : 0.0;  // (the exit state for the next shard)
  }
}

// The exact argmin (exact_argmin: the first index of the smallest correctly
// rounded NumPy-order root) behind an fp32 screen, for k <= kF64ScrK.  With
// every x_f and c_f zero or within [2^-60, 2^60] (normal fp32 squares), the
// fp32 value S = fma-chain sum of fl32(fl32(x) - fl32(c))^2 is within
//   (d + 5.01) 2^-24 sum_f (|x_f| + |c_f|)^2 <= (d + 5.01) 2^-23 (|x|^2 + |c|^2)
// of the real squared distance (two conversions and a subtraction per term,
// d fused steps of non-negative terms), plus 2^-126 per step for a result
// flushed below the normal range.  E = (d + 12) 2^-23 (xx + cc) + d 2^-125
// (xx, cc: the fp32 squared norms) covers that, the two roundings of S -+ E,
// the fp64 NumPy sum's own error and a relative gap of 2^-48 beyond it.  So a
// centroid with S - E > min_i (S_i + E_i) has an fp64 square at least 2^-48
// above the winner's and a strictly larger rounded root: it can neither win
// nor tie.  The rest (usually the winner alone) go through exact_argmin's
// comparison in index order, which gives exact_argmin's answer.  fp64 VALU is
// a quarter of the fp32 rate on gfx950 and the full pass was issue-bound
// (PMC: 66 % of wave cycles stalled on issue).
constexpr int kF64ScrK = 16;
// a centroid's fp32 row in LDS: its d values, then its squared norm, padded
// to whole 16-byte reads
template <int D>
struct F64ScrRow {
  static constexpr int P = (D + 1 + 3) & ~3;
};
__device__ __forceinline__ bool f64_screen_ok(double v) {
  const double a = fabs(v);
  return v == 0.0 || (a >= 0x1p-60 && a <= 0x1p60);
}
template <int D>
__device__ __forceinline__ int f64_screen_argmin(const double (&xr)[D], const double* cs64,
                                                 const float* cs32, int k) {
  constexpr int DP = F64ScrRow<D>::P;
  typedef float f4v __attribute__((ext_vector_type(4)));
  float xs[D];
  float xx = 0.0f;
  bool ok = true;
#pragma unroll
  for (int f = 0; f < D; ++f) {
    ok &= f64_screen_ok(xr[f]);
    xs[f] = (float)xr[f];
    xx = fmaf(xs[f], xs[f], xx);
  }
  if (!ok) return exact_argmin([&](int f) { return xr[f]; }, cs64, k, D);
  const float kE = (float)(D + 12) * 0x1p-23f, eabs = (float)D * 0x1p-125f;
  float lo[kF64ScrK];
  float best = INFINITY;
#pragma unroll
  for (int jj = 0; jj < kF64ScrK; ++jj) {
    lo[jj] = INFINITY;
    if (jj < k) {
      f4v cr[DP / 4];
#pragma unroll
      for (int q = 0; q < DP / 4; ++q) cr[q] = reinterpret_cast<const f4v*>(cs32 + jj * DP)[q];
      float acc = 0.0f;
#pragma unroll
      for (int f = 0; f < D; ++f) {
        const float t = xs[f] - cr[f >> 2][f & 3];
        acc = fmaf(t, t, acc);
      }
      const float e = fmaf(kE, xx + cr[D >> 2][D & 3], eabs);
      lo[jj] = acc - e;
      best = fminf(best, acc + e);
    }
  }
  unsigned cand = 0;
#pragma unroll
  for (int jj = 0; jj < kF64ScrK; ++jj)
    if (lo[jj] <= best) cand |= 1u << jj;
  double Rb = INFINITY, rb = INFINITY;
  int jb = 0;
  while (cand) {
    const int jj = __builtin_ctz(cand);
    cand &= cand - 1u;
    const double* cj = cs64 + jj * D;
    const double R = np_sqdist([&](int f) { return xr[f]; }, [&](int f) { return cj[f]; }, D);
    if (R < Rb) {
      const double r = sqrt(R);
      if (r < rb) {
        rb = r;
        Rb = R;
        jb = jj;
      }
    }
  }
  return jb;
}

// The screen's centroid table for one step (every f64_assign_block workgroup
// staged it in LDS before): the fp32 rows with their fp32 squared norms, as
// f64_screen_argmin reads them, and ok[0] = 1 when the screen applies (k <= 16,
// every value 0 or within [2^-60, 2^60]).  The assignment reads the rows with
// uniform addresses, i.e. scalar loads, instead of 32 LDS reads per row.
template <int D>
__global__ __launch_bounds__(64) void f64_cent_prep(const double* __restrict__ C, int k,
                                                    float* __restrict__ cs32, int* __restrict__ ok) {
  constexpr int DP = F64ScrRow<D>::P;
  const int t = threadIdx.x;
  bool bad = k > kF64ScrK;
  if (t < kF64ScrK) {
    float row[DP];
#pragma unroll
    for (int q = 0; q < DP; ++q) row[q] = 0.0f;
    if (t < k) {
#pragma unroll
      for (int f = 0; f < D; ++f) {
        const double v = C[t * D + f];
        row[f] = (float)v;
        bad |= !f64_screen_ok(v);
      }
      float sq = 0.0f;
#pragma unroll
      for (int f = 0; f < D; ++f) sq = fmaf(row[f], row[f], sq);
      row[D] = sq;
    }
#pragma unroll
    for (int q = 0; q < DP; ++q) cs32[t * DP + q] = row[q];
  }
  const bool any_bad = __ballot(bad) != 0ull;
  if (t == 0) ok[0] = any_bad ? 0 : 1;
}

// F64 mode, the assignment fused with the block pass (one workgroup per
// block of kFB rows): labels (exact_argmin, src/kmeans_plusplus.py:33-34),
// the block's approximate sums and exact counts in f64_blocksum's layout,
// and (XF) the block's transfers under Eprev, the previous step's predicted
// binades — labels change little between Lloyd steps, so they are mostly
// right, and a wrong one only makes f64_walk re-add that block element by
// element (exact either way).  The rows are staged in LDS; thread (j, f)
// walks its sequence's members in row order.  D <= 16, k <= 64.
template <int D, bool XF>
__global__ __launch_bounds__(kFB) void f64_assign_block(const double* __restrict__ X, int64_t n,
                                                        int64_t n_pad,
                                                        const double* __restrict__ C, int k,
                                                        int32_t* __restrict__ labels,
                                                        double* __restrict__ A,
                                                        unsigned* __restrict__ cnt,
                                                        const int* __restrict__ Eprev,
                                                        Xfer* __restrict__ T,
                                                        unsigned char* __restrict__ ordr,
                                                        const long long* __restrict__ gate,
                                                        const float* __restrict__ cs32g,
                                                        const int* __restrict__ scr_ok,
                                                        int* __restrict__ dlab) {
  // (the device-resident F64 run: a stopped run keeps the labels of the
  // assignment that stopped it)
  if (gate && gate[0] == 0) return;
  __shared__ double tab[kFMaxK * D];
  __shared__ unsigned cc[kFMaxK];
  __shared__ int coff[kFMaxK];
  __shared__ int wcnt[kFB / 64][kFMaxK];
  __shared__ double sx[XF ? D * kFB : 1];
  __shared__ int sj[XF ? kFB : 1];
  // Workgroups are dealt round-robin over the 8 XCDs; XCD x takes the
  // contiguous block range x * (nb / 8) + min(x, nb % 8) + [0, its share), so
  // the 8-byte writes of consecutive blocks into the sequence-major A and cnt
  // rows meet in one L2 and leave it as whole lines (with blockIdx.x as the
  // block, neighbouring blocks sit in different L2s and every write is partial)
  const int64_t nb = gridDim.x;
  const int64_t bq = nb >> 3, brm = nb & 7, bx = blockIdx.x & 7;
  const int64_t b = bx * bq + (bx < brm ? bx : brm) + (blockIdx.x >> 3);
  for (int i = threadIdx.x; i < k * D; i += kFB) tab[i] = 0.0;
  if (threadIdx.x < kFMaxK) cc[threadIdx.x] = 0u;
  const int64_t row = b * kFB + threadIdx.x;
  double xr[D];
  int jold = -1;  // (dlab: the previous label, for the transfer cache)
  if (row < n) {
#pragma unroll
    for (int f = 0; f < D; ++f) xr[f] = X[xidx(X, f, row, n_pad)];
    if (dlab) jold = labels[row];
  }
  // the screen's table (f64_cent_prep: fp32 rows and their fp32 squared
  // norms, read with uniform addresses) and the fp64 centroids for its
  // candidates, straight from global memory
  __syncthreads();  // (the zeroed tables)
  int j = -1;
  if (row < n) {
    j = scr_ok[0] ? f64_screen_argmin<D>(xr, C, cs32g, k)
                  : exact_argmin([&](int f) { return xr[f]; }, C, k, D);
    labels[row] = j;
  }
  if constexpr (XF) {
    sj[threadIdx.x] = j;
#pragma unroll
    for (int f = 0; f < D; ++f) sx[f * kFB + threadIdx.x] = j >= 0 ? xr[f] : 0.0;
  }
  // (the barrier; with dlab also whether any row of the block changed label)
  const int moved = __syncthreads_or(j != jold && dlab != nullptr);
  if (dlab && threadIdx.x == 0) dlab[b] = moved;
  if (j >= 0) {
    atomicAdd(&cc[j], 1u);
#pragma unroll
    for (int f = 0; f < D; ++f) atomicAdd(&tab[j * D + f], xr[f]);
  }
  // the block's rows in cluster order, row order inside a cluster (ordr: the
  // transfer pass walks each (cluster, feature) sequence through it): a
  // row's rank among its wave's rows of its cluster (one ballot per cluster
  // present), the earlier waves' counts, the cluster's offset
  int rank = 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (ordr) {
    for (int i = lane; i < kFMaxK; i += 64) wcnt[w][i] = 0;
    unsigned long long todo = __ballot(j >= 0);
    const unsigned long long below = (1ull << lane) - 1ull;
    while (todo) {
      const int l0 = __builtin_amdgcn_readfirstlane(__ffsll((long long)todo) - 1);
      const int lab = __builtin_amdgcn_readlane(j, l0);
      const unsigned long long m = __ballot(j == lab);
      if (j == lab) rank = __popcll(m & below);
      if (lane == 0) wcnt[w][lab] = __popcll(m);
      todo &= ~m;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < k * D; i += kFB) A[(int64_t)i * nb + b] = tab[i];
  for (int i = threadIdx.x; i < k; i += kFB) cnt[(int64_t)i * nb + b] = cc[i];
  if (ordr) {
    if (threadIdx.x == 0) {
      int o = 0;
      for (int q = 0; q < k; ++q) {
        coff[q] = o;
        o += (int)cc[q];
      }
    }
    __syncthreads();
    if (j >= 0) {
      int pos = coff[j] + rank;
      for (int ww = 0; ww < w; ++ww) pos += wcnt[ww][j];
      ordr[b * kFB + pos] = (unsigned char)threadIdx.x;
    }
  }
  if constexpr (XF) {
    for (int pr = threadIdx.x; pr < k * D; pr += kFB) {
      const int jj = pr / D, f = pr - jj * D;
      const int e = Eprev[(int64_t)pr * nb + b];
      long long m0 = 0;
      int mdd = 0, mfl = 2;  // P0 = 0, P1 = 1
      if (cc[jj]) {
        for (int r = 0; r < kFB; ++r)
          if (sj[r] == jj) xfer_add<double>(sx[f * kFB + r], e, m0, mdd, mfl);
      }
      T[(int64_t)pr * nb + b] = Xfer{m0, mdd, mfl};
    }
  }
}

// The transfers with one workgroup per block (f64_transfer's results): the
// block's rows and labels are staged in LDS with coalesced loads, then thread
// (j, f) walks its sequence's members in row order with its state in
// registers.  (f64_transfer, one thread per (block, feature) with k states
// in LDS each, ran at low occupancy: 0.24 ms at 10M x 5, k = 16.)
template <typename TA, typename S>
__global__ __launch_bounds__(kFB) void f64_transfer_block(const S* __restrict__ X, int64_t n,
                                                          int64_t n_pad, int d, int k,
                                                          const int32_t* __restrict__ labels,
                                                          const unsigned* __restrict__ cnt,
                                                          const int* __restrict__ E,
                                                          Xfer* __restrict__ T) {
  // [d][kFB] values, then int order[kFB], off[65], wcnt[4][64]
  extern __shared__ double tsx[];
  int* order = reinterpret_cast<int*>(tsx + (size_t)d * kFB);
  int* off = order + kFB;
  int* wcnt = off + 65;
  const int64_t b = blockIdx.x, nb = gridDim.x;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t row = b * kFB + t;
  const bool in = row < n;
  const int lj = in ? labels[row] : -1;
  for (int f = 0; f < d; ++f) tsx[f * kFB + t] = in ? (double)X[xidx(X, f, row, n_pad)] : 0.0;
  wcnt[t] = 0;  // (4 x 64 = kFB)
  if (t < k) off[t + 1] = (int)cnt[(int64_t)t * nb + b];
  __syncthreads();
  // the rows of each cluster in row order: a row's rank among its wave's
  // rows of the same cluster (one ballot per cluster present), plus the
  // earlier waves' counts of that cluster, plus the cluster's offset
  int rank = 0;
  {
    unsigned long long todo = __ballot(lj >= 0);
    const unsigned long long below = (1ull << lane) - 1ull;
    while (todo) {
      const int l0 = __builtin_amdgcn_readfirstlane(__ffsll((long long)todo) - 1);
      const int lab = __builtin_amdgcn_readlane(lj, l0);
      const unsigned long long m = __ballot(lj == lab);
      if (lj == lab) rank = __popcll(m & below);
      if (lane == 0) wcnt[w * 64 + lab] = __popcll(m);
      todo &= ~m;
    }
  }
  if (t == 0) {
    off[0] = 0;
    for (int j = 1; j <= k; ++j) off[j] += off[j - 1];
  }
  __syncthreads();
  if (lj >= 0) {
    int base = off[lj];
    for (int ww = 0; ww < w; ++ww) base += wcnt[ww * 64 + lj];
    order[base + rank] = t;
  }
  __syncthreads();
  for (int pr = t; pr < k * d; pr += kFB) {
    const int jj = pr / d, f = pr - jj * d;
    long long m0 = 0;
    int mdd = 0, mfl = 2;  // P0 = 0, P1 = 1
    const int o0 = off[jj], o1 = off[jj + 1];
    if (o1 > o0) {
      const int e = E[(int64_t)pr * nb + b];
      for (int o = o0; o < o1; ++o) xfer_add<TA>(tsx[f * kFB + order[o]], e, m0, mdd, mfl);
    }
    T[(int64_t)pr * nb + b] = Xfer{m0, mdd, mfl};
  }
}

// The transfers from the rows in cluster order (ordr, written by
// f64_assign_block): one thread per (block, feature) as f64_transfer, but a
// cluster's members are consecutive, so the running state lives in registers
// and is written out at the end of each run (f64_transfer keeps k states per
// thread in LDS, which capped it at 1-2 waves per SIMD: 0.24 ms at 10M x 5,
// k = 16).  Rows are read 16 at a time (one 16-byte load of their offsets,
// then the 16 values together).
template <typename TA, typename S>
__global__ __launch_bounds__(256) void f64_transfer_sorted(const S* __restrict__ X, int64_t n,
                                                           int64_t n_pad, int d, int k, int64_t nb,
                                                           const unsigned* __restrict__ cnt,
                                                           const int* __restrict__ E,
                                                           const unsigned char* __restrict__ ordr,
                                                           Xfer* __restrict__ T) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nb * d) return;
  const int64_t b = t / d;
  const int f = (int)(t % d);
  const int64_t r0 = b * kFB;
  const int nrow = (int)((n - r0) < kFB ? (n - r0) : kFB);
  // the first non-empty cluster and its run
  int jj = -1, left = 0;
  auto next_run = [&]() {
    while (left == 0 && jj + 1 < k) {
      ++jj;
      left = (int)cnt[(int64_t)jj * nb + b];
      if (left == 0) T[((int64_t)jj * d + f) * nb + b] = Xfer{0, 0, 2};
    }
  };
  next_run();
  long long m0 = 0;
  int mdd = 0, mfl = 2;  // P0 = 0, P1 = 1
  int e = left ? E[((int64_t)jj * d + f) * nb + b] : kENone;
  const uint4* ob = reinterpret_cast<const uint4*>(ordr + r0);
  for (int c0 = 0; c0 < nrow; c0 += 16) {
    const uint4 oq = ob[c0 >> 4];
    double xv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const unsigned word = u < 4 ? oq.x : u < 8 ? oq.y : u < 12 ? oq.z : oq.w;
      const int r = (int)((word >> (8 * (u & 3))) & 255u);
      xv[u] = c0 + u < nrow ? (double)X[xidx(X, f, r0 + r, n_pad)] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (c0 + u >= nrow || left == 0) break;
      xfer_add<TA>(xv[u], e, m0, mdd, mfl);
      if (--left == 0) {  // the run ends: its transfer, then the next run's state
        T[((int64_t)jj * d + f) * nb + b] = Xfer{m0, mdd, mfl};
        m0 = 0;
        mdd = 0;
        mfl = 2;
        next_run();
        if (left) e = E[((int64_t)jj * d + f) * nb + b];
      }
    }
  }
}

}  // namespace

// sums (k, d) on the device, exact sequential row-order fp64 sums; returns
// false when the shape is not covered (d < 2, k > 64): the caller runs the
// serial kernel.
// Sharded F64 sums (f64s_*): the earlier shards' approximate sums (off, k d),
// the predicted binade at this shard's end (Eend, k d), and either the walk
// from the exact entry state `entry` (rank 0: zeros) or no walk (the other
// ranks build programs from the transfers and group compositions instead).
struct F64Shard {
  const double* off = nullptr;
  const int* Eend = nullptr;
  const double* entry = nullptr;
  bool walk = true;
};
// The transfer cache of a device F64 run (f64_step_fused, tcache != 0): the
// assignment's per-block label-change flags, the per-block stamps of moved
// predictions, this step's stamp, whether every block is formed, the list and
// its counter pair.
struct F64TCache {
  const int* dlab = nullptr;
  int* dE = nullptr;
  int stamp = 0;
  int all = 1;
  int* list = nullptr;
  int* counters = nullptr;
  int par = 0;
};
template <typename TA, typename S>
static bool sums_after_block(Ctx& c, const S* X, int k, double* d_sums, int* Enew,
                             const int* Ewalk, bool have_T, const unsigned char* ordr = nullptr,
                             const F64Shard& sh = F64Shard(),
                             unsigned long long* d_counts = nullptr,
                             const F64TCache* tc = nullptr);

// TA: the summed (arithmetic) type; S: the storage type of X.  pre: the
// block sums and counts (f64x_A, f64x_cnt) were already written by the
// assignment (assign_blocksum_f64, lloyd.hip).
template <typename TA, typename S>
static bool sums_parallel(Ctx& c, const S* X, int k, double* d_sums, bool pre = false) {
  const int d = c.d;
  if (d < 2 || k < 1 || k > kFMaxK || c.n < 1) return false;
  const int64_t n = c.n, nb = ceil_div(n, kFB);
  const size_t kd = (size_t)k * d;
  c.f64x_A.ensure(sizeof(double) * nb * kd);
  c.f64x_cnt.ensure(sizeof(unsigned) * nb * k);
  c.f64x_E.ensure(sizeof(int) * nb * kd);
  c.f64x_T.ensure(sizeof(Xfer) * nb * kd);
  c.f64x_walk.ensure(sizeof(long long) * kd);
  if (!pre) {
    hipLaunchKernelGGL(f64_blocksum<S>, dim3(nb), dim3(kFB), sizeof(double) * kd + 4 * k, c.stream,
                       X, n, c.n_pad, d, k, c.labels.as<int32_t>(),
                       c.f64x_A.as<double>(), c.f64x_cnt.as<unsigned>());
    HIP_CHECK(hipGetLastError());
  }
  return sums_after_block<TA, S>(c, X, k, d_sums, c.f64x_E.as<int>(), c.f64x_E.as<int>(), false);
}

// After the block pass: the binade predictions into Enew; the transfers under
// Enew unless have_T (already formed under Ewalk by f64_assign_block); the
// group compositions and the walk under Ewalk.
template <typename TA, typename S>
static bool sums_after_block(Ctx& c, const S* X, int k, double* d_sums, int* Enew,
                             const int* Ewalk, bool have_T, const unsigned char* ordr,
                             const F64Shard& sh, unsigned long long* d_counts,
                             const F64TCache* tc) {
  const int d = c.d;
  const int64_t n = c.n, nb = ceil_div(n, kFB);
  const size_t kd = (size_t)k * d;
  const int64_t ng = ceil_div(nb, (int64_t)64);
  c.f64x_GS.ensure(sizeof(double) * ng * kd);
  const dim3 gwaves((unsigned)ceil_div((int64_t)kd * ng, (int64_t)4));
  unsigned long long* GC = nullptr;
  if (d_counts) {
    c.f64x_GC.ensure(sizeof(unsigned long long) * ng * k);
    GC = c.f64x_GC.as<unsigned long long>();
  }
  hipLaunchKernelGGL(f64_predict_a, gwaves, dim3(256), 0, c.stream, c.f64x_A.as<double>(),
                     c.f64x_cnt.as<unsigned>(), nb, d, k, ng, c.f64x_GS.as<double>(), GC);
  hipLaunchKernelGGL(f64_predict_b, dim3(ceil_div((int64_t)kd, 4)), dim3(256), 0, c.stream,
                     c.f64x_GS.as<double>(), (int)kd, ng, sh.off, GC, d, d_counts);
  hipLaunchKernelGGL(f64_predict_c, gwaves, dim3(256), 0, c.stream, c.f64x_A.as<double>(),
                     c.f64x_cnt.as<unsigned>(), nb, d, k, ng, c.f64x_GS.as<double>(), Enew,
                     tc ? tc->dE : nullptr, tc ? tc->stamp : 0);
  HIP_CHECK(hipGetLastError());
  const int* tlist = nullptr;
  const int* tcount = nullptr;
  if (tc && !have_T && !ordr) {
    hipLaunchKernelGGL(f64_dirty_list, dim3((unsigned)ceil_div(nb, (int64_t)256)), dim3(256), 0,
                       c.stream, tc->dlab, tc->dE, tc->stamp, tc->all, nb, tc->list,
                       tc->counters, tc->par);
    HIP_CHECK(hipGetLastError());
    tlist = tc->list;
    tcount = tc->counters + tc->par;
  }
  // 80 KB of per-thread states per workgroup (k <= 64): two workgroups per CU
  const int nts = k <= 16 ? 8 : (k <= 32 ? 7 : 6);
  const int nt = 1 << nts;
  const size_t lds = (size_t)nt * k * (8 + 4 + 4 + 4);
  // (CDR_F64_TBLOCK=1: the one-workgroup-per-block transfer; measured slower
  // at 10M x 5, k = 16: 0.25-0.30 ms against f64_transfer's 0.24 ms)
  static const bool tb_env = exp_env("CDR_F64_TBLOCK") && std::atoi(exp_env("CDR_F64_TBLOCK"));
  if (!have_T && ordr) {
    hipLaunchKernelGGL((f64_transfer_sorted<TA, S>), dim3((unsigned)ceil_div(nb * d, (int64_t)256)),
                       dim3(256), 0, c.stream, X, n, c.n_pad, d, k, nb, c.f64x_cnt.as<unsigned>(),
                       Ewalk, ordr, c.f64x_T.as<Xfer>());
    HIP_CHECK(hipGetLastError());
  } else if (!have_T && tb_env && d <= 32) {
    hipLaunchKernelGGL((f64_transfer_block<TA, S>), dim3((unsigned)nb), dim3(kFB),
                       sizeof(double) * d * kFB + sizeof(int) * (2 * kFB + 65), c.stream, X, n,
                       c.n_pad, d, k,
                       c.labels.as<int32_t>(), c.f64x_cnt.as<unsigned>(), Ewalk,
                       c.f64x_T.as<Xfer>());
    HIP_CHECK(hipGetLastError());
  } else if (!have_T) {
    auto fn = nts == 8 ? f64_transfer<TA, S, 8> : (nts == 7 ? f64_transfer<TA, S, 7>
                                                              : f64_transfer<TA, S, 6>);
    hipLaunchKernelGGL(fn, dim3(ceil_div(nb * d * kTQ, (int64_t)nt)), dim3(nt), lds, c.stream,
                       X, n, c.n_pad, d, k, nb, c.labels.as<int32_t>(), Ewalk,
                       c.f64x_T.as<Xfer>(), tlist, tcount);
    HIP_CHECK(hipGetLastError());
  }
  c.f64x_G.ensure(sizeof(GXfer) * ng * kd);
  static const bool prof_on = exp_env("CDR_F64_PROF") != nullptr;
  if (prof_on) c.f64x_prof.ensure(sizeof(long long) * 4 * kd);
  hipLaunchKernelGGL(f64_group, dim3(ceil_div((int64_t)kd * ng, (int64_t)4)), dim3(256), 0,
                     c.stream, c.f64x_cnt.as<unsigned>(), Ewalk,
                     c.f64x_T.as<Xfer>(), nb, d, k, ng, c.f64x_G.as<GXfer>(), sh.Eend);
  HIP_CHECK(hipGetLastError());
  if (!sh.walk) return true;
  hipLaunchKernelGGL((f64_walk<TA, S>), dim3(ceil_div((int64_t)kd, 4)), dim3(256), 0, c.stream,
                     X, n, c.n_pad, d, k, nb, c.labels.as<int32_t>(),
                     c.f64x_cnt.as<unsigned>(), Ewalk, c.f64x_T.as<Xfer>(),
                     c.f64x_G.as<GXfer>(), ng, d_sums, c.f64x_walk.as<long long>(),
                     prof_on ? c.f64x_prof.as<long long>() : nullptr, sh.entry);
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

bool f64_sums_parallel(Ctx& c, int k, double* d_sums, bool pre) {
  return sums_parallel<double, double>(c, c.x64.as<double>(), k, d_sums, pre);
}
// The F64 step's assignment and sums as one pipeline: f64_assign_block
// (labels, block sums, counts and — when the previous step left binade
// predictions for this (k, n) — the transfers), the cluster counts, the new
// predictions, the transfers otherwise, groups and walk.  false: shape not
// covered (d > 16, d < 2, k > 64), nothing launched.
// The step's screen table (f64_cent_prep) into c.f64x_cs; returns {rows, ok}.
static std::pair<const float*, const int*> f64_cent_table(Ctx& c, int d, int k, const double* dC) {
  constexpr int kRows = kF64ScrK * 20;  // (DP <= 20 floats at d <= 16)
  c.f64x_cs.ensure(sizeof(float) * kRows + 64);
  float* cs = c.f64x_cs.as<float>();
  int* ok = reinterpret_cast<int*>(cs + kRows);
  typedef void (*Pf)(const double*, int, float*, int*);
#define CDR_FCP(D_) f64_cent_prep<D_>
  static const Pf pfn[17] = {nullptr,     CDR_FCP(1),  CDR_FCP(2),  CDR_FCP(3),  CDR_FCP(4),
                             CDR_FCP(5),  CDR_FCP(6),  CDR_FCP(7),  CDR_FCP(8),  CDR_FCP(9),
                             CDR_FCP(10), CDR_FCP(11), CDR_FCP(12), CDR_FCP(13), CDR_FCP(14),
                             CDR_FCP(15), CDR_FCP(16)};
#undef CDR_FCP
  hipLaunchKernelGGL(pfn[d], dim3(1), dim3(64), 0, c.stream, dC, k, cs, ok);
  HIP_CHECK(hipGetLastError());
  return {cs, ok};
}

bool f64_step_fused(Ctx& c, int k, const double* dC, double* d_sums,
                    unsigned long long* d_counts, bool prof, const long long* gate,
                    int tcache) {
  const int d = c.d;
  if (d < 2 || d > 16 || k < 1 || k > kFMaxK || c.n < 1) return false;
  const int64_t n = c.n, nb = ceil_div(n, kFB);
  const size_t kd = (size_t)k * d;
  c.f64x_A.ensure(sizeof(double) * nb * kd);
  c.f64x_cnt.ensure(sizeof(unsigned) * nb * k);
  c.f64x_E.ensure(sizeof(int) * nb * kd);
  c.f64x_E2.ensure(sizeof(int) * nb * kd);
  c.f64x_T.ensure(sizeof(Xfer) * nb * kd);
  c.f64x_walk.ensure(sizeof(long long) * kd);
  // transfers under the previous step's predictions (CDR_F64_CARRY=1): right
  // only near convergence — between early steps 8-25 % of the blocks' binades
  // move and every such block is re-added element by element — so off by default
  static const bool carry = exp_env("CDR_F64_CARRY") && std::atoi(exp_env("CDR_F64_CARRY"));
  const bool xf = carry && c.f64x_e_ok && c.f64x_e_k == k && c.f64x_e_nb == nb;
  int* Ecur = (c.f64x_e_cur ? c.f64x_E2 : c.f64x_E).as<int>();
  int* Eoth = (c.f64x_e_cur ? c.f64x_E : c.f64x_E2).as<int>();
  // the rows in cluster order per block and f64_transfer_sorted (CDR_F64_SORTED=1;
  // measured slower at 10M x 5, k = 16: 0.43 ms against f64_transfer's 0.24 ms,
  // the order itself +0.04 ms in the assignment)
  static const bool sorted_env = exp_env("CDR_F64_SORTED") && std::atoi(exp_env("CDR_F64_SORTED"));
  unsigned char* ordr = nullptr;
  if (sorted_env && !xf) {
    c.f64x_ord.ensure((size_t)nb * kFB);
    ordr = c.f64x_ord.as<unsigned char>();
  }
  // The transfer cache (tcache != 0, the device run's steps): a block keeps
  // its transfers when none of its labels changed in this assignment and none
  // of its binade predictions moved since they were formed — its (cluster,
  // feature) sequences then hold the same values under the same binades, so
  // the transfers are the same integers.  Near convergence few blocks change.
  F64TCache tc;
  const bool use_tc = tcache != 0 && !xf && !ordr;
  if (use_tc) {
    const size_t need = sizeof(int) * (3 * (size_t)nb + 2);
    const bool fresh = c.f64x_dirty.bytes < need;
    c.f64x_dirty.ensure(need);
    int* base = c.f64x_dirty.as<int>();
    tc.dlab = base;
    tc.dE = base + nb;
    tc.list = base + 2 * nb;
    tc.counters = base + 3 * nb;
    tc.stamp = ++c.f64x_stamp;
    tc.par = tc.stamp & 1;
    tc.all = tcache == 1 || fresh;
    if (tc.all) HIP_CHECK(hipMemsetAsync(tc.counters, 0, 2 * sizeof(int), c.stream));
  }
  typedef void (*Fn)(const double*, int64_t, int64_t, const double*, int, int32_t*, double*,
                     unsigned*, const int*, Xfer*, unsigned char*, const long long*, const float*,
                     const int*, int*);
#define CDR_FAB(D_) f64_assign_block<D_, false>, f64_assign_block<D_, true>
  static const Fn fns[17][2] = {{nullptr, nullptr}, {CDR_FAB(1)},  {CDR_FAB(2)},  {CDR_FAB(3)},
                                {CDR_FAB(4)},       {CDR_FAB(5)},  {CDR_FAB(6)},  {CDR_FAB(7)},
                                {CDR_FAB(8)},       {CDR_FAB(9)},  {CDR_FAB(10)}, {CDR_FAB(11)},
                                {CDR_FAB(12)},      {CDR_FAB(13)}, {CDR_FAB(14)}, {CDR_FAB(15)},
                                {CDR_FAB(16)}};
#undef CDR_FAB
  const auto ctab = f64_cent_table(c, d, k, dC);
  hipLaunchKernelGGL(fns[d][xf ? 1 : 0], dim3((unsigned)nb), dim3(kFB), 0, c.stream,
                     c.x64.as<double>(), n, c.n_pad, dC, k, c.labels.as<int32_t>(),
                     c.f64x_A.as<double>(), c.f64x_cnt.as<unsigned>(), Ecur, c.f64x_T.as<Xfer>(),
                     ordr, gate, ctab.first, ctab.second,
                     use_tc ? const_cast<int*>(tc.dlab) : nullptr);
  HIP_CHECK(hipGetLastError());
  if (prof) prof_mark(c, 1);
  // (the counts: written by f64_predict_b from f64_predict_a's group counts)
  // with transfers formed under Ecur: predict into the other buffer, walk
  // under Ecur; else predict into Ecur and form the transfers under it
  int* Enew = xf ? Eoth : Ecur;
  sums_after_block<double, double>(c, c.x64.as<double>(), k, d_sums, Enew, xf ? Ecur : Enew, xf,
                                   ordr, F64Shard(), d_counts, use_tc ? &tc : nullptr);
  static const bool xcheck = exp_env("CDR_F64_XCHECK") != nullptr;
  if (xcheck && xf) {  // (diagnostics) the fused transfers vs f64_transfer under the same E
    DevBuf t2;
    t2.ensure(sizeof(Xfer) * nb * kd);
    const int nt = 64;  // (k <= 64)
    hipLaunchKernelGGL((f64_transfer<double, double, 6>), dim3(ceil_div(nb * d * kTQ, (int64_t)nt)), dim3(nt),
                       (size_t)nt * k * 20, c.stream, c.x64.as<double>(), n, c.n_pad, d, k, nb,
                       c.labels.as<int32_t>(), Ecur, t2.as<Xfer>(), (const int*)nullptr,
                       (const int*)nullptr);
    std::vector<Xfer> a(nb * kd), b(nb * kd);
    std::vector<int> e0(nb * kd), e1(nb * kd);
    HIP_CHECK(hipMemcpyAsync(a.data(), c.f64x_T.p, sizeof(Xfer) * a.size(), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipMemcpyAsync(b.data(), t2.p, sizeof(Xfer) * b.size(), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipMemcpyAsync(e0.data(), Ecur, sizeof(int) * e0.size(), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipMemcpyAsync(e1.data(), Enew, sizeof(int) * e1.size(), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    size_t bad = 0, ediff = 0, inval = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      if (a[i].d0 != b[i].d0 || a[i].dd != b[i].dd || a[i].flags != b[i].flags) {
        if (bad < 4)
          fprintf(stderr, "xcheck T[%zu]: fused (%lld,%d,%d) ref (%lld,%d,%d)\n", i, a[i].d0,
                  a[i].dd, a[i].flags, b[i].d0, b[i].dd, b[i].flags);
        ++bad;
      }
      ediff += e0[i] != e1[i];
      inval += (b[i].flags & 4) != 0;
    }
    fprintf(stderr, "xcheck: %zu of %zu transfers differ; E prev vs new differ %zu; ref invalid %zu\n",
            bad, a.size(), ediff, inval);
    t2.release();
  }
  if (xf) c.f64x_e_cur ^= 1;  // the new predictions are the next step's
  c.f64x_e_ok = true;
  c.f64x_e_k = k;
  c.f64x_e_nb = nb;
  return true;
}
// ---------------------------------------------------------------------------
// Sharded F64 sums (include/cdr.h cdr_f64s_*).  Rows are sharded in rank
// order, so sums[j][f] is the sequential sum over shard 0's members, then
// shard 1's, ...: every shard but the first needs the exact running value the
// earlier shards leave, which is not known until they are done.  Instead of a
// rank chain, every shard describes its part of each sequence as a PROGRAM
// built from approximate quantities only, and every rank runs all programs in
// rank order from the exact start:
//   * each rank all-gathers its approximate per-sequence totals (any order)
//     and member counts; a shard's blocks get their binade predictions from
//     the earlier shards' approximate total + its own approximate prefix
//     (f64_predict_*, offset), and their transfers under them (f64_transfer);
//   * rank 0 starts from the exact start (nothing), so it walks (f64_walk)
//     and publishes the exact result: CONST {s, any};
//   * rank r > 0 publishes, per sequence, RUN {e, D0, D1} for every maximal
//     run of member blocks predicted in one binade e with no crossing inside
//     (the start and end predictions agree) and usable transfers, composed
//     (xc_compose; whole groups from f64_group with the end condition), and
//     ELEM {x} for every member of any other block (a binade crossing, a
//     flagged transfer, the sequence's first member, a negative addend);
//   * composing (f64s_compose): a RUN applies only when the exact running
//     value is in its binade and stays there (the transfer test: exact, as
//     in f64_walk); ELEM adds x in real fp64 (NumPy's first row starts the
//     reduce).  Every rank composes the same all-gathered programs, so the
//     sums and the verdict are the same on every rank; a failed test (a
//     prediction off by a binade) or an overfull program makes every rank
//     take the exact rank chain instead (f64s_chain: each shard walks from
//     the exact entry in turn).
// ---------------------------------------------------------------------------
namespace {

struct F64Item {
  long long a, b;  // RUN: D0, D1; ELEM / CONST: the value's bits
  int e, kind;     // RUN: binade; CONST: any
};
static_assert(sizeof(F64Item) == 24, "item layout (include/cdr.h)");
constexpr int kF64Run = 1, kF64Elem = 2, kF64Const = 3;

// per-sequence approximate totals [k d] then member counts [k] (as doubles,
// exact below 2^53): one wave per row
__global__ __launch_bounds__(256) void f64s_totals(const double* __restrict__ A,
                                                   const unsigned* __restrict__ cnt, int64_t nb,
                                                   int kd, int k, double* __restrict__ out) {
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= kd + k) return;
  double v = 0.0;
  if (r < kd) {
    for (int64_t b = lane; b < nb; b += 64) v += A[(int64_t)r * nb + b];
  } else {
    unsigned long long c = 0;
    for (int64_t b = lane; b < nb; b += 64) c += cnt[(int64_t)(r - kd) * nb + b];
    v = (double)c;
  }
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if (lane == 0) out[r] = v;
}

// this rank's offsets (the earlier shards' approximate totals, added left to
// right) and the predicted binade at its end
__global__ __launch_bounds__(256) void f64s_offsets(const double* __restrict__ tot, int nranks,
                                                    int rank, int kd, int k,
                                                    double* __restrict__ off,
                                                    int* __restrict__ Eend) {
  const int stride = kd + k;
  for (int t = threadIdx.x; t < kd; t += blockDim.x) {
    double o = 0.0;
    for (int r = 0; r < rank; ++r) o += tot[(int64_t)r * stride + t];
    off[t] = o;
    Eend[t] = binade_e(o + tot[(int64_t)rank * stride + t]);
  }
}

// rank 0: the walk's exact result as one CONST item per sequence
__global__ __launch_bounds__(256) void f64s_const(const double* __restrict__ sums,
                                                  const double* __restrict__ tot, int kd, int d,
                                                  int k, int cap, F64Item* __restrict__ slot) {
  for (int t = threadIdx.x; t < kd; t += blockDim.x) {
    F64Item* it = slot + (int64_t)t * (cap + 1);
    const bool any = tot[kd + t / d] > 0.0;
    it[0] = F64Item{1, 0, 0, 0};
    it[1] = F64Item{__double_as_longlong(sums[t]), 0, any ? 1 : 0, kF64Const};
  }
}

// rank r > 0: one wave per (cluster, feature) sequence builds its program
// (header item: count, or -1 when it would exceed cap items)
template <typename TA>
__global__ __launch_bounds__(256) void f64s_program(const double* __restrict__ X, int64_t n,
                                                    int64_t n_pad, int d, int k, int64_t nb,
                                                    const int32_t* __restrict__ labels,
                                                    const unsigned* __restrict__ cnt,
                                                    const int* __restrict__ E,
                                                    const int* __restrict__ Eend,
                                                    const Xfer* __restrict__ T,
                                                    const GXfer* __restrict__ G, int64_t ng,
                                                    int cap, F64Item* __restrict__ slot) {
  const int t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (t >= k * d) return;
  const int j = t / d, f = t % d;
  F64Item* out = slot + (int64_t)t * (cap + 1);
  int nit = 0;  // items so far (wave-uniform)
  auto emit = [&](long long a, long long b, int e, int kind) {
    if (nit < cap && lane == 0) out[1 + nit] = F64Item{a, b, e, kind};
    ++nit;
  };
  bool run_on = false;
  int run_e = kENone;
  XferC run{0, 0, 2};
  auto add_run = [&](int e, long long d0, long long d1, int p) {
    const XferC x{d0, d1, p};
    if (run_on && run_e == e) {
      run = xc_compose(run, x);
    } else {
      if (run_on) emit(run.d0, run.d1, run_e, kF64Run);
      run = x;
      run_e = e;
      run_on = true;
    }
  };
  auto rd64 = [&](long long v, int l) {
    return (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(v >> 32), l)
                        << 32) |
                       (unsigned)__builtin_amdgcn_readlane((int)v, l));
  };
  const GXfer* Gt = G + (int64_t)t * ng;
  for (int64_t g0 = 0; g0 < ng; g0 += 64) {
    const GXfer gl = g0 + lane < ng ? Gt[g0 + lane] : GXfer{0, 0, kENone, 0};
    unsigned long long todo = __ballot((gl.p & 8) != 0);
    while (todo) {
      const int gi = __builtin_amdgcn_readfirstlane(__ffsll((long long)todo) - 1);
      todo &= todo - 1;
      const int gp = __builtin_amdgcn_readlane(gl.p, gi);
      if (gp & 4) {  // every member usable, one binade, no crossing inside
        add_run(__builtin_amdgcn_readlane(gl.e, gi), rd64(gl.d0, gi), rd64(gl.d1, gi), gp & 3);
        continue;
      }
      const int64_t b0 = (g0 + gi) * 64;
      const int64_t bl = b0 + lane;
      const bool in = bl < nb;
      const unsigned c = in ? cnt[(int64_t)j * nb + bl] : 0u;
      const int el = in ? E[(int64_t)t * nb + bl] : kENone;
      const int ea = in ? (bl + 1 < nb ? E[(int64_t)t * nb + bl + 1] : Eend[t]) : kENone;
      const Xfer xl = in ? T[(int64_t)t * nb + bl] : Xfer{0, 0, 4};
      const bool safe = c != 0 && !(xl.flags & 4) && el != kENone && ea == el;
      unsigned long long mem = __ballot(c != 0);
      const unsigned long long sm = __ballot(safe);
      while (mem) {
        const int i = __builtin_amdgcn_readfirstlane(__ffsll((long long)mem) - 1);
        mem &= mem - 1;
        if ((sm >> i) & 1ull) {
          const long long d0 = rd64(xl.d0, i);
          const int dd = __builtin_amdgcn_readlane(xl.dd, i);
          add_run(__builtin_amdgcn_readlane(el, i), d0, d0 + dd,
                  __builtin_amdgcn_readlane(xl.flags, i) & 3);
          continue;
        }
        // the block's members one by one (row order)
        if (run_on) emit(run.d0, run.d1, run_e, kF64Run);
        run_on = false;
        const int64_t r0 = (b0 + i) * kFB;
        int lj[4];
        double lx[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t row = r0 + 64 * q + lane;
          lj[q] = row < n ? labels[row] : -1;
          lx[q] = row < n ? (double)X[xidx(X, f, row, n_pad)] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          unsigned long long mk = __ballot(lj[q] == j);
          while (mk) {
            const int l = __builtin_amdgcn_readfirstlane(__ffsll((long long)mk) - 1);
            mk &= mk - 1;
            emit(rd64(__double_as_longlong(lx[q]), l), 0, 0, kF64Elem);
          }
        }
      }
    }
  }
  if (run_on) emit(run.d0, run.d1, run_e, kF64Run);
  if (lane == 0) out[0] = F64Item{nit <= cap ? nit : -1, 0, 0, 0};
}

// every rank: the programs of ranks 0 .. nranks-1 in order, one thread per
// sequence; sums[t], counts[j] (exact, from the gathered totals), and
// status |= 1 when a RUN's transfer test failed or a program overflowed
template <typename TA>
__global__ __launch_bounds__(256) void f64s_compose(const F64Item* __restrict__ progs,
                                                    int64_t slot_items, const double* __restrict__ tot,
                                                    int nranks, int kd, int k, int cap,
                                                    double* __restrict__ sums,
                                                    long long* __restrict__ counts,
                                                    int* __restrict__ status) {
  constexpr int MB = SumTraits<TA>::MB, kMinE = SumTraits<TA>::kMinE;
  constexpr long long kTop = 1ll << (MB + 1);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < k) {
    double c = 0.0;
    for (int r = 0; r < nranks; ++r) c += tot[(int64_t)r * (kd + k) + kd + t];
    counts[t] = (long long)c;
  }
  if (t >= kd) return;
  double s = 0.0;
  bool any = false, ok = true;
  for (int r = 0; r < nranks && ok; ++r) {
    const F64Item* it = progs + (int64_t)r * slot_items + (int64_t)t * (cap + 1);
    const long long m = it[0].a;
    if (m < 0 || m > cap) {
      ok = false;
      break;
    }
    for (long long i = 1; i <= m; ++i) {
      const F64Item x = it[i];
      if (x.kind == kF64Run) {
        ok = false;
        if (any && s > 0.0) {
          int ex;
          frexp(s, &ex);
          if (ex - 1 == x.e && x.e >= kMinE) {
            const long long g = (long long)ldexp(s, MB - x.e);  // exact: s is on the grid
            const long long g2 = g + ((g & 1) ? x.b : x.a);
            if (g2 < kTop) {
              s = ldexp((double)g2, x.e - MB);
              ok = true;
            }
          }
        }
        if (!ok) break;
      } else if (x.kind == kF64Elem) {
        const double v = __longlong_as_double(x.a);
        s = any ? (double)((TA)s + (TA)v) : v;  // NumPy's reduce: the first row starts it
        any = true;
      } else if (x.kind == kF64Const) {
        s = __longlong_as_double(x.a);
        any = x.e != 0;
      }
    }
  }
  sums[t] = s;
  if (!ok) atomicOr(status, 1);
}

}  // namespace

int f64s_cap() {
  static const int cap = exp_env("CDR_F64S_CAP") ? std::max(1, std::atoi(exp_env("CDR_F64S_CAP"))) : 127;
  return cap;
}

// The step's assignment (labels, block sums and counts) and this shard's
// totals into tot_slot (k d + k doubles).  false: shape not covered.
bool f64s_assign_totals(Ctx& c, int k, const double* dC, double* tot_slot) {
  const int d = c.d;
  if (d < 2 || d > 16 || k < 1 || k > kFMaxK) return false;
  const int64_t n = c.n, nb = ceil_div(std::max<int64_t>(n, 1), kFB);
  const size_t kd = (size_t)k * d;
  c.f64x_A.ensure(sizeof(double) * nb * kd);
  c.f64x_cnt.ensure(sizeof(unsigned) * nb * k);
  c.f64x_E.ensure(sizeof(int) * nb * kd);
  c.f64x_T.ensure(sizeof(Xfer) * nb * kd);
  c.f64x_walk.ensure(sizeof(long long) * kd);
  c.f64x_e_ok = false;  // (the fused step's carried predictions belong to other rows)
  if (n > 0) {
    typedef void (*Fn)(const double*, int64_t, int64_t, const double*, int, int32_t*, double*,
                       unsigned*, const int*, Xfer*, unsigned char*, const long long*,
                       const float*, const int*, int*);
    static const Fn fns[17] = {nullptr, f64_assign_block<1, false>, f64_assign_block<2, false>,
                               f64_assign_block<3, false>, f64_assign_block<4, false>,
                               f64_assign_block<5, false>, f64_assign_block<6, false>,
                               f64_assign_block<7, false>, f64_assign_block<8, false>,
                               f64_assign_block<9, false>, f64_assign_block<10, false>,
                               f64_assign_block<11, false>, f64_assign_block<12, false>,
                               f64_assign_block<13, false>, f64_assign_block<14, false>,
                               f64_assign_block<15, false>, f64_assign_block<16, false>};
    const auto ctab = f64_cent_table(c, d, k, dC);
    hipLaunchKernelGGL(fns[d], dim3((unsigned)nb), dim3(kFB), 0, c.stream, c.x64.as<double>(), n,
                       c.n_pad, dC, k, c.labels.as<int32_t>(), c.f64x_A.as<double>(),
                       c.f64x_cnt.as<unsigned>(), c.f64x_E.as<int>(), c.f64x_T.as<Xfer>(),
                       nullptr, nullptr, ctab.first, ctab.second, nullptr);
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(f64s_totals, dim3((unsigned)ceil_div((int64_t)kd + k, 4)), dim3(256), 0,
                       c.stream, c.f64x_A.as<double>(), c.f64x_cnt.as<unsigned>(), nb, (int)kd, k,
                       tot_slot);
  } else {
    HIP_CHECK(hipMemsetAsync(tot_slot, 0, sizeof(double) * (kd + k), c.stream));
  }
  HIP_CHECK(hipGetLastError());
  return true;
}

// This shard's program into its slot of prog_all ([nranks][k d][cap + 1]
// items) from the gathered totals tot_all ([nranks][k d + k]).
void f64s_build(Ctx& c, int k, int nranks, int rank, const double* tot_all, void* prog_all) {
  const int d = c.d, cap = f64s_cap();
  const int64_t n = c.n, nb = ceil_div(std::max<int64_t>(n, 1), kFB);
  const int kd = k * d;
  const int64_t slot_items = (int64_t)kd * (cap + 1);
  F64Item* slot = static_cast<F64Item*>(prog_all) + (size_t)rank * slot_items;
  c.f64s_off.ensure(sizeof(double) * kd + sizeof(int) * kd);
  double* off = c.f64s_off.as<double>();
  int* Eend = reinterpret_cast<int*>(off + kd);
  hipLaunchKernelGGL(f64s_offsets, dim3(1), dim3(256), 0, c.stream, tot_all, nranks, rank, kd, k,
                     off, Eend);
  HIP_CHECK(hipGetLastError());
  c.f64_sums.ensure(sizeof(double) * 2 * kd);
  if (n > 0) {
    F64Shard sh;
    sh.off = off;
    sh.Eend = rank > 0 ? Eend : nullptr;  // (rank 0 walks: no crossing condition needed)
    sh.walk = rank == 0;
    sums_after_block<double, double>(c, c.x64.as<double>(), k, c.f64_sums.as<double>(),
                                     c.f64x_E.as<int>(), c.f64x_E.as<int>(), false, nullptr, sh);
  }
  if (rank == 0) {
    if (n == 0) HIP_CHECK(hipMemsetAsync(c.f64_sums.p, 0, sizeof(double) * kd, c.stream));
    hipLaunchKernelGGL(f64s_const, dim3(1), dim3(256), 0, c.stream, c.f64_sums.as<double>(),
                       tot_all, kd, d, k, cap, slot);
  } else if (n > 0) {
    const int64_t ng = ceil_div(nb, (int64_t)64);
    hipLaunchKernelGGL(f64s_program<double>, dim3((unsigned)ceil_div((int64_t)kd, 4)), dim3(256), 0,
                       c.stream, c.x64.as<double>(), n, c.n_pad, d, k, nb,
                       c.labels.as<int32_t>(), c.f64x_cnt.as<unsigned>(), c.f64x_E.as<int>(),
                       Eend, c.f64x_T.as<Xfer>(), c.f64x_G.as<GXfer>(), ng, cap, slot);
  } else {  // an empty shard: the identity (no items)
    std::vector<F64Item> z((size_t)slot_items, F64Item{0, 0, 0, 0});
    HIP_CHECK(hipMemcpyAsync(slot, z.data(), sizeof(F64Item) * z.size(), hipMemcpyHostToDevice,
                             c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
  }
  HIP_CHECK(hipGetLastError());
}

void f64s_compose_all(Ctx& c, int k, int nranks, const double* tot_all, const void* prog_all,
                      double* d_sums, long long* d_counts, int* d_status) {
  const int kd = k * c.d, cap = f64s_cap();
  const int64_t slot_items = (int64_t)kd * (cap + 1);
  HIP_CHECK(hipMemsetAsync(d_status, 0, sizeof(int), c.stream));
  hipLaunchKernelGGL(f64s_compose<double>, dim3((unsigned)ceil_div(std::max(kd, k), 256)),
                     dim3(256), 0, c.stream, static_cast<const F64Item*>(prog_all), slot_items,
                     tot_all, nranks, kd, k, cap, d_sums, d_counts, d_status);
  HIP_CHECK(hipGetLastError());
}

// The exact rank chain (fallback): this shard walks from the exact entry
// chain[0, 2 k d) = {s, any} and leaves its exit there.
void f64s_chain_walk(Ctx& c, int k, double* chain) {
  const int kd = k * c.d;
  if (c.n == 0) return;  // nothing added: the entry is the exit
  F64Shard sh;
  sh.off = chain;  // the exact entry predicts every binade
  sh.entry = chain;
  sh.walk = true;
  c.f64s_off.ensure(sizeof(double) * kd + sizeof(int) * kd);
  sums_after_block<double, double>(c, c.x64.as<double>(), k, chain, c.f64x_E.as<int>(),
                                   c.f64x_E.as<int>(), false, nullptr, sh);
}

// The reference's float32 runs: sequential fp32 sums of fp32 points (X:
// F32X storage, or F64 storage holding fp32 values), returned as doubles.
bool f32_sums_parallel(Ctx& c, int k, double* d_sums) {
  if (c.mode == CDR_MODE_F32X) return sums_parallel<float, float>(c, c.x32.as<float>(), k, d_sums);
  return sums_parallel<float, double>(c, c.x64.as<double>(), k, d_sums);
}

}  // namespace cdr
