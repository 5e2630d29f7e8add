// radix.hip — hand-written stable LSD radix sort of (key, value) pairs, the
// group-by's fallback for shapes its packed partition cannot hold (features.hip:
// over ~268M files per rank, seconds beyond 2^40, (file, second) keys over 40
// bits).  Replaces the library sort the fallback used before round 5.
//
// One pass per 8-bit digit of [0, end_bit), four kernels each:
//   rs_hist     per tile of kRsTile elements: the digit counts, stored
//               digit-major ([digit][tile]) for the scan
//   rs_scan     one workgroup per digit: the exclusive prefix of its tile
//               counts (in place) and the digit's total
//   rs_base     the digits' bases (exclusive scan of the 256 totals)
//   rs_scatter  per tile, in element order chunk by chunk (256 elements per
//               chunk, one per thread): a stable rank among equal digits
//               (peers from 8 ballots, earlier waves' and chunks' counts from
//               LDS), then the element to its place
// Stable, so keys sorted on a later digit keep the earlier digits' order: the
// time-ordered fast path relies on it (events of a file stay in time order).
#include <cstdint>

#include "cdr_internal.h"

namespace cdr {

namespace {

constexpr int kRsThreads = 256;
constexpr int kRsItems = 16;                     // chunks per tile
constexpr int kRsTile = kRsThreads * kRsItems;   // elements per tile
constexpr int kRsBins = 256;

template <typename K>
__device__ __forceinline__ unsigned rs_digit(K k, int shift) {
  return (unsigned)((unsigned long long)k >> shift) & 255u;
}

template <typename K>
__global__ __launch_bounds__(kRsThreads) void rs_hist(const K* __restrict__ keys, int64_t n,
                                                      int shift, int64_t ntiles,
                                                      unsigned* __restrict__ th) {
  __shared__ unsigned h[kRsBins];
  const int t = threadIdx.x;
  const int64_t tile = blockIdx.x;
  h[t] = 0;
  __syncthreads();
  const int64_t base = tile * kRsTile;
#pragma unroll
  for (int c = 0; c < kRsItems; ++c) {
    const int64_t i = base + (int64_t)c * kRsThreads + t;
    if (i < n) atomicAdd(&h[rs_digit(keys[i], shift)], 1u);
  }
  __syncthreads();
  th[(int64_t)t * ntiles + tile] = h[t];
}

// one workgroup per digit: the exclusive prefix of its tiles' counts (in
// place) and the digit's total
__global__ __launch_bounds__(kRsThreads) void rs_scan(unsigned* __restrict__ th, int64_t ntiles,
                                                      unsigned long long* __restrict__ dtot) {
  __shared__ unsigned wsum[kRsThreads / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int dgt = blockIdx.x;
  unsigned* row = th + (int64_t)dgt * ntiles;
  unsigned long long carry = 0;
  for (int64_t t0 = 0; t0 < ntiles; t0 += kRsThreads) {
    const int64_t i = t0 + t;
    const unsigned v = i < ntiles ? row[i] : 0u;
    unsigned inc = v;
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned u = __shfl_up(inc, o);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    unsigned wb = 0;
    for (int q = 0; q < w; ++q) wb += wsum[q];
    if (i < ntiles) row[i] = (unsigned)(carry + wb + inc - v);
    const unsigned tot = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
    __syncthreads();
    carry += tot;
  }
  if (t == 0) dtot[dgt] = carry;
}

// the digits' bases: an exclusive scan of the 256 totals (one workgroup)
__global__ __launch_bounds__(kRsThreads) void rs_base(unsigned long long* __restrict__ dtot) {
  __shared__ unsigned long long v[kRsBins];
  const int t = threadIdx.x;
  v[t] = dtot[t];
  __syncthreads();
  if (t == 0) {
    unsigned long long s = 0;
    for (int i = 0; i < kRsBins; ++i) {
      const unsigned long long x = v[i];
      v[i] = s;
      s += x;
    }
  }
  __syncthreads();
  dtot[t] = v[t];
}

template <typename K, typename V>
__global__ __launch_bounds__(kRsThreads) void rs_scatter(const K* __restrict__ kin,
                                                         const V* __restrict__ vin, int64_t n,
                                                         int shift, int64_t ntiles,
                                                         const unsigned* __restrict__ th,
                                                         const unsigned long long* __restrict__ dbase,
                                                         K* __restrict__ kout,
                                                         V* __restrict__ vout) {
  __shared__ unsigned run[kRsBins];                    // this tile's elements placed so far
  __shared__ unsigned wcnt[kRsThreads / 64][kRsBins];  // this chunk's per-wave counts
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t tile = blockIdx.x;
  run[t] = (unsigned)(dbase[t] + th[(int64_t)t * ntiles + tile]);  // the tile's first slot of digit t
  const int64_t base = tile * kRsTile;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int c = 0; c < kRsItems; ++c) {
    const int64_t i = base + (int64_t)c * kRsThreads + t;
    const bool in = i < n;
    K k = 0;
    V v = 0;
    if (in) {
      k = kin[i];
      v = vin[i];
    }
    const unsigned dg = in ? rs_digit(k, shift) : 0u;
    // lanes of this wave with the same digit (8 ballots)
    unsigned long long peers = __ballot(in);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const unsigned long long m = __ballot((dg >> b) & 1u);
      peers &= ((dg >> b) & 1u) ? m : ~m;
    }
    if (!in) peers = 0;
    const unsigned rank = (unsigned)__popcll(peers & below);
    for (int e = lane; e < kRsBins; e += 64) wcnt[w][e] = 0;
    __syncthreads();
    // the lowest lane of each peer group publishes its wave's count
    if (in && (peers & below) == 0) wcnt[w][dg] = (unsigned)__popcll(peers);
    __syncthreads();
    if (in) {
      unsigned pos = run[dg] + rank;
      for (int q = 0; q < w; ++q) pos += wcnt[q][dg];
      kout[pos] = k;
      vout[pos] = v;
    }
    __syncthreads();
    // this chunk's counts into the running slots (thread t: digit t)
    run[t] += (wcnt[0][t] + wcnt[1][t]) + (wcnt[2][t] + wcnt[3][t]);
    __syncthreads();
  }
}

}  // namespace

// Sorts n (key, value) pairs stably by key bits [0, end_bit), ping-ponging
// between (k0, v0) and (k1, v1); returns true when the result is in (k1, v1).
template <typename K, typename V>
bool radix_sort_pairs(Ctx& c, K* k0, K* k1, V* v0, V* v1, int64_t n, int end_bit) {
  if (n <= 1 || end_bit <= 0) return false;
  const int64_t ntiles = ceil_div(n, (int64_t)kRsTile);
  if (n >= (int64_t(1) << 32)) CDR_FAIL(CDR_ERR_UNSUPPORTED, "radix sort: n >= 2^32");
  c.rs_hist.ensure(sizeof(unsigned) * (size_t)kRsBins * ntiles + sizeof(unsigned long long) * kRsBins);
  unsigned* th = c.rs_hist.as<unsigned>();
  unsigned long long* dtot = reinterpret_cast<unsigned long long*>(th + (size_t)kRsBins * ntiles);
  bool flip = false;
  for (int shift = 0; shift < end_bit; shift += 8) {
    const K* ki = flip ? k1 : k0;
    const V* vi = flip ? v1 : v0;
    K* ko = flip ? k0 : k1;
    V* vo = flip ? v0 : v1;
    hipLaunchKernelGGL((rs_hist<K>), dim3((unsigned)ntiles), dim3(kRsThreads), 0, c.stream, ki, n,
                       shift, ntiles, th);
    hipLaunchKernelGGL(rs_scan, dim3(kRsBins), dim3(kRsThreads), 0, c.stream, th, ntiles, dtot);
    hipLaunchKernelGGL(rs_base, dim3(1), dim3(kRsThreads), 0, c.stream, dtot);
    hipLaunchKernelGGL((rs_scatter<K, V>), dim3((unsigned)ntiles), dim3(kRsThreads), 0, c.stream,
                       ki, vi, n, shift, ntiles, th, dtot, ko, vo);
    HIP_CHECK(hipGetLastError());
    flip = !flip;
  }
  return flip;
}

template bool radix_sort_pairs<unsigned, unsigned long long>(Ctx&, unsigned*, unsigned*,
                                                             unsigned long long*,
                                                             unsigned long long*, int64_t, int);
template bool radix_sort_pairs<unsigned long long, uint8_t>(Ctx&, unsigned long long*,
                                                            unsigned long long*, uint8_t*,
                                                            uint8_t*, int64_t, int);

}  // namespace cdr
