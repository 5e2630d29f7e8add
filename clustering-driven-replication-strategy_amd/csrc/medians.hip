// medians.hip — per-cluster per-feature medians (reference src/scoring.py:40-55).
//
// np.median(list) of m values: the elements of sorted rank (m-1)/2 and m/2
// (0-based), then np.mean of those one or two values, i.e. ((0.0 + a) + b) / 2
// (or (0.0 + a) / 1): the sum starts from +0.0, so median([-0.0]) is +0.0.
// Empty -> NaN; any NaN -> NaN (numpy _median_nancheck).
//
// Selection is an MSB radix select over order-preserving unsigned keys, one
// workgroup per segment: each pass histograms (in LDS) the 8-bit digit of the
// elements that still match the prefix found so far, for both target ranks.
// 64-bit keys (fp64 values) take 8 passes, 32-bit keys (F32X points) take 4.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "cdr_internal.h"

namespace cdr {

__device__ __forceinline__ unsigned long long okey64(double v) {
  const unsigned long long b = __double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double from_okey64(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double(b);
}
__device__ __forceinline__ unsigned okey32(float v) {
  const unsigned b = __float_as_uint(v);
  return (b >> 31) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float from_okey32(unsigned k) {
  const unsigned b = (k >> 31) ? (k & 0x7FFFFFFFu) : ~k;
  return __uint_as_float(b);
}

template <typename V>
struct KeyOf;
template <>
struct KeyOf<double> {
  typedef unsigned long long K;
  static constexpr int BITS = 64;
  __device__ static K key(double v) { return okey64(v); }
  __device__ static double val(K k) { return from_okey64(k); }
  __device__ static bool isnan_(double v) { return isnan(v); }
};
template <>
struct KeyOf<float> {
  typedef unsigned K;
  static constexpr int BITS = 32;
  __device__ static K key(float v) { return okey32(v); }
  __device__ static double val(K k) { return (double)from_okey32(k); }
  __device__ static bool isnan_(float v) { return isnan(v); }
};

// Segment s = vals[off[s] .. off[s+1]) (element stride 1).  out[s] = median.
template <typename V>
__global__ __launch_bounds__(256) void seg_median_kernel(const V* __restrict__ vals,
                                                         const int64_t* __restrict__ off,
                                                         int64_t nseg, double* __restrict__ out) {
  typedef typename KeyOf<V>::K K;
  __shared__ unsigned hist[2][256];
  __shared__ K sprefix[2];
  __shared__ long long srank[2];
  __shared__ int snan;
  for (int64_t s = blockIdx.x; s < nseg; s += gridDim.x) {
    const int64_t lo = off[s], hi = off[s + 1];
    const int64_t m = hi - lo;
    if (m <= 0) {
      if (threadIdx.x == 0) out[s] = NAN;
      continue;
    }
    if (threadIdx.x == 0) snan = 0;
    __syncthreads();
    int anynan = 0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) anynan |= KeyOf<V>::isnan_(vals[i]);
    if (anynan) atomicOr(&snan, 1);
    __syncthreads();
    if (snan) {
      if (threadIdx.x == 0) out[s] = NAN;
      __syncthreads();
      continue;
    }
    if (threadIdx.x == 0) {
      sprefix[0] = 0;
      sprefix[1] = 0;
      srank[0] = (m - 1) / 2;
      srank[1] = m / 2;
    }
    __syncthreads();
    K mask = 0;
    for (int shift = KeyOf<V>::BITS - 8; shift >= 0; shift -= 8) {
      for (int i = threadIdx.x; i < 512; i += blockDim.x) (&hist[0][0])[i] = 0;
      __syncthreads();
      const K p0 = sprefix[0], p1 = sprefix[1];
      const bool two = p0 != p1;
      for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        const K key = KeyOf<V>::key(vals[i]);
        const unsigned dig = (unsigned)((key >> shift) & 0xFF);
        if ((key & mask) == p0) atomicAdd(&hist[0][dig], 1u);
        if (two && (key & mask) == p1) atomicAdd(&hist[1][dig], 1u);
      }
      __syncthreads();
      if (threadIdx.x < 2) {
        const int w = threadIdx.x;
        const int hsel = (w == 1 && !two) ? 0 : w;
        long long r = srank[w];
        unsigned dsel = 255;
        for (unsigned dgt = 0; dgt < 256; ++dgt) {
          const long long c = hist[hsel][dgt];
          if (r < c) {
            dsel = dgt;
            break;
          }
          r -= c;
        }
        srank[w] = r;
        sprefix[w] = (w == 0 ? p0 : p1) | ((K)dsel << shift);
      }
      mask |= ((K)0xFF << shift);
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      const double a = KeyOf<V>::val(sprefix[0]);
      if (m & 1) {
        out[s] = (0.0 + a) / 1.0;
      } else {
        const double b = KeyOf<V>::val(sprefix[1]);
        out[s] = ((0.0 + a) + b) / 2.0;
      }
    }
    __syncthreads();
  }
}

// ---- medians of the resident points grouped by label (main.py:96-107) ----
// The rows of each cluster are gathered once into a point-major copy (a
// two-pass counting sort: per-block LDS label counts, a column scan for the
// block offsets, a scatter with LDS ranks: no global cursor atomics), then
// every (cluster, feature) pair is selected by an MSB radix select over
// order-preserving keys, 8 bits per pass, for both middle ranks at once: one
// workgroup per cluster and 64-feature chunk histograms its rows in LDS
// ([64][2][256] counters), the histograms go to global memory (where a
// sharded run all-reduces them), and one thread per pair
// picks the next digit of each rank.  Ranks are of the global cluster sizes.
constexpr int kMgBlock = 4096;   // points per counting-sort block
constexpr int kMgRange = 64;     // blocks per column-scan range
constexpr int kMgMaxK = 8192;
constexpr int kMgFeat = 64;      // features per histogram workgroup

__global__ __launch_bounds__(256) void mg_count(const int32_t* __restrict__ labels, int64_t n,
                                                int k, unsigned* __restrict__ cnt) {
  extern __shared__ unsigned hc[];
  for (int j = threadIdx.x; j < k; j += 256) hc[j] = 0;
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * kMgBlock;
  for (int i = threadIdx.x; i < kMgBlock; i += 256)
    if (i0 + i < n) atomicAdd(&hc[labels[i0 + i]], 1u);
  __syncthreads();
  for (int j = threadIdx.x; j < k; j += 256) cnt[(int64_t)blockIdx.x * k + j] = hc[j];
}

// column scan of cnt [nblk][k]: a) range sums, b) range bases + label totals
// and bases (one workgroup), c) absolute block offsets in place
__global__ __launch_bounds__(256) void mg_scan_a(const unsigned* __restrict__ cnt, int64_t nblk,
                                                 int k, unsigned long long* __restrict__ rsum) {
  const int64_t r0 = (int64_t)blockIdx.x * kMgRange;
  for (int j = threadIdx.x; j < k; j += 256) {
    unsigned long long s = 0;
    for (int r = 0; r < kMgRange && r0 + r < nblk; ++r) s += cnt[(r0 + r) * k + j];
    rsum[(int64_t)blockIdx.x * k + j] = s;
  }
}

__global__ __launch_bounds__(1024) void mg_scan_b(unsigned long long* __restrict__ rsum,
                                                  int64_t nr, int k,
                                                  long long* __restrict__ base,
                                                  long long* __restrict__ total) {
  __shared__ long long wsum[16];
  __shared__ long long carry;
  for (int j = threadIdx.x; j < k; j += 1024) {
    unsigned long long run = 0;
    for (int64_t r = 0; r < nr; ++r) {
      const unsigned long long v = rsum[r * k + j];
      rsum[r * k + j] = run;
      run += v;
    }
    total[j] = (long long)run;
  }
  __syncthreads();
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int j0 = 0; j0 < k; j0 += 1024) {
    const int j = j0 + threadIdx.x;
    const long long v = j < k ? total[j] : 0;
    long long inc = v;
    for (int o = 1; o < 64; o <<= 1) {
      const long long u = __shfl_up(inc, o);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    long long pre = carry;
    for (int q = 0; q < w; ++q) pre += wsum[q];
    if (j < k) base[j] = pre + inc - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = pre + inc;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void mg_scan_c(unsigned* __restrict__ cnt, int64_t nblk, int k,
                                                 const unsigned long long* __restrict__ rbase,
                                                 const long long* __restrict__ base) {
  const int64_t r0 = (int64_t)blockIdx.x * kMgRange;
  for (int j = threadIdx.x; j < k; j += 256) {
    unsigned long long run = (unsigned long long)base[j] + rbase[(int64_t)blockIdx.x * k + j];
    for (int r = 0; r < kMgRange && r0 + r < nblk; ++r) {
      const unsigned v = cnt[(r0 + r) * k + j];
      cnt[(r0 + r) * k + j] = (unsigned)run;
      run += v;
    }
  }
}

// Ranks first (one thread per point, LDS cursors), then the rows copied with
// the lanes of a wave over (point, feature): each point's row is written as
// one contiguous run.
template <typename V>
__global__ __launch_bounds__(256) void mg_scatter(const V* __restrict__ X, int64_t n,
                                                  int64_t n_pad, int d,
                                                  const int32_t* __restrict__ labels, int k,
                                                  const unsigned* __restrict__ off,
                                                  V* __restrict__ rows) {
  extern __shared__ unsigned cur[];
  __shared__ unsigned pos[kMgBlock];
  for (int j = threadIdx.x; j < k; j += 256) cur[j] = off[(int64_t)blockIdx.x * k + j];
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * kMgBlock;
  const int np = (int)min((int64_t)kMgBlock, n - i0);
  for (int i = threadIdx.x; i < np; i += 256) pos[i] = atomicAdd(&cur[labels[i0 + i]], 1u);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int D2 = 1;
  while (D2 < d && D2 < 64) D2 <<= 1;
  const int rpw = 64 / D2;                    // points per wave step
  const int sub = lane / D2, fl = lane % D2;
  for (int p0 = w * rpw; p0 < np; p0 += 4 * rpw) {
    const int pi = p0 + sub;
    if (pi >= np) continue;
    V* dst = rows + (int64_t)pos[pi] * d;
    for (int f = fl; f < d; f += D2) dst[f] = X[xidx(X, f, i0 + pi, n_pad)];
  }
}

// Pass p (digit shift sh) for cluster j = blockIdx.x, features [f0, f0 + 64):
// counts of the digit among the rows whose key matches each rank's prefix.
// Both ranks share one histogram while their prefixes are equal (flag in
// two[]), as the selection step reads it.
template <typename V>
__global__ __launch_bounds__(1024) void mg_hist(const V* __restrict__ rows, int d, int k,
                                                const long long* __restrict__ base,
                                                const long long* __restrict__ cnt_local,
                                                const unsigned long long* __restrict__ pref,
                                                int sh, unsigned* __restrict__ H) {
  typedef typename KeyOf<V>::K K;
  // counters of feature f, rank t, digit g at f * kMgHs + t * 257 + g: the
  // odd strides put the lanes of a wave (different features, often the same
  // digit) in different banks
  constexpr int kMgHs = 515;
  constexpr int kU = 8;  // rows in flight per lane
  __shared__ unsigned h[kMgFeat * kMgHs];
  __shared__ K sp[kMgFeat][2];
  const int j = blockIdx.x;
  const int f0 = blockIdx.y * kMgFeat;
  const int nfc = min(kMgFeat, d - f0);
  for (int i = threadIdx.x; i < kMgFeat * kMgHs; i += 1024) h[i] = 0;
  for (int i = threadIdx.x; i < 2 * nfc; i += 1024)
    sp[i >> 1][i & 1] = (K)pref[((int64_t)j * d + f0) * 2 + i];
  __syncthreads();
  const K mask = sh + 8 >= KeyOf<V>::BITS ? (K)0 : (K)(~(K)0 << (sh + 8));
  const int64_t lo = base[j], m = cnt_local[j];
  // lanes over (row, feature): a wave reads whole rows (contiguous) and, for
  // d >= 64, its lanes count different features (no counter shared in a
  // wave); kU rows per lane are loaded before any is counted
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int D2 = 1;
  while (D2 < nfc) D2 <<= 1;
  const int rpw = 64 / D2;
  const int sub = lane / D2, f = lane % D2;
  if (f < nfc) {
    const K p0 = sp[f][0], p1 = sp[f][1];
    const bool two = p1 != p0;
    const int64_t step = (int64_t)16 * rpw;  // 16 waves
    for (int64_t r0 = (int64_t)w * rpw + sub; r0 < m; r0 += kU * step) {
      V v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t r = r0 + u * step;
        v[u] = r < m ? rows[(lo + r) * d + f0 + f] : (V)0;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (r0 + u * step >= m) break;
        const K key = KeyOf<V>::key(v[u]);
        const unsigned dig = (unsigned)((key >> sh) & 0xFF);
        if ((key & mask) == p0) atomicAdd(&h[f * kMgHs + dig], 1u);
        if (two && (key & mask) == p1) atomicAdd(&h[f * kMgHs + 257 + dig], 1u);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nfc * 512; i += 1024) {
    const int ff = i >> 9, t = (i >> 8) & 1, g = i & 255;
    H[((int64_t)j * d + f0) * 512 + i] = h[ff * kMgHs + t * 257 + g];
  }
}

// One thread per (cluster, feature): the next digit of both ranks.
template <typename V>
__global__ void mg_select(const unsigned* __restrict__ H, int d, int k,
                          const long long* __restrict__ cnt_global, int sh,
                          unsigned long long* __restrict__ pref, long long* __restrict__ rank) {
  typedef typename KeyOf<V>::K K;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= k * d) return;
  if (cnt_global[t / d] <= 0) return;
  const K p0 = (K)pref[2 * t], p1 = (K)pref[2 * t + 1];
  const bool two = p0 != p1;
  for (int w = 0; w < 2; ++w) {
    const unsigned* hist = H + (int64_t)t * 512 + ((w == 1 && two) ? 256 : 0);
    long long r = rank[2 * t + w];
    unsigned dsel = 255;
    for (unsigned g = 0; g < 256; ++g) {
      const long long c = hist[g];
      if (r < c) {
        dsel = g;
        break;
      }
      r -= c;
    }
    rank[2 * t + w] = r;
    pref[2 * t + w] = (unsigned long long)((w == 0 ? p0 : p1) | ((K)dsel << sh));
  }
}

template <typename V>
__global__ void mg_finish(const long long* __restrict__ cnt_global, int d, int k,
                          const unsigned long long* __restrict__ pref, double* __restrict__ out) {
  typedef typename KeyOf<V>::K K;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= k * d) return;
  const long long m = cnt_global[t / d];
  if (m <= 0) {
    out[t] = NAN;
    return;
  }
  const double a = KeyOf<V>::val((K)pref[2 * t]);
  if (m & 1) {
    out[t] = (0.0 + a) / 1.0;
  } else {
    const double b = KeyOf<V>::val((K)pref[2 * t + 1]);
    out[t] = ((0.0 + a) + b) / 2.0;
  }
}

__global__ void mg_begin(const long long* __restrict__ cnt_global, int d, int k,
                         unsigned long long* __restrict__ pref, long long* __restrict__ rank) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= k * d) return;
  const long long m = cnt_global[t / d];
  pref[2 * t] = 0;
  pref[2 * t + 1] = 0;
  rank[2 * t] = m > 0 ? (m - 1) / 2 : 0;
  rank[2 * t + 1] = m > 0 ? m / 2 : 0;
}

static int grid_cap(int64_t work, int threads, int cap) {
  int64_t g = (work + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

void medians_segmented(Ctx& c, const double* values, const int64_t* offsets, int64_t nseg,
                       double* out) {
  if (nseg < 0) CDR_FAIL(CDR_ERR_ARG, "n_segments < 0");
  if (nseg == 0) return;
  const int64_t total = offsets[nseg] - offsets[0];
  if (total < 0) CDR_FAIL(CDR_ERR_ARG, "offsets must be non-decreasing");
  for (int64_t s = 0; s < nseg; ++s)
    if (offsets[s + 1] < offsets[s]) CDR_FAIL(CDR_ERR_ARG, "offsets must be non-decreasing");
  c.med_vals.ensure(sizeof(double) * (total > 0 ? total : 1));
  c.med_off.ensure(sizeof(int64_t) * (nseg + 1));
  c.med_out.ensure(sizeof(double) * nseg);
  std::vector<int64_t> off0(nseg + 1);
  for (int64_t s = 0; s <= nseg; ++s) off0[s] = offsets[s] - offsets[0];
  if (total > 0)
    HIP_CHECK(hipMemcpyAsync(c.med_vals.p, values + offsets[0], sizeof(double) * total,
                             hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipMemcpyAsync(c.med_off.p, off0.data(), sizeof(int64_t) * (nseg + 1),
                           hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(seg_median_kernel<double>, dim3(grid_cap(nseg, 1, 65536)), dim3(256), 0,
                     c.stream, c.med_vals.as<double>(), c.med_off.as<int64_t>(), nseg,
                     c.med_out.as<double>());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(out, c.med_out.p, sizeof(double) * nseg, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
}

// ---- host side of the label medians (single shard or one rank of several) --
static int mg_passes(const Ctx& c) { return c.mode == CDR_MODE_F32X ? 4 : 8; }

void medians_group(Ctx& c, int32_t k, int64_t* counts) {
  if (!c.have_labels) CDR_FAIL(CDR_ERR_STATE, "no Lloyd labels: run cdr_lloyd_step first");
  if (k < 1 || k < c.last_k) CDR_FAIL(CDR_ERR_ARG, "k smaller than the labels' k");
  if (k > kMgMaxK) CDR_FAIL(CDR_ERR_UNSUPPORTED, "medians: k > 8192");
  const int d = c.d;
  const int64_t n = c.n;
  if (n >= (1ll << 32)) CDR_FAIL(CDR_ERR_UNSUPPORTED, "medians: 2^32 points or more per shard");
  const bool f32 = c.mode == CDR_MODE_F32X;
  const size_t vsz = f32 ? 4 : 8;
  const int64_t nblk = std::max<int64_t>(1, ceil_div(n, kMgBlock));
  const int64_t nr = ceil_div(nblk, kMgRange);
  c.med_tmp.ensure(sizeof(unsigned) * (size_t)nblk * k);
  c.med_tmp2.ensure(sizeof(unsigned long long) * (size_t)nr * k);
  c.med_off.ensure(sizeof(long long) * 2 * (size_t)k);
  unsigned* cnt = c.med_tmp.as<unsigned>();
  long long* base = c.med_off.as<long long>();
  long long* total = base + k;
  const size_t lds = sizeof(unsigned) * k;
  hipLaunchKernelGGL(mg_count, dim3(nblk), dim3(256), lds, c.stream, c.labels.as<int32_t>(), n,
                     k, cnt);
  hipLaunchKernelGGL(mg_scan_a, dim3(nr), dim3(256), 0, c.stream, cnt, nblk, k,
                     c.med_tmp2.as<unsigned long long>());
  hipLaunchKernelGGL(mg_scan_b, dim3(1), dim3(1024), 0, c.stream,
                     c.med_tmp2.as<unsigned long long>(), nr, k, base, total);
  hipLaunchKernelGGL(mg_scan_c, dim3(nr), dim3(256), 0, c.stream, cnt, nblk, k,
                     c.med_tmp2.as<unsigned long long>(), base);
  HIP_CHECK(hipGetLastError());
  c.med_vals.ensure(vsz * (size_t)d * (n > 0 ? n : 1));
  if (n > 0) {
    if (f32)
      hipLaunchKernelGGL(mg_scatter<float>, dim3(nblk), dim3(256), lds, c.stream,
                         c.x32.as<float>(), n, c.n_pad, d, c.labels.as<int32_t>(), k, cnt,
                         c.med_vals.as<float>());
    else
      hipLaunchKernelGGL(mg_scatter<double>, dim3(nblk), dim3(256), lds, c.stream,
                         c.x64.as<double>(), n, c.n_pad, d, c.labels.as<int32_t>(), k, cnt,
                         c.med_vals.as<double>());
    HIP_CHECK(hipGetLastError());
  }
  HIP_CHECK(hipMemcpyAsync(counts, total, sizeof(long long) * k, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.med_k = k;
}

int medians_begin(Ctx& c, const int64_t* global_counts) {
  const int k = c.med_k, d = c.d;
  if (k <= 0) CDR_FAIL(CDR_ERR_STATE, "medians: group the rows first (cdr_medians_group)");
  for (int j = 0; j < k; ++j)
    if (global_counts[j] >= (1ll << 32))
      CDR_FAIL(CDR_ERR_UNSUPPORTED, "medians: a cluster of 2^32 points or more");
  const size_t kd = (size_t)k * d;
  c.med_out.ensure(sizeof(long long) * k + sizeof(unsigned long long) * 2 * kd +
                   sizeof(long long) * 2 * kd + sizeof(double) * kd);
  long long* gcnt = c.med_out.as<long long>();
  unsigned long long* pref = reinterpret_cast<unsigned long long*>(gcnt + k);
  long long* rank = reinterpret_cast<long long*>(pref + 2 * kd);
  HIP_CHECK(hipMemcpyAsync(gcnt, global_counts, sizeof(long long) * k, hipMemcpyHostToDevice,
                           c.stream));
  hipLaunchKernelGGL(mg_begin, dim3(ceil_div((int64_t)kd, 256)), dim3(256), 0, c.stream, gcnt, d,
                     k, pref, rank);
  HIP_CHECK(hipGetLastError());
  c.med_hist.ensure(sizeof(unsigned) * 512 * kd);
  return mg_passes(c);
}

// hist: where the pass's histograms go ([k][d][2][256] u32; host or device
// memory; nullptr = leave them in the context for the select step)
void medians_pass_hist(Ctx& c, int pass, void* hist) {
  const int k = c.med_k, d = c.d, P = mg_passes(c);
  if (pass < 0 || pass >= P) CDR_FAIL(CDR_ERR_ARG, "medians: pass out of range");
  const size_t kd = (size_t)k * d;
  long long* gcnt = c.med_out.as<long long>();
  unsigned long long* pref = reinterpret_cast<unsigned long long*>(gcnt + k);
  const int sh = (P - 1 - pass) * 8;
  const long long* base = c.med_off.as<long long>();
  const long long* total = base + k;
  dim3 grid(k, (unsigned)ceil_div(d, kMgFeat));
  if (c.mode == CDR_MODE_F32X)
    hipLaunchKernelGGL(mg_hist<float>, grid, dim3(1024), 0, c.stream, c.med_vals.as<float>(), d, k,
                       base, total, pref, sh, c.med_hist.as<unsigned>());
  else
    hipLaunchKernelGGL(mg_hist<double>, grid, dim3(1024), 0, c.stream, c.med_vals.as<double>(), d,
                       k, base, total, pref, sh, c.med_hist.as<unsigned>());
  HIP_CHECK(hipGetLastError());
  if (hist) {
    HIP_CHECK(hipMemcpyAsync(hist, c.med_hist.p, sizeof(unsigned) * 512 * kd, hipMemcpyDefault,
                             c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
  }
}

void medians_pass_select(Ctx& c, int pass, const void* hist) {
  const int k = c.med_k, d = c.d, P = mg_passes(c);
  if (pass < 0 || pass >= P) CDR_FAIL(CDR_ERR_ARG, "medians: pass out of range");
  const size_t kd = (size_t)k * d;
  long long* gcnt = c.med_out.as<long long>();
  unsigned long long* pref = reinterpret_cast<unsigned long long*>(gcnt + k);
  long long* rank = reinterpret_cast<long long*>(pref + 2 * kd);
  if (hist)
    HIP_CHECK(hipMemcpyAsync(c.med_hist.p, hist, sizeof(unsigned) * 512 * kd, hipMemcpyDefault,
                             c.stream));
  const int sh = (P - 1 - pass) * 8;
  if (c.mode == CDR_MODE_F32X)
    hipLaunchKernelGGL(mg_select<float>, dim3(ceil_div((int64_t)kd, 256)), dim3(256), 0, c.stream,
                       c.med_hist.as<unsigned>(), d, k, gcnt, sh, pref, rank);
  else
    hipLaunchKernelGGL(mg_select<double>, dim3(ceil_div((int64_t)kd, 256)), dim3(256), 0,
                       c.stream, c.med_hist.as<unsigned>(), d, k, gcnt, sh, pref, rank);
  HIP_CHECK(hipGetLastError());
}

void medians_finish(Ctx& c, double* out) {
  const int k = c.med_k, d = c.d;
  const size_t kd = (size_t)k * d;
  long long* gcnt = c.med_out.as<long long>();
  unsigned long long* pref = reinterpret_cast<unsigned long long*>(gcnt + k);
  double* res = reinterpret_cast<double*>(reinterpret_cast<long long*>(pref + 2 * kd) + 2 * kd);
  if (c.mode == CDR_MODE_F32X)
    hipLaunchKernelGGL(mg_finish<float>, dim3(ceil_div((int64_t)kd, 256)), dim3(256), 0, c.stream,
                       gcnt, d, k, pref, res);
  else
    hipLaunchKernelGGL(mg_finish<double>, dim3(ceil_div((int64_t)kd, 256)), dim3(256), 0,
                       c.stream, gcnt, d, k, pref, res);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(out, res, sizeof(double) * kd, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
}

void medians_by_label(Ctx& c, int32_t k, double* out) {
  std::vector<int64_t> counts(k);
  medians_group(c, k, counts.data());
  const int P = medians_begin(c, counts.data());
  for (int p = 0; p < P; ++p) {
    medians_pass_hist(c, p, nullptr);
    medians_pass_select(c, p, nullptr);
  }
  medians_finish(c, out);
}

}  // namespace cdr

using namespace cdr;

extern "C" {

int cdr_medians_segmented(cdr_ctx* h, const double* values, const int64_t* offsets,
                          int64_t n_segments, double* out) {
  CDR_TRY
  if (!h || !offsets || (n_segments > 0 && !out)) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  medians_segmented(h->c, values, offsets, n_segments, out);
  CDR_CATCH
}

int cdr_medians_group(cdr_ctx* h, int32_t k, int64_t* counts) {
  CDR_TRY
  if (!h || !counts) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  medians_group(h->c, k, counts);
  CDR_CATCH
}

int cdr_medians_begin(cdr_ctx* h, const int64_t* global_counts, int32_t* passes,
                      int64_t* hist_words) {
  CDR_TRY
  if (!h || !global_counts || !passes || !hist_words) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  *passes = medians_begin(h->c, global_counts);
  *hist_words = (int64_t)h->c.med_k * h->c.d * 512;
  CDR_CATCH
}

int cdr_medians_pass_hist(cdr_ctx* h, int32_t pass, void* hist) {
  CDR_TRY
  if (!h || !hist) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  medians_pass_hist(h->c, pass, hist);
  CDR_CATCH
}

int cdr_medians_pass_select(cdr_ctx* h, int32_t pass, const void* hist) {
  CDR_TRY
  if (!h || !hist) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  medians_pass_select(h->c, pass, hist);
  CDR_CATCH
}

int cdr_medians_finish(cdr_ctx* h, double* out) {
  CDR_TRY
  if (!h || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  medians_finish(h->c, out);
  CDR_CATCH
}

int cdr_medians_by_label(cdr_ctx* h, int32_t k, double* out) {
  CDR_TRY
  if (!h || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  medians_by_label(h->c, k, out);
  CDR_CATCH
}

}  // extern "C"
