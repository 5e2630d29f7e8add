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

// Group the points of an F32X/F64 shard by label: counts, offsets, scatter.
__global__ void label_hist(const int32_t* __restrict__ labels, int64_t n,
                           unsigned long long* __restrict__ cnt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[labels[i]], 1ull);
}

template <typename V>
__global__ void scatter_by_label(const V* __restrict__ X, int64_t n, int64_t n_pad, int d,
                                 const int32_t* __restrict__ labels, int k,
                                 unsigned long long* __restrict__ cursor,
                                 const int64_t* __restrict__ seg_off, V* __restrict__ dst) {
  // dst layout: feature-major segments: segment (f, j) = dst[f * n + off[j] ..]
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int j = labels[i];
    const unsigned long long pos = atomicAdd(&cursor[j], 1ull);
    for (int f = 0; f < d; ++f) dst[(int64_t)f * n + seg_off[j] + (int64_t)pos] = X[xidx(f, i, n_pad)];
  }
}

__global__ void make_feature_offsets(const int64_t* __restrict__ seg_off, int k, int d, int64_t n,
                                     int64_t* __restrict__ off2) {
  // segment order (j, f) -> out index j*d + f; values live at f*n + seg_off[j]
  // we emit offsets per (f, j) in f-major order: off2[f*k + j] .. + count
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t > k * d) return;
  if (t == k * d) {
    off2[t] = (int64_t)d * n;
    return;
  }
  const int f = t / k, j = t % k;
  off2[t] = (int64_t)f * n + seg_off[j];
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

void medians_by_label(Ctx& c, int32_t k, double* out) {
  if (!c.have_labels) CDR_FAIL(CDR_ERR_STATE, "no Lloyd labels: run cdr_lloyd_step first");
  if (k < 1 || k < c.last_k) CDR_FAIL(CDR_ERR_ARG, "k smaller than the labels' k");
  const int d = c.d;
  const int64_t n = c.n;
  const bool f32 = c.mode == CDR_MODE_F32X;
  const size_t vsz = f32 ? 4 : 8;
  c.med_tmp.ensure(sizeof(unsigned long long) * k * 2);
  unsigned long long* cnt = c.med_tmp.as<unsigned long long>();
  HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(unsigned long long) * k * 2, c.stream));
  hipLaunchKernelGGL(label_hist, dim3(grid_cap(n, 256, 4096)), dim3(256), 0, c.stream,
                     c.labels.as<int32_t>(), n, cnt);
  HIP_CHECK(hipGetLastError());
  std::vector<unsigned long long> hc(k);
  HIP_CHECK(hipMemcpyAsync(hc.data(), cnt, sizeof(unsigned long long) * k,
                           hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  std::vector<int64_t> seg(k + 1, 0);
  for (int j = 0; j < k; ++j) seg[j + 1] = seg[j] + (int64_t)hc[j];
  c.med_off.ensure(sizeof(int64_t) * ((size_t)k * d + 1 + k + 1));
  int64_t* dseg = c.med_off.as<int64_t>() + (size_t)k * d + 1;
  HIP_CHECK(hipMemcpyAsync(dseg, seg.data(), sizeof(int64_t) * (k + 1), hipMemcpyHostToDevice,
                           c.stream));
  c.med_vals.ensure(vsz * (size_t)d * (n > 0 ? n : 1));
  unsigned long long* cursor = cnt + k;
  if (n > 0) {
    if (f32)
      hipLaunchKernelGGL(scatter_by_label<float>, dim3(grid_cap(n, 256, 4096)), dim3(256), 0,
                         c.stream, c.x32.as<float>(), n, c.n_pad, d, c.labels.as<int32_t>(), k,
                         cursor, dseg, c.med_vals.as<float>());
    else
      hipLaunchKernelGGL(scatter_by_label<double>, dim3(grid_cap(n, 256, 4096)), dim3(256), 0,
                         c.stream, c.x64.as<double>(), n, c.n_pad, d, c.labels.as<int32_t>(),
                         k, cursor, dseg, c.med_vals.as<double>());
    HIP_CHECK(hipGetLastError());
  }
  int64_t* off2 = c.med_off.as<int64_t>();
  hipLaunchKernelGGL(make_feature_offsets, dim3((k * d + 256) / 256), dim3(256), 0, c.stream,
                     dseg, k, d, n, off2);
  HIP_CHECK(hipGetLastError());
  // (f, j) segments are contiguous in f-major order; compute them all.
  const int64_t nseg = (int64_t)k * d;
  c.med_out.ensure(sizeof(double) * nseg);
  if (f32)
    hipLaunchKernelGGL(seg_median_kernel<float>, dim3(grid_cap(nseg, 1, 65536)), dim3(256), 0,
                       c.stream, c.med_vals.as<float>(), off2, nseg, c.med_out.as<double>());
  else
    hipLaunchKernelGGL(seg_median_kernel<double>, dim3(grid_cap(nseg, 1, 65536)), dim3(256), 0,
                       c.stream, c.med_vals.as<double>(), off2, nseg, c.med_out.as<double>());
  HIP_CHECK(hipGetLastError());
  std::vector<double> fm(nseg);
  HIP_CHECK(hipMemcpyAsync(fm.data(), c.med_out.p, sizeof(double) * nseg, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  for (int j = 0; j < k; ++j)
    for (int f = 0; f < d; ++f) out[(size_t)j * d + f] = fm[(size_t)f * k + j];
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

int cdr_medians_by_label(cdr_ctx* h, int32_t k, double* out) {
  CDR_TRY
  if (!h || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  medians_by_label(h->c, k, out);
  CDR_CATCH
}

}  // extern "C"
