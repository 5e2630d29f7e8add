// simulate.hip — the access simulator (src/access_simulator.py) on the device,
// for the config-4 scale runs: a resident, time-ordered event log whose
// per-file statistics follow the reference's generator.
//
// Per file (global id g = file_begin + f; counter-based random numbers keyed
// by (seed, g, event, stream), so any shard regenerates its own files):
//   category hot / shared / moderate / archival with weights .10/.20/.50/.20
//     (src/generator.py:45), primary node uniform over the clients (:44);
//   read_rate  = max(0, N(r, max(1e-4, 0.2 r)))         access_simulator.py:55
//   write_rate = max(0, N(w, max(1e-4, 0.5 w)))         :56
//   locality   = clamp(N(b, 0.2), 0, 1)                 :57
//   (r, w, b) from the category table                    :42-47
//   arrivals: t += Exp(read + write) while t < duration  :19-29
//   op READ with p = read / (read + write + 1e-12)       :30-31
//   client = primary with p = locality, else uniform     :33-36
//   ts = sim_start + t, written with milliseconds        :5-6, :38
//     -> microseconds = floor((t0_us + rint(t 1e6)) / 1000) * 1000
// then the log is sorted by timestamp (:60) with a counting sort over the
// milliseconds (events of one millisecond in no particular order).
#include <algorithm>
#include <cmath>

#include "cdr_internal.h"

namespace cdr {

namespace {

__device__ __forceinline__ unsigned long long smix(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// uniform in (0, 1]
__device__ __forceinline__ double sim_u(unsigned long long seed, long long g, long long j,
                                        unsigned stream) {
  const unsigned long long h =
      smix(seed ^ smix((unsigned long long)g * 0xD1B54A32D192ED03ull ^
                       ((unsigned long long)j << 8) ^ stream));
  return (double)((h >> 11) + 1) * 0x1.0p-53;
}

__device__ __forceinline__ double sim_gauss(unsigned long long seed, long long g, unsigned s) {
  const double u1 = sim_u(seed, g, -1, s), u2 = sim_u(seed, g, -1, s + 1);
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

struct FileRates {
  double lam, p_read, loc;
  int primary;
};

__device__ FileRates sim_rates(unsigned long long seed, long long g, int n_clients) {
  // hot, shared, moderate, archival (access_simulator.py:42-47)
  const double R[4] = {0.8, 0.6, 0.1, 0.005};
  const double W[4] = {0.2, 0.02, 0.01, 0.001};
  const double B[4] = {0.7, 0.3, 0.5, 0.9};
  const double uc = sim_u(seed, g, -1, 1);
  const int cat = uc <= 0.10 ? 0 : (uc <= 0.30 ? 1 : (uc <= 0.80 ? 2 : 3));
  const double r = fmax(0.0, R[cat] + fmax(1e-4, R[cat] * 0.2) * sim_gauss(seed, g, 2));
  const double w = fmax(0.0, W[cat] + fmax(1e-4, W[cat] * 0.5) * sim_gauss(seed, g, 4));
  const double b = fmin(1.0, fmax(0.0, B[cat] + 0.2 * sim_gauss(seed, g, 6)));
  FileRates fr;
  fr.lam = fmax(0.0, r + w);
  fr.p_read = r / (fr.lam + 1e-12);
  fr.loc = b;
  fr.primary = min(n_clients - 1, (int)(sim_u(seed, g, -1, 8) * n_clients));
  return fr;
}

__global__ void sim_count(int64_t nf, int64_t file_begin, double duration, int n_clients,
                          unsigned long long seed, long long* __restrict__ cnt,
                          int32_t* __restrict__ primary) {
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < nf;
       f += (int64_t)gridDim.x * blockDim.x) {
    const long long g = file_begin + f;
    const FileRates fr = sim_rates(seed, g, n_clients);
    long long n = 0;
    if (fr.lam > 0) {
      double t = 0.0;
      while (true) {
        t += -log(sim_u(seed, g, n, 9)) / fr.lam;
        if (t >= duration) break;
        ++n;
      }
    }
    cnt[f] = n;
    primary[f] = fr.primary;
  }
}

__global__ void sim_emit(int64_t nf, int64_t file_begin, double duration, int n_clients,
                         unsigned long long seed, long long t0_us, long long t0_ms,
                         const long long* __restrict__ off, long long* __restrict__ ts,
                         int32_t* __restrict__ file, uint8_t* __restrict__ op,
                         int32_t* __restrict__ client, unsigned* __restrict__ mhist) {
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < nf;
       f += (int64_t)gridDim.x * blockDim.x) {
    const long long g = file_begin + f;
    const FileRates fr = sim_rates(seed, g, n_clients);
    const long long o = off[f], n = off[f + 1] - o;
    double t = 0.0;
    for (long long j = 0; j < n; ++j) {
      t += -log(sim_u(seed, g, j, 9)) / fr.lam;
      const long long us = t0_us + (long long)rint(t * 1e6);
      const long long ms = us >= 0 ? us / 1000 : -((-us + 999) / 1000);
      ts[o + j] = ms * 1000;
      file[o + j] = (int32_t)f;
      op[o + j] = sim_u(seed, g, j, 10) < fr.p_read ? 2 : 1;
      client[o + j] = sim_u(seed, g, j, 11) < fr.loc
                          ? fr.primary
                          : min(n_clients - 1, (int)(sim_u(seed, g, j, 12) * n_clients));
      atomicAdd(&mhist[ms - t0_ms], 1u);
    }
  }
}

__global__ void sim_place(int64_t ne, long long t0_ms, const long long* __restrict__ ts_in,
                          const int32_t* __restrict__ f_in, const uint8_t* __restrict__ op_in,
                          const int32_t* __restrict__ cl_in, const long long* __restrict__ mbase,
                          unsigned* __restrict__ mcur, long long* __restrict__ ts,
                          int32_t* __restrict__ file, uint8_t* __restrict__ op,
                          int32_t* __restrict__ client) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne;
       i += (int64_t)gridDim.x * blockDim.x) {
    const long long m = ts_in[i] / 1000 - t0_ms;
    const long long pos = mbase[m] + atomicAdd(&mcur[m], 1u);
    ts[pos] = ts_in[i];
    file[pos] = f_in[i];
    op[pos] = op_in[i];
    client[pos] = cl_in[i];
  }
}

// Exclusive scan of n int64 (or uint32 when U32) counts into out[0..n]
// (out[n] = total), three passes: 1024-element block sums, one workgroup over
// the block sums, block-local scans plus the block base.
constexpr int kScanBlock = 1024;

template <typename T>
__global__ __launch_bounds__(256) void scan_blocks(const T* __restrict__ in, int64_t n,
                                                   long long* __restrict__ bsum) {
  __shared__ long long red[4];
  const int64_t b0 = (int64_t)blockIdx.x * kScanBlock;
  long long s = 0;
  for (int i = threadIdx.x; i < kScanBlock; i += 256)
    if (b0 + i < n) s += (long long)in[b0 + i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(1024) void scan_sums(long long* __restrict__ bsum, int64_t nb) {
  __shared__ long long wsum[16];
  __shared__ long long carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < nb; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const long long v = i < nb ? bsum[i] : 0;
    long long inc = v;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
      const long long u = __shfl_up(inc, o);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    long long pre = carry;
    for (int k = 0; k < w; ++k) pre += wsum[k];
    if (i < nb) bsum[i] = pre + inc - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = pre + inc;
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[nb] = carry;
}

template <typename T>
__global__ __launch_bounds__(256) void scan_apply(const T* __restrict__ in, int64_t n,
                                                  const long long* __restrict__ bsum,
                                                  long long* __restrict__ out) {
  __shared__ long long wsum[4];
  const int64_t b0 = (int64_t)blockIdx.x * kScanBlock;
  // 4 consecutive elements per thread
  long long v[4], s = 0;
  for (int k = 0; k < 4; ++k) {
    const int64_t i = b0 + threadIdx.x * 4 + k;
    v[k] = i < n ? (long long)in[i] : 0;
    s += v[k];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  long long inc = s;
  for (int o = 1; o < 64; o <<= 1) {
    const long long u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  long long pre = bsum[blockIdx.x];
  for (int k = 0; k < w; ++k) pre += wsum[k];
  pre += inc - s;
  for (int k = 0; k < 4; ++k) {
    const int64_t i = b0 + threadIdx.x * 4 + k;
    if (i < n) out[i] = pre;
    pre += v[k];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = bsum[gridDim.x];
}

template <typename T>
void scan_exclusive(Ctx& c, const T* in, int64_t n, long long* out, DevBuf& tmp) {
  const int64_t nb = std::max<int64_t>(1, ceil_div(n, kScanBlock));
  tmp.ensure(sizeof(long long) * (nb + 1));
  hipLaunchKernelGGL(scan_blocks<T>, dim3(nb), dim3(256), 0, c.stream, in, n,
                     tmp.as<long long>());
  hipLaunchKernelGGL(scan_sums, dim3(1), dim3(1024), 0, c.stream, tmp.as<long long>(), nb);
  hipLaunchKernelGGL(scan_apply<T>, dim3(nb), dim3(256), 0, c.stream, in, n,
                     tmp.as<long long>(), out);
  HIP_CHECK(hipGetLastError());
}

}  // namespace

int64_t features_simulate(Ctx& c, int64_t nf, int64_t file_begin, double duration_s,
                          int n_clients, unsigned long long seed, long long t0_us) {
  if (nf < 1 || nf >= (1ll << 31)) CDR_FAIL(CDR_ERR_ARG, "simulate: need 1 <= n_files < 2^31");
  if (!(duration_s > 0) || duration_s > 1e7) CDR_FAIL(CDR_ERR_ARG, "simulate: duration");
  if (n_clients < 1) CDR_FAIL(CDR_ERR_ARG, "simulate: n_clients >= 1");
  // per-file counts and primaries
  DevBuf& cnt = c.sim_cnt;
  cnt.ensure(sizeof(long long) * (nf + 1));
  c.ev_primary.ensure(4 * (size_t)nf);
  hipLaunchKernelGGL(sim_count, dim3(std::min<int64_t>(ceil_div(nf, 256), 8192)), dim3(256), 0,
                     c.stream, nf, file_begin, duration_s, n_clients, seed,
                     cnt.as<long long>(), c.ev_primary.as<int32_t>());
  HIP_CHECK(hipGetLastError());
  c.sim_off.ensure(sizeof(long long) * (nf + 1));
  scan_exclusive<long long>(c, cnt.as<long long>(), nf, c.sim_off.as<long long>(), c.sim_tmp);
  long long ne = 0;
  HIP_CHECK(hipMemcpyAsync(&ne, c.sim_off.as<long long>() + nf, 8, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  if (ne >= (1ll << 31)) CDR_FAIL(CDR_ERR_UNSUPPORTED, "simulate: 2^31 events or more");
  const size_t ne1 = ne > 0 ? (size_t)ne : 1;
  // file-major events, then the counting sort over milliseconds
  const long long t0_ms = t0_us >= 0 ? t0_us / 1000 : -((-t0_us + 999) / 1000);
  const int64_t M = (int64_t)std::ceil(duration_s * 1000.0) + 2;
  c.ev_scratch.ensure(17 * ne1 + 64);
  long long* ts_t = c.ev_scratch.as<long long>();
  int32_t* f_t = reinterpret_cast<int32_t*>(ts_t + ne1);
  int32_t* cl_t = f_t + ne1;
  uint8_t* op_t = reinterpret_cast<uint8_t*>(cl_t + ne1);
  c.sim_ms.ensure(sizeof(unsigned) * 2 * M);
  unsigned* mh = c.sim_ms.as<unsigned>();
  unsigned* mcur = mh + M;
  HIP_CHECK(hipMemsetAsync(mh, 0, sizeof(unsigned) * 2 * M, c.stream));
  hipLaunchKernelGGL(sim_emit, dim3(std::min<int64_t>(ceil_div(nf, 256), 8192)), dim3(256), 0,
                     c.stream, nf, file_begin, duration_s, n_clients, seed, t0_us, t0_ms,
                     c.sim_off.as<long long>(), ts_t, f_t, op_t, cl_t, mh);
  HIP_CHECK(hipGetLastError());
  c.sim_mbase.ensure(sizeof(long long) * (M + 1));
  scan_exclusive<unsigned>(c, mh, M, c.sim_mbase.as<long long>(), c.sim_tmp);
  c.ev_file.ensure(4 * ne1);
  c.ev_op.ensure(ne1);
  c.ev_client.ensure(4 * ne1);
  c.ev_ts.ensure(8 * ne1);
  c.ev_out.ensure(8 * 6 * (size_t)nf + 64);
  if (ne > 0)
    hipLaunchKernelGGL(sim_place, dim3(std::min<int64_t>(ceil_div(ne, 256), 16384)), dim3(256),
                       0, c.stream, (int64_t)ne, t0_ms, ts_t, f_t, op_t, cl_t,
                       c.sim_mbase.as<long long>(), mcur, c.ev_ts.as<long long>(),
                       c.ev_file.as<int32_t>(), c.ev_op.as<uint8_t>(),
                       c.ev_client.as<int32_t>());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.ev_n = ne;
  events_ts_range(c, ne);
  c.ev_nf = nf;
  c.ev_cmax = n_clients - 1;
  return ne;
}

}  // namespace cdr

using namespace cdr;

extern "C" int cdr_features_simulate(cdr_ctx* h, int64_t n_files, int64_t file_begin,
                                     double duration_s, int32_t n_clients, uint64_t seed,
                                     int64_t t0_us, int64_t* n_events) {
  CDR_TRY
  if (!h || !n_events) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  *n_events = features_simulate(h->c, n_files, file_begin, duration_s, n_clients, seed, t0_us);
  CDR_CATCH
}
