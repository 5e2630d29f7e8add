// exchange.hip — the access-log events of one rank sent to the ranks that own
// their files (feature aggregation over several GPUs).
//
// The reference aggregates one log in one Spark job (src/compute_features.py:
// 31-46).  Sharded, every rank ingests a slice of the log (any events) and
// owns a contiguous range of manifest rows [bounds[r], bounds[r+1]); one
// all-to-all (RCCL on the GPU path) brings each file's events to its owner,
// whose group-by then sees every event of its files and computes exactly the
// single-process counters.  Events of paths outside the manifest are not sent
// (they only enter max(ts_epoch), :48, which the pack returns for the MAX
// all-reduce).
//
// Record (16 bytes): ts int64 | file int32 (global row) | client << 8 | op
// (client as a signed 24-bit value).
#include <algorithm>

#include "cdr_internal.h"

namespace cdr {

namespace {

constexpr int kXMaxRanks = 1024;
constexpr long long kTsNullX = LLONG_MIN;

struct XRec {
  long long ts;
  int32_t file;
  int32_t cop;
};

__device__ __forceinline__ int owner_of(const long long* b, int nr, long long f) {
  int lo = 0, hi = nr;  // b[lo] <= f < b[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (b[mid] <= f) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Pass 1: per-rank record counts (LDS histogram, one global add per rank and
// workgroup) and the non-null timestamp maximum over every event.
__global__ __launch_bounds__(256) void x_count(const int32_t* __restrict__ file,
                                               const long long* __restrict__ ts, int64_t ne,
                                               const long long* __restrict__ bounds, int nr,
                                               unsigned long long* __restrict__ cnt,
                                               unsigned long long* __restrict__ mx) {
  __shared__ long long b[kXMaxRanks + 1];
  __shared__ unsigned h[kXMaxRanks];
  __shared__ long long red[4];
  for (int i = threadIdx.x; i <= nr; i += 256) b[i] = bounds[i];
  for (int i = threadIdx.x; i < nr; i += 256) h[i] = 0;
  __syncthreads();
  long long hi = LLONG_MIN;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < ne;
       e += (int64_t)gridDim.x * 256) {
    const long long t = ts[e];
    if (t != kTsNullX) hi = max(hi, t);
    const long long f = file[e];
    if (f >= b[0] && f < b[nr]) atomicAdd(&h[owner_of(b, nr, f)], 1u);
  }
  for (int o = 32; o > 0; o >>= 1) hi = max(hi, __shfl_xor(hi, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = hi;
  __syncthreads();
  for (int i = threadIdx.x; i < nr; i += 256)
    if (h[i]) atomicAdd(&cnt[i], (unsigned long long)h[i]);
  if (threadIdx.x == 0) {
    hi = max(max(red[0], red[1]), max(red[2], red[3]));
    if (hi != LLONG_MIN) atomicMax(mx, (unsigned long long)(hi ^ LLONG_MIN));
  }
}

// Pass 2: records into the per-rank regions (order inside a region is free:
// the owner's group-by is order-independent).
__global__ __launch_bounds__(256) void x_pack(const int32_t* __restrict__ file,
                                              const uint8_t* __restrict__ op,
                                              const int32_t* __restrict__ client,
                                              const long long* __restrict__ ts, int64_t ne,
                                              const long long* __restrict__ bounds, int nr,
                                              unsigned long long* __restrict__ cursor,
                                              XRec* __restrict__ out) {
  __shared__ long long b[kXMaxRanks + 1];
  __shared__ unsigned h[kXMaxRanks];
  __shared__ unsigned long long base[kXMaxRanks];
  for (int i = threadIdx.x; i <= nr; i += 256) b[i] = bounds[i];
  for (int64_t e0 = (int64_t)blockIdx.x * 256; e0 < ne; e0 += (int64_t)gridDim.x * 256) {
    for (int i = threadIdx.x; i < nr; i += 256) h[i] = 0;
    __syncthreads();
    const int64_t e = e0 + threadIdx.x;
    int r = -1;
    unsigned rk = 0;
    if (e < ne) {
      const long long f = file[e];
      if (f >= b[0] && f < b[nr]) {
        r = owner_of(b, nr, f);
        rk = atomicAdd(&h[r], 1u);
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nr; i += 256)
      base[i] = h[i] ? atomicAdd(&cursor[i], (unsigned long long)h[i]) : 0ull;
    __syncthreads();
    if (r >= 0) {
      XRec x;
      x.ts = ts[e];
      x.file = file[e];
      x.cop = (int32_t)(((unsigned)client[e] << 8) | op[e]);
      out[base[r] + rk] = x;
    }
    __syncthreads();
  }
}

// Also the largest client id received (*cmax, zeroed by the caller): the
// group-by sizes its packed client field from it, and records from a rank
// whose slice went through the host tokeniser may carry ids no local ingest saw.
__global__ __launch_bounds__(256) void x_unpack(const XRec* __restrict__ in, int64_t n,
                                                long long file_begin, int32_t* __restrict__ file,
                                                uint8_t* __restrict__ op,
                                                int32_t* __restrict__ client,
                                                long long* __restrict__ ts, int* __restrict__ cmax) {
  int hi = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const XRec x = in[i];
    ts[i] = x.ts;
    file[i] = (int32_t)(x.file - file_begin);
    op[i] = (uint8_t)(x.cop & 0xFF);
    const int cl = x.cop >> 8;  // arithmetic shift: the signed 24-bit client
    client[i] = cl;
    hi = max(hi, cl);
  }
  for (int o = 32; o > 0; o >>= 1) hi = max(hi, __shfl_xor(hi, o));
  if ((threadIdx.x & 63) == 0 && hi > 0) atomicMax(cmax, hi);
}

int xgrid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 256), 4096)); }

}  // namespace

}  // namespace cdr

using namespace cdr;

extern "C" {

int cdr_features_exchange_pack(cdr_ctx* h, int32_t nranks, const int64_t* bounds, void* send,
                               int64_t* counts, int64_t* max_ts_us) {
  CDR_TRY
  if (!h || !bounds || !counts || !max_ts_us) CDR_FAIL(CDR_ERR_ARG, "null argument");
  if (nranks < 1 || nranks > kXMaxRanks) CDR_FAIL(CDR_ERR_ARG, "exchange: 1..1024 ranks");
  for (int r = 0; r < nranks; ++r)
    if (bounds[r] > bounds[r + 1] || bounds[r] < 0)
      CDR_FAIL(CDR_ERR_ARG, "exchange: bounds must be non-decreasing and >= 0");
  Ctx& c = h->c;
  if (c.ev_nf <= 0 && c.ev_n > 0) CDR_FAIL(CDR_ERR_STATE, "exchange: no resident events");
  if (bounds[nranks] > c.ev_nf) CDR_FAIL(CDR_ERR_ARG, "exchange: bounds beyond the manifest");
  HIP_CHECK(hipSetDevice(c.device));
  const int64_t ne = c.ev_n;
  c.x_small.ensure(8 * (2 * (size_t)nranks + 2) + 8 * ((size_t)nranks + 1));
  long long* dbounds = c.x_small.as<long long>();
  unsigned long long* cnt = reinterpret_cast<unsigned long long*>(dbounds + nranks + 1);
  unsigned long long* cur = cnt + nranks;
  unsigned long long* mx = cur + nranks;
  HIP_CHECK(hipMemcpyAsync(dbounds, bounds, 8 * (nranks + 1), hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipMemsetAsync(cnt, 0, 8 * (2 * (size_t)nranks + 1), c.stream));
  if (ne > 0)
    hipLaunchKernelGGL(x_count, dim3(xgrid(ne)), dim3(256), 0, c.stream, c.ev_file.as<int32_t>(),
                       c.ev_ts.as<long long>(), ne, dbounds, nranks, cnt, mx);
  HIP_CHECK(hipGetLastError());
  std::vector<unsigned long long> hc(nranks + 1);
  HIP_CHECK(hipMemcpyAsync(hc.data(), cnt, 8 * nranks, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(&hc[nranks], mx, 8, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  std::vector<unsigned long long> off(nranks, 0);
  unsigned long long tot = 0;
  for (int r = 0; r < nranks; ++r) {
    off[r] = tot;
    tot += hc[r];
    counts[r] = (int64_t)hc[r];
  }
  *max_ts_us = hc[nranks] == 0 ? LLONG_MIN : (int64_t)(hc[nranks] ^ (unsigned long long)LLONG_MIN);
  if (tot > 0) {
    if (!send) CDR_FAIL(CDR_ERR_ARG, "exchange: null send buffer");
    HIP_CHECK(hipMemcpyAsync(cur, off.data(), 8 * nranks, hipMemcpyHostToDevice, c.stream));
    c.x_buf.ensure(sizeof(XRec) * tot);
    hipLaunchKernelGGL(x_pack, dim3(xgrid(ne)), dim3(256), 0, c.stream, c.ev_file.as<int32_t>(),
                       c.ev_op.as<uint8_t>(), c.ev_client.as<int32_t>(),
                       c.ev_ts.as<long long>(), ne, dbounds, nranks, cur, c.x_buf.as<XRec>());
    HIP_CHECK(hipGetLastError());
    // the caller's buffer may be host or device memory (unified addressing)
    HIP_CHECK(hipMemcpyAsync(send, c.x_buf.p, sizeof(XRec) * tot, hipMemcpyDefault, c.stream));
  }
  HIP_CHECK(hipStreamSynchronize(c.stream));
  CDR_CATCH
}

int cdr_features_exchange_unpack(cdr_ctx* h, const void* recv, int64_t n, int64_t file_begin,
                                 int64_t file_end) {
  CDR_TRY
  if (!h || (n > 0 && !recv)) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  if (file_begin < 0 || file_end < file_begin || file_end > c.ev_nf)
    CDR_FAIL(CDR_ERR_ARG, "exchange: file range outside the manifest");
  if (n < 0 || n >= (1ll << 31)) CDR_FAIL(CDR_ERR_ARG, "exchange: 0 <= n < 2^31");
  HIP_CHECK(hipSetDevice(c.device));
  const size_t n1 = n > 0 ? (size_t)n : 1;
  c.x_buf.ensure(sizeof(XRec) * n1);
  if (n > 0)
    HIP_CHECK(hipMemcpyAsync(c.x_buf.p, recv, sizeof(XRec) * n, hipMemcpyDefault, c.stream));
  c.ev_file.ensure(4 * n1);
  c.ev_op.ensure(n1);
  c.ev_client.ensure(4 * n1);
  c.ev_ts.ensure(8 * n1);
  c.x_small.ensure(64);
  int* dcmax = c.x_small.as<int>();
  HIP_CHECK(hipMemsetAsync(dcmax, 0, sizeof(int), c.stream));
  if (n > 0)
    hipLaunchKernelGGL(x_unpack, dim3(xgrid(n)), dim3(256), 0, c.stream, c.x_buf.as<XRec>(), n,
                       (long long)file_begin, c.ev_file.as<int32_t>(), c.ev_op.as<uint8_t>(),
                       c.ev_client.as<int32_t>(), c.ev_ts.as<long long>(), dcmax);
  HIP_CHECK(hipGetLastError());
  int cmax = 0;
  HIP_CHECK(hipMemcpyAsync(&cmax, dcmax, sizeof(int), hipMemcpyDeviceToHost, c.stream));
  // the owned rows' primaries move to the front
  const int64_t nfl = file_end - file_begin;
  if (nfl > 0 && file_begin > 0) {
    c.x_prim.ensure(4 * (size_t)nfl);
    HIP_CHECK(hipMemcpyAsync(c.x_prim.p, c.ev_primary.as<int32_t>() + file_begin, 4 * nfl,
                             hipMemcpyDeviceToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(c.ev_primary.p, c.x_prim.p, 4 * nfl, hipMemcpyDeviceToDevice,
                             c.stream));
  }
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.ev_n = n;
  events_ts_range(c, n);
  c.ev_nf = nfl;
  // the packed client field must hold every received id (and the owned
  // primaries the local manifest gave: keep the wider of the two)
  c.ev_cmax = std::max(c.ev_cmax, cmax);
  CDR_CATCH
}

int cdr_features_load_events(cdr_ctx* h, int64_t n, const int32_t* file, const uint8_t* op,
                             const int32_t* client, const int64_t* ts, int64_t n_files,
                             const int32_t* primary) {
  CDR_TRY
  if (!h || (n > 0 && (!file || !op || !client || !ts)) || (n_files > 0 && !primary))
    CDR_FAIL(CDR_ERR_ARG, "null argument");
  if (n < 0 || n >= (1ll << 31) || n_files < 0 || n_files >= (1ll << 31))
    CDR_FAIL(CDR_ERR_ARG, "load_events: sizes");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  const size_t n1 = n > 0 ? (size_t)n : 1, f1 = n_files > 0 ? (size_t)n_files : 1;
  c.ev_file.ensure(4 * n1);
  c.ev_op.ensure(n1);
  c.ev_client.ensure(4 * n1);
  c.ev_ts.ensure(8 * n1);
  c.ev_primary.ensure(4 * f1);
  c.ev_out.ensure(8 * 6 * f1 + 64);
  if (n > 0) {
    HIP_CHECK(hipMemcpyAsync(c.ev_file.p, file, 4 * n, hipMemcpyHostToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(c.ev_op.p, op, n, hipMemcpyHostToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(c.ev_client.p, client, 4 * n, hipMemcpyHostToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(c.ev_ts.p, ts, 8 * n, hipMemcpyHostToDevice, c.stream));
  }
  if (n_files > 0)
    HIP_CHECK(hipMemcpyAsync(c.ev_primary.p, primary, 4 * n_files, hipMemcpyHostToDevice,
                             c.stream));
  int cmax = 0;
  for (int64_t i = 0; i < n; ++i) cmax = std::max(cmax, (int)client[i]);
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.ev_n = n;
  events_ts_range(c, n);
  c.ev_nf = n_files;
  c.ev_cmax = cmax;
  CDR_CATCH
}

}  // extern "C"
