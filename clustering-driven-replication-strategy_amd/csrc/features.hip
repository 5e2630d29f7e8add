// features.hip — per-file access-log features (reference src/compute_features.py).
//
// K5 aggregate (:31-46, :48-51): per manifest file
//   access_freq = count(events)                       :32
//   writes / reads = sum[op == WRITE] / sum[op == READ] :33-34
//   local_accesses = sum[client == primary_node]      :38-41
//   total_accesses = count(events)                    :42
//   max_concurrency = max over sec of count(file, sec), sec = floor(ts_epoch) :44-46
//   max_ts = max(ts_epoch) over the whole log         :48
// Events are keyed (file << 32 | sec - sec_min), radix-sorted (radix.hip, a
// hand-written stable LSD sort; skipped when the input is already grouped by
// file and ordered by second, which is what the per-file Poisson generator
// produces), then each file's run is reduced.
// Integer counts are exact by construction.
//
// K6 finalize (:53-94): age = observation_end - creation_ts_epoch (0 when the
// creation time is null, na.fill at :60), write_ratio = writes / mean(writes)
// (mean 0 -> 1.0), locality = local / total (total 0 -> 1.0), then min-max
// normalisation of the five columns (max == min -> 0.0).  Long columns are
// normalised as double(v - min) / double(max - min), as Spark's `/` does.

#include <algorithm>
#include <cmath>
#include <cstring>

#include "cdr_internal.h"

namespace cdr {

__device__ __forceinline__ long long sec_of(long long ts_us) {
  // Spark: floor(cast(ts as double)) with cast = micros / 1e6 in fp64.  For
  // 0 <= ts < 9e15 the fp64 quotient never rounds across an integer (an
  // integer ts is >= 1e-6 below the next multiple, far above half an ulp),
  // so the integer floor division is the same number and much cheaper.
  if (ts_us >= 0 && ts_us < 9000000000000000ll) return ts_us / 1000000;
  return (long long)floor((double)ts_us / 1000000.0);
}

// Null timestamps (Spark's to_timestamp of an unparseable string, :28): the
// event still counts (:31-42), its second is the null group of its file
// (:44-46: groupBy(path, sec) keeps a null key), and max(ts_epoch) (:48)
// ignores it.
constexpr long long kTsNull = LLONG_MIN;

// Timestamp range (non-null) and order check: per-workgroup partials
// (part[2b], part[2b+1] = min, max), then ts_minmax_fin; one atomic pair per
// workgroup on the same two words serialised (0.3 ms at 125M events).  Any
// null marks the log unordered (the general path groups the nulls).
__global__ __launch_bounds__(256) void ts_minmax(const long long* __restrict__ ts, int64_t n,
                                                 long long* __restrict__ part,
                                                 int* __restrict__ unordered) {
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  int bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const long long t = ts[i];
    if (t == kTsNull) {
      bad = 1;
      continue;
    }
    lo = min(lo, t);
    hi = max(hi, t);
    if (i + 1 < n) bad |= t > ts[i + 1];
  }
  bad = __syncthreads_or(bad);
  if (bad && threadIdx.x == 0 && *(volatile int*)unordered == 0) atomicOr(unordered, 1);
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o));
    hi = max(hi, __shfl_xor(hi, o));
  }
  __shared__ long long red[2][4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = lo;
    red[1][w] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) {
      lo = min(lo, red[0][i]);
      hi = max(hi, red[1][i]);
    }
    part[2 * blockIdx.x] = lo;
    part[2 * blockIdx.x + 1] = hi;
  }
}

__global__ __launch_bounds__(256) void ts_minmax_fin(const long long* __restrict__ part, int nb,
                                                     unsigned long long* __restrict__ mm) {
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  for (int b = threadIdx.x; b < nb; b += 256) {
    lo = min(lo, part[2 * b]);
    hi = max(hi, part[2 * b + 1]);
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o));
    hi = max(hi, __shfl_xor(hi, o));
  }
  __shared__ long long red[2][4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = lo;
    red[1][w] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) {
      lo = min(lo, red[0][i]);
      hi = max(hi, red[1][i]);
    }
    mm[0] = (unsigned long long)(lo ^ LLONG_MIN);
    mm[1] = (unsigned long long)(hi ^ LLONG_MIN);
  }
}

// Null seconds take the all-ones code of sbits (a group of their own, after
// every real second of the file).
__global__ void make_keys(const int32_t* __restrict__ file, const uint8_t* __restrict__ op,
                          const int32_t* __restrict__ client, const long long* __restrict__ ts,
                          int64_t n, int64_t n_files, const int32_t* __restrict__ primary,
                          long long sec_min, int sbits, unsigned long long* __restrict__ keys,
                          uint8_t* __restrict__ flags) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int f = file[i];
    unsigned long long key = ~0ull;
    uint8_t fl = 0;
    if (f >= 0 && f < n_files) {
      const long long t = ts[i];
      const unsigned long long so = t == kTsNull ? (1ull << sbits) - 1
                                                 : (unsigned long long)(sec_of(t) - sec_min);
      key = ((unsigned long long)f << sbits) | so;
      fl = (op[i] == 1 ? 1 : 0) | (op[i] == 2 ? 2 : 0);
      const int pr = primary[f];
      if (client[i] >= 0 && pr >= 0 && client[i] == pr) fl |= 4;
    }
    keys[i] = key;
    flags[i] = fl;
  }
}

// Time-ordered logs (the usual case: an access log is appended in time
// order): a STABLE sort by file alone keeps every file's events in time
// order, so equal seconds stay adjacent.  Key = file (all ones = not in the
// manifest, sorts last within fbits), value = client << 32 | (sec - sec_min)
// << 3 | flags.
__global__ void make_keys32(const int32_t* __restrict__ file, const uint8_t* __restrict__ op,
                            const int32_t* __restrict__ client, const long long* __restrict__ ts,
                            int64_t n, int64_t n_files, const int32_t* __restrict__ primary,
                            long long sec_min, unsigned invalid, unsigned* __restrict__ keys,
                            unsigned long long* __restrict__ vals) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int f = file[i];
    unsigned key = invalid;
    unsigned long long v = 0;
    if (f >= 0 && f < n_files) {
      key = (unsigned)f;
      const unsigned fl = (op[i] == 1 ? 1u : 0u) | (op[i] == 2 ? 2u : 0u);
      // the client rides along (the primary node is looked up once per file
      // after the sort, instead of a random gather per event here)
      v = ((unsigned long long)(unsigned)client[i] << 32) |
          (((unsigned)(sec_of(ts[i]) - sec_min) << 3) | fl);
    }
    keys[i] = key;
    vals[i] = v;
  }
}

__global__ void check_sorted32(const unsigned* __restrict__ keys, int64_t n,
                               int* __restrict__ unsorted) {
  int bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n;
       i += (int64_t)gridDim.x * blockDim.x)
    bad |= keys[i] > keys[i + 1];
  // read before the atomic: on an unsorted log every wave finds a descent,
  // and one atomic per wave on one word serialised (0.38 ms at 20M events)
  if (__any(bad) && (threadIdx.x & 63) == 0 && *(volatile int*)unsorted == 0)
    atomicOr(unsorted, 1);
}

__global__ void mark_runs32(const unsigned* __restrict__ keys, int64_t n, unsigned invalid,
                            long long* __restrict__ start, long long* __restrict__ end) {
  // neighbours by lane shuffles (one load per key instead of three); the
  // loop bound is wave-uniform so every lane takes part in the shuffles
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); base < n;
       base += stride) {
    const int64_t i = base + lane;
    const unsigned f = i < n ? keys[i] : invalid;
    unsigned prev = __shfl(f, (lane + 63) & 63), next = __shfl(f, (lane + 1) & 63);
    if (lane == 0 && i > 0 && i - 1 < n) prev = keys[i - 1];
    if (lane == 63 && i + 1 < n) next = keys[i + 1];
    if (i >= n || f == invalid) continue;
    if (i == 0 || prev != f) start[f] = i;
    if (i == n - 1 || next != f) end[f] = i + 1;
  }
}

// One wave per 64 consecutive files: their events are one contiguous span of
// the sorted values, staged into LDS with coalesced loads (spans over
// kPerFileStage values read global memory), then one lane per file walks its
// run.  Before: a grid-stride thread per file walking global memory (each
// load instruction touching 64 lines; 0.74 ms at 12.5M files).
constexpr int kPerFileStage = 768;  // 6 KiB of values per wave

__device__ __forceinline__ void per_file_run(const unsigned long long* src, long long s,
                                             long long e, int pr, long long* o) {
  long long cnt = 0, w = 0, r = 0, loc = 0, best = 0, run = 0;
  unsigned prev = 0xFFFFFFFFu;
  for (long long i = s; i < e; ++i) {
    const unsigned long long vv = src[i];
    const unsigned v = (unsigned)vv;
    const int cl = (int)(unsigned)(vv >> 32);
    const unsigned sec = v >> 3;
    ++cnt;
    w += v & 1;
    r += (v >> 1) & 1;
    loc += (cl >= 0 && pr >= 0 && cl == pr) ? 1 : 0;
    run = (sec == prev) ? run + 1 : 1;
    prev = sec;
    best = run > best ? run : best;
  }
  o[0] = cnt;
  o[1] = w;
  o[2] = r;
  o[3] = loc;
  o[4] = cnt;
  o[5] = best;
}

__global__ __launch_bounds__(64) void per_file32(const unsigned long long* __restrict__ vals,
                                                 int64_t n_files,
                                                 const int32_t* __restrict__ primary,
                                                 const long long* __restrict__ start,
                                                 const long long* __restrict__ end,
                                                 long long* __restrict__ out) {
  __shared__ unsigned long long stage[kPerFileStage];
  const int64_t f = (int64_t)blockIdx.x * 64 + threadIdx.x;
  long long s = -1, e = -1;
  if (f < n_files) {
    s = start[f];
    if (s >= 0) e = end[f];
  }
  long long lo = s >= 0 ? s : LLONG_MAX, hi = e;
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o));
    hi = max(hi, __shfl_xor(hi, o));
  }
  long long o6[6];
  if (lo != LLONG_MAX && hi - lo <= kPerFileStage) {
    for (long long i = threadIdx.x; i < hi - lo; i += 64) stage[i] = vals[lo + i];
    __syncthreads();
    if (f < n_files) {
      if (s >= 0) per_file_run(stage, s - lo, e - lo, primary[f], o6);
      else per_file_run(stage, 0, 0, 0, o6);
    }
  } else if (f < n_files) {
    if (s >= 0) per_file_run(vals, s, e, primary[f], o6);
    else per_file_run(vals, 0, 0, 0, o6);
  }
  if (f < n_files) {
    long long* o = out + f * 6;
#pragma unroll
    for (int j = 0; j < 6; ++j) o[j] = o6[j];
  }
}

__global__ void check_sorted(const unsigned long long* __restrict__ keys, int64_t n,
                             int* __restrict__ unsorted) {
  int bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n;
       i += (int64_t)gridDim.x * blockDim.x)
    bad |= keys[i] > keys[i + 1];
  // read before the atomic: on an unsorted log every wave finds a descent,
  // and one atomic per wave on one word serialised (0.38 ms at 20M events)
  if (__any(bad) && (threadIdx.x & 63) == 0 && *(volatile int*)unsorted == 0)
    atomicOr(unsorted, 1);
}

__global__ void mark_runs(const unsigned long long* __restrict__ keys, int64_t n, int sbits,
                          long long* __restrict__ start, long long* __restrict__ end) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long k = keys[i];
    if (k == ~0ull) continue;
    const unsigned long long f = k >> sbits;
    if (i == 0 || (keys[i - 1] >> sbits) != f) start[f] = i;
    if (i == n - 1 || keys[i + 1] == ~0ull || (keys[i + 1] >> sbits) != f) end[f] = i + 1;
  }
}

__global__ void per_file(const unsigned long long* __restrict__ keys,
                         const uint8_t* __restrict__ flags, int64_t n_files, int sbits,
                         const long long* __restrict__ start, const long long* __restrict__ end,
                         long long* __restrict__ out) {
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n_files;
       f += (int64_t)gridDim.x * blockDim.x) {
    long long cnt = 0, w = 0, r = 0, loc = 0, best = 0;
    const long long s = start[f];
    if (s >= 0) {
      const long long e = end[f];
      unsigned prev = 0xFFFFFFFFu;
      long long run = 0;
      for (long long i = s; i < e; ++i) {
        const uint8_t fl = flags[i];
        const unsigned sec = (unsigned)(keys[i] & ((1ull << sbits) - 1));
        ++cnt;
        w += fl & 1;
        r += (fl >> 1) & 1;
        loc += (fl >> 2) & 1;
        run = (sec == prev) ? run + 1 : 1;
        prev = sec;
        best = run > best ? run : best;
      }
    }
    long long* o = out + f * 6;
    o[0] = cnt;
    o[1] = w;
    o[2] = r;
    o[3] = loc;
    o[4] = cnt;
    o[5] = best;
  }
}

static int gcap(int64_t work, int threads, int cap) {
  int64_t g = (work + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

static void ensure_events(Ctx& c, int64_t ne, int64_t n_files) {
  const size_t ne1 = ne > 0 ? ne : 1, nf1 = n_files > 0 ? n_files : 1;
  c.ev_file.ensure(4 * ne1);
  c.ev_op.ensure(ne1);
  c.ev_client.ensure(4 * ne1);
  c.ev_ts.ensure(8 * ne1);
  c.ev_primary.ensure(4 * nf1);
  c.ev_out.ensure(8 * 6 * nf1 + 64);
}

void features_aggregate_resident(Ctx& c, int64_t ne, int64_t n_files, int64_t* out,
                                 int64_t* max_ts);

void features_aggregate(Ctx& c, int64_t ne, const int32_t* file_idx, const uint8_t* op,
                        const int32_t* client, const int64_t* ts_us, int64_t n_files,
                        const int32_t* primary, int64_t* out, int64_t* max_ts) {
  if (ne < 0 || n_files < 0) CDR_FAIL(CDR_ERR_ARG, "negative sizes");
  if (n_files >= (1ll << 31)) CDR_FAIL(CDR_ERR_UNSUPPORTED, "n_files >= 2^31");
  *max_ts = LLONG_MIN;
  if (n_files == 0 && ne == 0) return;
  ensure_events(c, ne, n_files);
  if (ne > 0) {
    HIP_CHECK(hipMemcpyAsync(c.ev_file.p, file_idx, 4 * ne, hipMemcpyHostToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(c.ev_op.p, op, ne, hipMemcpyHostToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(c.ev_client.p, client, 4 * ne, hipMemcpyHostToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(c.ev_ts.p, ts_us, 8 * ne, hipMemcpyHostToDevice, c.stream));
  }
  c.ev_tsr_valid = false;  // the group-by computes the range itself
  if (n_files > 0)
    HIP_CHECK(hipMemcpyAsync(c.ev_primary.p, primary, 4 * n_files, hipMemcpyHostToDevice,
                             c.stream));
  int cmax = 0;
  for (int64_t i = 0; i < ne; ++i) cmax = std::max(cmax, (int)client[i]);
  c.ev_cmax = cmax;
  features_aggregate_resident(c, ne, n_files, out, max_ts);
}

// The group-by over the events resident in c.ev_* (uploaded or generated).
// out: host (n_files, 6) or null (results stay in c.ev_out).
void features_aggregate_resident(Ctx& c, int64_t ne, int64_t n_files, int64_t* out,
                                 int64_t* max_ts) {
  *max_ts = LLONG_MIN;
  if (n_files == 0 && ne == 0) return;
  if (groupby_resident(c, ne, n_files, out, max_ts)) return;  // groupby.hip
  // sort-based path: shapes the packed payload cannot hold
  const size_t ne1 = ne > 0 ? ne : 1, nf1 = n_files > 0 ? n_files : 1;
  // timestamp range
  unsigned long long mm_init[2] = {~0ull, 0ull};
  unsigned long long* dmm = reinterpret_cast<unsigned long long*>(c.ev_out.as<char>() + 8 * 6 * nf1);
  HIP_CHECK(hipMemcpyAsync(dmm, mm_init, 16, hipMemcpyHostToDevice, c.stream));
  int* ts_unordered = reinterpret_cast<int*>(c.ev_out.as<char>() + 8 * 6 * nf1 + 20);
  HIP_CHECK(hipMemsetAsync(ts_unordered, 0, 4, c.stream));
  if (ne > 0) {
    const int nb = gcap(ne, 256, 4096);
    c.ev_part.ensure(16 * 4096);
    hipLaunchKernelGGL(ts_minmax, dim3(nb), dim3(256), 0, c.stream, c.ev_ts.as<long long>(), ne,
                       c.ev_part.as<long long>(), ts_unordered);
    hipLaunchKernelGGL(ts_minmax_fin, dim3(1), dim3(256), 0, c.stream,
                       c.ev_part.as<long long>(), nb, dmm);
    HIP_CHECK(hipGetLastError());
  }
  unsigned long long mm[3];
  HIP_CHECK(hipMemcpyAsync(mm, dmm, 24, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  const bool time_ordered = (reinterpret_cast<const int*>(&mm[2])[1]) == 0;
  long long sec_min = 0, sec_max = 0;
  const long long tmin = (long long)(mm[0] ^ (unsigned long long)LLONG_MIN);
  const long long tmax = (long long)(mm[1] ^ (unsigned long long)LLONG_MIN);
  if (ne > 0 && tmin <= tmax) {  // some timestamp is not null
    *max_ts = tmax;
    sec_min = (long long)std::floor((double)tmin / 1000000.0);
    sec_max = (long long)std::floor((double)tmax / 1000000.0);
    if (sec_max - sec_min >= (1ll << 32) - 1)
      CDR_FAIL(CDR_ERR_UNSUPPORTED, "access log spans more than 2^32 seconds");
  }
  // compact sort keys: file << sbits | (sec - sec_min), the null second all
  // ones; invalid events are all ones and sort after every valid key within
  // end_bit
  int sbits = 1, fbits = 1;
  while ((1ll << sbits) - 1 <= sec_max - sec_min) ++sbits;
  while ((1ll << fbits) < n_files) ++fbits;
  const int end_bit = std::min(64, sbits + fbits + 1);
  c.fin_red.ensure(16 * nf1);
  long long* start = c.fin_red.as<long long>();
  long long* end = start + nf1;
  int* unsorted = reinterpret_cast<int*>(c.ev_out.as<char>() + 8 * 6 * nf1 + 16);
  // fast path: time-ordered log, stable 32-bit sort by file only
  int fb32 = 1;
  while ((1ll << fb32) <= n_files) ++fb32;  // all ones (invalid) is not a file id
  if (ne > 1 && time_ordered && fb32 <= 31 && sec_max - sec_min < (1ll << 29)) {
    const unsigned invalid = (unsigned)((1ull << fb32) - 1);
    c.ev_scratch.ensure((size_t)24 * ne1 + 64);
    unsigned long long* v0 = c.ev_scratch.as<unsigned long long>();
    unsigned long long* v1 = v0 + ne1;
    unsigned* k0 = reinterpret_cast<unsigned*>(v1 + ne1);
    unsigned* k1 = k0 + ne1;
    HIP_CHECK(hipMemsetAsync(unsorted, 0, 4, c.stream));
    hipLaunchKernelGGL(make_keys32, dim3(gcap(ne, 256, 8192)), dim3(256), 0, c.stream,
                       c.ev_file.as<int32_t>(), c.ev_op.as<uint8_t>(), c.ev_client.as<int32_t>(),
                       c.ev_ts.as<long long>(), ne, n_files, c.ev_primary.as<int32_t>(), sec_min,
                       invalid, k0, v0);  // primary unused here (per_file32 reads it)
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(check_sorted32, dim3(gcap(ne, 256, 8192)), dim3(256), 0, c.stream, k0,
                       ne, unsorted);
    HIP_CHECK(hipGetLastError());
    int hunsorted = 0;
    HIP_CHECK(hipMemcpyAsync(&hunsorted, unsorted, 4, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    unsigned* keys = k0;
    unsigned long long* vals = v0;
    if (hunsorted) {  // stable: a file's events keep their time order (radix.hip)
      if (radix_sort_pairs(c, k0, k1, v0, v1, ne, fb32)) {
        keys = k1;
        vals = v1;
      }
    }
    HIP_CHECK(hipMemsetAsync(start, 0xFF, 8 * nf1, c.stream));  // -1
    HIP_CHECK(hipMemsetAsync(end, 0, 8 * nf1, c.stream));
    hipLaunchKernelGGL(mark_runs32, dim3(gcap(ne, 256, 8192)), dim3(256), 0, c.stream, keys, ne,
                       invalid, start, end);
    HIP_CHECK(hipGetLastError());
    if (n_files > 0) {
      hipLaunchKernelGGL(per_file32, dim3(ceil_div(n_files, 64)), dim3(64), 0, c.stream,
                         vals, n_files, c.ev_primary.as<int32_t>(), start, end,
                         c.ev_out.as<long long>());
      HIP_CHECK(hipGetLastError());
      if (out)
        HIP_CHECK(hipMemcpyAsync(out, c.ev_out.p, 8 * 6 * n_files, hipMemcpyDeviceToHost,
                                 c.stream));
    }
    HIP_CHECK(hipStreamSynchronize(c.stream));
    return;
  }
  // general path: 64-bit (file, second) keys
  // keys + flags
  c.ev_scratch.ensure((8 + 1) * ne1 * 2 + 64);
  unsigned long long* k0 = c.ev_scratch.as<unsigned long long>();
  unsigned long long* k1 = k0 + ne1;
  uint8_t* f0 = reinterpret_cast<uint8_t*>(k1 + ne1);
  uint8_t* f1 = f0 + ne1;
  HIP_CHECK(hipMemsetAsync(unsorted, 0, 4, c.stream));
  if (ne > 0) {
    hipLaunchKernelGGL(make_keys, dim3(gcap(ne, 256, 8192)), dim3(256), 0, c.stream,
                       c.ev_file.as<int32_t>(), c.ev_op.as<uint8_t>(), c.ev_client.as<int32_t>(),
                       c.ev_ts.as<long long>(), ne, n_files, c.ev_primary.as<int32_t>(), sec_min,
                       sbits, k0, f0);
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(check_sorted, dim3(gcap(ne, 256, 8192)), dim3(256), 0, c.stream, k0, ne,
                       unsorted);
    HIP_CHECK(hipGetLastError());
  }
  int hunsorted = 0;
  HIP_CHECK(hipMemcpyAsync(&hunsorted, unsorted, 4, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  unsigned long long* keys = k0;
  uint8_t* flags = f0;
  if (hunsorted && ne > 1) {
    if (radix_sort_pairs(c, k0, k1, f0, f1, ne, end_bit)) {
      keys = k1;
      flags = f1;
    }
  }
  // runs per file
  HIP_CHECK(hipMemsetAsync(start, 0xFF, 8 * nf1, c.stream));  // -1
  HIP_CHECK(hipMemsetAsync(end, 0, 8 * nf1, c.stream));
  if (ne > 0) {
    hipLaunchKernelGGL(mark_runs, dim3(gcap(ne, 256, 8192)), dim3(256), 0, c.stream, keys, ne,
                       sbits, start, end);
    HIP_CHECK(hipGetLastError());
  }
  if (n_files > 0) {
    hipLaunchKernelGGL(per_file, dim3(gcap(n_files, 256, 8192)), dim3(256), 0, c.stream, keys,
                       flags, n_files, sbits, start, end, c.ev_out.as<long long>());
    HIP_CHECK(hipGetLastError());
    if (out)
      HIP_CHECK(hipMemcpyAsync(out, c.ev_out.p, 8 * 6 * n_files, hipMemcpyDeviceToHost,
                               c.stream));
  }
  HIP_CHECK(hipStreamSynchronize(c.stream));
}

// ---- synthetic access log (device, for the config-4 scale runs) ----------
// A time-ordered log of ne events over n_files manifest files (counter-based,
// so any shard regenerates the same events): event e at ts = t0 + e span / ne
// microseconds, file = uniform over the files (file_begin + ...), op WRITE
// with probability 1/10 else READ, client uniform over 3 datanodes;
// primary[f] uniform over the same 3 (access_simulator.py's dn1..dn3).
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void gen_events(int64_t ne, int64_t n_files, unsigned long long seed, long long t0,
                           long long span, int32_t* __restrict__ file, uint8_t* __restrict__ op,
                           int32_t* __restrict__ client, long long* __restrict__ ts,
                           int32_t* __restrict__ primary) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += stride) {
    const unsigned long long h = mix64(seed ^ ((unsigned long long)e * 0xD1B54A32D192ED03ull));
    file[e] = (int32_t)(((h >> 32) * (unsigned long long)n_files) >> 32);
    op[e] = (((h & 0xFFFFull) * 10ull) >> 16) == 0 ? 1 : 2;
    client[e] = (int32_t)((((h >> 16) & 0xFFFFull) * 3ull) >> 16);
    ts[e] = t0 + (long long)((e * span) / ne);
  }
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n_files; f += stride)
    primary[f] = (int32_t)((((mix64(seed ^ 0x5EEDull ^ ((unsigned long long)f << 1)) >> 48) * 3ull) >> 16));
}

void features_generate(Ctx& c, int64_t ne, int64_t n_files, unsigned long long seed,
                       long long t0_us, long long span_us) {
  if (ne < 0 || n_files < 1) CDR_FAIL(CDR_ERR_ARG, "need n_events >= 0 and n_files >= 1");
  if (n_files >= (1ll << 31)) CDR_FAIL(CDR_ERR_UNSUPPORTED, "n_files >= 2^31");
  if (ne > 0 && span_us > (long long)(LLONG_MAX / ne)) CDR_FAIL(CDR_ERR_ARG, "span too large");
  ensure_events(c, ne, n_files);
  hipLaunchKernelGGL(gen_events, dim3(8192), dim3(256), 0, c.stream, ne, n_files, seed, t0_us,
                     span_us, c.ev_file.as<int32_t>(), c.ev_op.as<uint8_t>(),
                     c.ev_client.as<int32_t>(), c.ev_ts.as<long long>(),
                     c.ev_primary.as<int32_t>());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.ev_n = ne;
  events_ts_range(c, ne);
  c.ev_nf = n_files;
  c.ev_cmax = 2;
}

// ---- K6 -------------------------------------------------------------------
__device__ __forceinline__ unsigned long long fkey(double v) {
  const unsigned long long b = __double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__host__ __device__ inline double fkey_val(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  double v;
  memcpy(&v, &b, 8);
  return v;
}

// red layout (u64): 0 sum_writes, 1/2 min/max af (x^sign), 3/4 min/max writes,
// 5/6 min/max conc, 7/8 min/max age key, 9/10 min/max locality key
__global__ void fin_reduce(const long long* __restrict__ cnt, const double* __restrict__ creation,
                           int64_t n, double obs_end, unsigned long long* __restrict__ red) {
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n;
       f += (int64_t)gridDim.x * blockDim.x) {
    const long long* c = cnt + f * 6;
    const double cr = creation[f];
    const double age = isnan(cr) ? 0.0 : obs_end - cr;
    const double loc = c[4] > 0 ? (double)c[3] / (double)c[4] : 1.0;
    atomicAdd(&red[0], (unsigned long long)c[1]);
    atomicMin(&red[1], (unsigned long long)(c[0] ^ LLONG_MIN));
    atomicMax(&red[2], (unsigned long long)(c[0] ^ LLONG_MIN));
    atomicMin(&red[3], (unsigned long long)(c[1] ^ LLONG_MIN));
    atomicMax(&red[4], (unsigned long long)(c[1] ^ LLONG_MIN));
    atomicMin(&red[5], (unsigned long long)(c[5] ^ LLONG_MIN));
    atomicMax(&red[6], (unsigned long long)(c[5] ^ LLONG_MIN));
    atomicMin(&red[7], fkey(age));
    atomicMax(&red[8], fkey(age));
    atomicMin(&red[9], fkey(loc));
    atomicMax(&red[10], fkey(loc));
  }
}

struct FinConst {
  double obs_end, mean_w;
  long long af_min, af_max, con_min, con_max;
  double age_min, age_max, wr_min, wr_max, loc_min, loc_max;
};

__global__ void fin_apply(const long long* __restrict__ cnt, const double* __restrict__ creation,
                          int64_t n, FinConst k, double* __restrict__ out) {
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n;
       f += (int64_t)gridDim.x * blockDim.x) {
    const long long* c = cnt + f * 6;
    const double cr = creation[f];
    const double age = isnan(cr) ? 0.0 : k.obs_end - cr;
    const double wr = (double)c[1] / k.mean_w;
    const double loc = c[4] > 0 ? (double)c[3] / (double)c[4] : 1.0;
    double* o = out + f * 10;
    o[0] = (double)c[0];
    o[1] = age;
    o[2] = wr;
    o[3] = loc;
    o[4] = (double)c[5];
    o[5] = k.af_max == k.af_min ? 0.0 : (double)(c[0] - k.af_min) / (double)(k.af_max - k.af_min);
    o[6] = k.age_max == k.age_min ? 0.0 : (age - k.age_min) / (k.age_max - k.age_min);
    o[7] = k.wr_max == k.wr_min ? 0.0 : (wr - k.wr_min) / (k.wr_max - k.wr_min);
    o[8] = k.loc_max == k.loc_min ? 0.0 : (loc - k.loc_min) / (k.loc_max - k.loc_min);
    o[9] = k.con_max == k.con_min ? 0.0
                                  : (double)(c[5] - k.con_min) / (double)(k.con_max - k.con_min);
  }
}

// Uploads counts / creation and reduces them: istats = {sum writes, min/max
// access_freq, min/max writes, min/max concurrency}, dstats = {min/max age,
// min/max locality} (identities when n == 0), the inputs of :62-83.
static void fin_stats(Ctx& c, int64_t n, const int64_t* counts, const double* creation,
                      double obs_end, int64_t* istats, double* dstats) {
  auto sx = [](unsigned long long v) { return (long long)(v ^ (unsigned long long)LLONG_MIN); };
  unsigned long long init[11] = {0, ~0ull, 0, ~0ull, 0, ~0ull, 0, ~0ull, 0, ~0ull, 0};
  unsigned long long r[11];
  if (n > 0) {
    c.fin_counts.ensure(8 * 6 * n);
    c.fin_creation.ensure(8 * n);
    c.fin_red.ensure(8 * 16);
    HIP_CHECK(hipMemcpyAsync(c.fin_counts.p, counts, 8 * 6 * n, hipMemcpyHostToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(c.fin_creation.p, creation, 8 * n, hipMemcpyHostToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(c.fin_red.p, init, sizeof(init), hipMemcpyHostToDevice, c.stream));
    hipLaunchKernelGGL(fin_reduce, dim3(gcap(n, 256, 4096)), dim3(256), 0, c.stream,
                       c.fin_counts.as<long long>(), c.fin_creation.as<double>(), n, obs_end,
                       c.fin_red.as<unsigned long long>());
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(r, c.fin_red.p, sizeof(r), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    istats[0] = (long long)r[0];
    for (int i = 1; i <= 6; ++i) istats[i] = sx(r[i]);
    for (int i = 0; i < 4; ++i) dstats[i] = fkey_val(r[7 + i]);
  } else {
    istats[0] = 0;
    for (int i = 1; i <= 5; i += 2) {
      istats[i] = LLONG_MAX;
      istats[i + 1] = LLONG_MIN;
    }
    for (int i = 0; i < 4; i += 2) {
      dstats[i] = INFINITY;
      dstats[i + 1] = -INFINITY;
    }
  }
}

// The table of n rows (counts / creation already on the device when
// uploaded is true) from global statistics over n_rows rows.
static void fin_apply(Ctx& c, int64_t n, const int64_t* counts, const double* creation,
                      double obs_end, const int64_t* istats, const double* dstats,
                      int64_t n_rows, bool uploaded, double* out) {
  if (n == 0) return;
  if (!uploaded) {
    c.fin_counts.ensure(8 * 6 * n);
    c.fin_creation.ensure(8 * n);
    HIP_CHECK(hipMemcpyAsync(c.fin_counts.p, counts, 8 * 6 * n, hipMemcpyHostToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(c.fin_creation.p, creation, 8 * n, hipMemcpyHostToDevice, c.stream));
  }
  c.fin_out.ensure(8 * 10 * n);
  FinConst k;
  k.obs_end = obs_end;
  double mean = (double)istats[0] / (double)n_rows;  // Spark avg: double sum / count
  if (mean == 0.0) mean = 1.0;
  k.mean_w = mean;
  k.af_min = istats[1];
  k.af_max = istats[2];
  k.con_min = istats[5];
  k.con_max = istats[6];
  k.age_min = dstats[0];
  k.age_max = dstats[1];
  k.wr_min = (double)istats[3] / mean;  // x -> x / mean is monotone
  k.wr_max = (double)istats[4] / mean;
  k.loc_min = dstats[2];
  k.loc_max = dstats[3];
  hipLaunchKernelGGL(fin_apply, dim3(gcap(n, 256, 4096)), dim3(256), 0, c.stream,
                     c.fin_counts.as<long long>(), c.fin_creation.as<double>(), n, k,
                     c.fin_out.as<double>());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(out, c.fin_out.p, 8 * 10 * n, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
}

void features_finalize(Ctx& c, int64_t n, const int64_t* counts, const double* creation,
                       double obs_end, double* out) {
  if (n < 0) CDR_FAIL(CDR_ERR_ARG, "negative n_files");
  if (n == 0) return;
  int64_t is[7];
  double ds[4];
  fin_stats(c, n, counts, creation, obs_end, is, ds);
  fin_apply(c, n, counts, creation, obs_end, is, ds, n, true, out);
}

}  // namespace cdr

using namespace cdr;

extern "C" {

int cdr_features_aggregate(cdr_ctx* h, int64_t n_events, const int32_t* file_idx,
                           const uint8_t* op, const int32_t* client, const int64_t* ts_us,
                           int64_t n_files, const int32_t* primary, int64_t* out,
                           int64_t* max_ts_us) {
  CDR_TRY
  if (!h || !max_ts_us || (n_events > 0 && (!file_idx || !op || !client || !ts_us)) ||
      (n_files > 0 && (!primary || !out)))
    CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  features_aggregate(h->c, n_events, file_idx, op, client, ts_us, n_files, primary, out,
                     max_ts_us);
  CDR_CATCH
}

int cdr_features_generate(cdr_ctx* h, int64_t n_events, int64_t n_files, uint64_t seed,
                          int64_t t0_us, int64_t span_us) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  HIP_CHECK(hipSetDevice(h->c.device));
  features_generate(h->c, n_events, n_files, seed, t0_us, span_us);
  CDR_CATCH
}

int cdr_features_aggregate_resident(cdr_ctx* h, int64_t* out, int64_t* max_ts_us) {
  CDR_TRY
  if (!h || !max_ts_us) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  if (c.ev_nf <= 0) CDR_FAIL(CDR_ERR_STATE, "no resident events (cdr_features_generate)");
  HIP_CHECK(hipSetDevice(c.device));
  features_aggregate_resident(c, c.ev_n, c.ev_nf, out, max_ts_us);
  CDR_CATCH
}

int cdr_features_groupby_info(cdr_ctx* h, int64_t* info) {
  CDR_TRY
  if (!h || !info) CDR_FAIL(CDR_ERR_ARG, "null argument");
  const Ctx& c = h->c;
  info[0] = c.gb_last_hand;
  info[1] = c.gb_last_L;
  info[2] = c.gb_last_passes;
  info[3] = c.gb_last_pbytes;
  info[4] = c.gb_last_big;
  info[5] = c.gb_last_dense;
  info[6] = c.gb_last_grid;
  CDR_CATCH
}

int cdr_features_events_read(cdr_ctx* h, int32_t* file_idx, uint8_t* op, int32_t* client,
                             int64_t* ts_us, int32_t* primary) {
  CDR_TRY
  if (!h || !file_idx || !op || !client || !ts_us || !primary)
    CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  if (c.ev_nf <= 0) CDR_FAIL(CDR_ERR_STATE, "no resident events (cdr_features_generate)");
  HIP_CHECK(hipSetDevice(c.device));
  const int64_t ne = c.ev_n;
  if (ne > 0) {
    HIP_CHECK(hipMemcpyAsync(file_idx, c.ev_file.p, 4 * ne, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipMemcpyAsync(op, c.ev_op.p, ne, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipMemcpyAsync(client, c.ev_client.p, 4 * ne, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipMemcpyAsync(ts_us, c.ev_ts.p, 8 * ne, hipMemcpyDeviceToHost, c.stream));
  }
  HIP_CHECK(hipMemcpyAsync(primary, c.ev_primary.p, 4 * c.ev_nf, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  CDR_CATCH
}

int cdr_features_finalize_stats(cdr_ctx* h, int64_t n_rows, const int64_t* counts,
                                const double* creation_s, double observation_end,
                                int64_t* istats, double* dstats) {
  CDR_TRY
  if (!h || !istats || !dstats || (n_rows > 0 && (!counts || !creation_s)))
    CDR_FAIL(CDR_ERR_ARG, "null argument");
  if (n_rows < 0) CDR_FAIL(CDR_ERR_ARG, "negative n_rows");
  HIP_CHECK(hipSetDevice(h->c.device));
  fin_stats(h->c, n_rows, counts, creation_s, observation_end, istats, dstats);
  CDR_CATCH
}

int cdr_features_finalize_apply(cdr_ctx* h, int64_t n_rows, const int64_t* counts,
                                const double* creation_s, double observation_end,
                                const int64_t* istats, const double* dstats,
                                int64_t n_rows_total, double* out) {
  CDR_TRY
  if (!h || !istats || !dstats || (n_rows > 0 && (!counts || !creation_s || !out)))
    CDR_FAIL(CDR_ERR_ARG, "null argument");
  if (n_rows < 0 || n_rows_total < n_rows || n_rows_total < 1)
    CDR_FAIL(CDR_ERR_ARG, "need 0 <= n_rows <= n_rows_total, n_rows_total >= 1");
  HIP_CHECK(hipSetDevice(h->c.device));
  fin_apply(h->c, n_rows, counts, creation_s, observation_end, istats, dstats, n_rows_total,
            false, out);
  CDR_CATCH
}

int cdr_features_finalize(cdr_ctx* h, int64_t n_files, const int64_t* counts,
                          const double* creation_s, double observation_end, double* out) {
  CDR_TRY
  if (!h || (n_files > 0 && (!counts || !creation_s || !out)))
    CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  features_finalize(h->c, n_files, counts, creation_s, observation_end, out);
  CDR_CATCH
}

}  // extern "C"
