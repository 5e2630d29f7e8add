// groupby.hip — the access-log group-by of src/compute_features.py:31-46 as a
// two-level MSD partition of the events by file id followed by one LDS hash
// group-by per bucket of 2^L consecutive files.  No library sort.
//
// Per event the counters are (:31-42) count, WRITE, READ, local (client ==
// primary node of its file); max_concurrency (:44-46) is the largest count of
// one (file, second) pair, the null second (unparseable timestamp) being a
// pair of its own.  All of them are order-independent sums and maxima, so the
// partition may place events of one bucket in any order.
//
//   K1  gb_hist1    per 8192-event tile: histogram of the pass-1 digit (the
//                   top B1 bits of the file id), in-chunk prefix per tile;
//                   timestamp min / max / null flag (file 4 B + ts 8 B read)
//   S1  gb_scan1    chunk bases, digit bases, pass-2 tile starts, ts range
//   --- host reads the ts range (the payload layout depends on it) ---
//   P1  gb_scatter1 tile -> LDS-ranked by digit -> coalesced runs into the
//                   digit regions; builds the packed payload
//                   [file low bits | second code | op | client code]
//                   (17 B read, 4 or 8 B written)
//   H2  gb_hist2    per pass-2 tile (a slice of one digit region): histogram
//                   of the pass-2 digit (payload read)
//   S2  gb_scan2    one workgroup per pass-1 digit: tile offsets and bucket
//                   bases
//   P2  gb_scatter2 like P1 within each digit region (payload read + written)
//   K4  gb_bucket   one workgroup per bucket: LDS hash of (file, second) ->
//                   count (one 64-bit slot = key << CB | count), per-file
//                   count / write / read / local sums and the concurrency
//                   maximum in LDS, then the (files, 6) int64 rows; buckets
//                   over the LDS capacity are listed and redone by
//                   gb_bucket_big with the hash in global memory.
// With B <= 9 bucket bits one partition pass suffices (H2/S2/P2 skipped).
#include <algorithm>
#include <cmath>

#include "cdr_internal.h"

namespace cdr {

int lloyd_num_cus(int device);

namespace {

constexpr int kGbTile = 8192;                   // events per partition tile
constexpr int kGbThreads = 512;                 // partition / histogram workgroups
constexpr int kGbPer = kGbTile / kGbThreads;    // events per thread in a tile
constexpr int kGbChunkTiles = 8;                // tiles per gb_hist1 workgroup
constexpr int kGbRange = 16;                    // chunks per gb_scan1a/c workgroup
constexpr int kGbMaxDigit = 9;                  // bits per partition pass
constexpr int kGbMaxBins = 1 << kGbMaxDigit;
constexpr int kGbBThreads = 256;                // bucket workgroups
constexpr int kGbSlots = 4096;                  // LDS hash slots per bucket
constexpr int kGbLdsCap = 3072;                 // events per bucket in LDS (load <= 3/4)
constexpr int kGbReg = kGbLdsCap / kGbBThreads; // payloads per bucket thread
constexpr int kGbMaxL = 10;                     // files per bucket <= 1024
constexpr long long kTsNullG = LLONG_MIN;
constexpr unsigned long long kEmpty = ~0ull;

__device__ __forceinline__ long long sec_of_g(long long ts_us) {
  // Spark floor(cast(ts as double)); see features.hip sec_of
  if (ts_us >= 0 && ts_us < 9000000000000000ll) return ts_us / 1000000;
  return (long long)floor((double)ts_us / 1000000.0);
}

// Payload layout (host-computed, passed by value).
struct GbPay {
  int fshift;   // bit position of the file-low field
  int sshift;   // bit position of the second code (= 2 + cbits)
  int cbits;    // client code bits (code 0 = not a node id, else client + 1)
  int sbits;    // second code bits (all ones = null)
  int L;        // file-local bits (files per bucket = 2^L)
  long long sec_min;
  unsigned long long low_mask;  // file-low field mask (fbits - B1 bits)
};

template <typename T>
__device__ __forceinline__ T gb_make(const GbPay& p, unsigned flow, long long ts, uint8_t op,
                                     int client) {
  const unsigned long long sc = ts == kTsNullG ? ((1ull << p.sbits) - 1)
                                               : (unsigned long long)(sec_of_g(ts) - p.sec_min);
  const unsigned long long oc = op == 1 ? 1ull : (op == 2 ? 2ull : 0ull);
  const unsigned long long cc = client >= 0 ? (unsigned long long)client + 1ull : 0ull;
  return (T)(((unsigned long long)flow << p.fshift) | (sc << p.sshift) | (oc << p.cbits) | cc);
}

// Exclusive scan of n <= 512 LDS counters by a 512-thread workgroup (one
// counter per thread).
__device__ __forceinline__ void lds_scan(const unsigned* cnt, unsigned* lp, int n,
                                         unsigned* wsum) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const unsigned v = t < n ? cnt[t] : 0u;
  unsigned inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  unsigned base = 0;
  for (int i = 0; i < w; ++i) base += wsum[i];
  if (t < n) lp[t] = base + inc - v;
  __syncthreads();
}

// ---- K1 --------------------------------------------------------------------
// TS = false: the producer already has the timestamp range (events_ts_range),
// only the file ids are read (4 B per event instead of 12).
template <bool TS>
__global__ __launch_bounds__(kGbThreads) void gb_hist1(
    const int32_t* __restrict__ file, const long long* __restrict__ ts, int64_t ne, int64_t nf,
    int shift1, int R1, unsigned* __restrict__ tilepref, unsigned* __restrict__ chunksum,
    long long* __restrict__ part) {
  __shared__ unsigned hist[kGbMaxBins];
  __shared__ long long red[3][kGbThreads / 64];
  const int tid = threadIdx.x;
  const int64_t c = blockIdx.x;
  unsigned run = 0;  // thread r owns digit r
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  long long nul = 0;
  for (int tt = 0; tt < kGbChunkTiles; ++tt) {
    const int64_t t = c * kGbChunkTiles + tt;
    const int64_t base = t * kGbTile;
    if (base >= ne) break;
    if (tid < R1) hist[tid] = 0;
    int fr[kGbPer];
    long long tv[kGbPer];
#pragma unroll
    for (int j = 0; j < kGbPer; ++j) {
      const int64_t e = base + j * kGbThreads + tid;
      fr[j] = e < ne ? file[e] : -1;
      tv[j] = (TS && e < ne) ? ts[e] : kTsNullG;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kGbPer; ++j) {
      const int64_t e = base + j * kGbThreads + tid;
      if (!TS) {
      } else if (tv[j] == kTsNullG) {
        nul |= e < ne;
      } else {
        lo = min(lo, tv[j]);
        hi = max(hi, tv[j]);
      }
      if (fr[j] >= 0 && fr[j] < nf) atomicAdd(&hist[(unsigned)fr[j] >> shift1], 1u);
    }
    __syncthreads();
    if (tid < R1) {
      tilepref[t * R1 + tid] = run;
      run += hist[tid];
    }
  }
  if (tid < R1) chunksum[c * R1 + tid] = run;
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o));
    hi = max(hi, __shfl_xor(hi, o));
    nul |= __shfl_xor(nul, o);
  }
  const int w = tid >> 6;
  if ((tid & 63) == 0) {
    red[0][w] = lo;
    red[1][w] = hi;
    red[2][w] = nul;
  }
  __syncthreads();
  if (tid == 0) {
    for (int i = 1; i < kGbThreads / 64; ++i) {
      lo = min(lo, red[0][i]);
      hi = max(hi, red[1][i]);
      nul |= red[2][i];
    }
    part[3 * c] = lo;
    part[3 * c + 1] = hi;
    part[3 * c + 2] = nul;
  }
}

// ---- S1: chunk bases in three small kernels ---------------------------------
// a: per range of kGbRange chunks, the digit sums; b (one workgroup): range
// bases per digit, digit bases, pass-2 tile starts, the timestamp range;
// c: absolute chunk bases (digit base + range base + in-range prefix).
__global__ __launch_bounds__(kGbMaxBins) void gb_scan1a(const unsigned* __restrict__ chunk,
                                                        int64_t C, int R1,
                                                        unsigned* __restrict__ rsum) {
  const int r = threadIdx.x;
  if (r >= R1) return;
  const int64_t c0 = (int64_t)blockIdx.x * kGbRange;
  unsigned v[kGbRange];
#pragma unroll
  for (int j = 0; j < kGbRange; ++j) v[j] = c0 + j < C ? chunk[(c0 + j) * R1 + r] : 0u;
  unsigned s = 0;
#pragma unroll
  for (int j = 0; j < kGbRange; ++j) s += v[j];
  rsum[(int64_t)blockIdx.x * R1 + r] = s;
}

__global__ __launch_bounds__(kGbMaxBins) void gb_scan1b(unsigned* __restrict__ rsum, int64_t G,
                                                        int R1, const long long* __restrict__ part,
                                                        int64_t C, unsigned* __restrict__ binbase,
                                                        int* __restrict__ tile2start,
                                                        long long* __restrict__ res,
                                                        const long long* __restrict__ tsr) {
  __shared__ long long wred[3][8];
  __shared__ unsigned wsum[8], wt[8];
  const int tid = threadIdx.x;
  unsigned run = 0;
  if (tid < R1) {
    for (int64_t g0 = 0; g0 < G; g0 += 16) {
      unsigned v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = g0 + j < G ? rsum[(g0 + j) * R1 + tid] : 0u;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (g0 + j < G) rsum[(g0 + j) * R1 + tid] = run;
        run += v[j];
      }
    }
  }
  long long lo = LLONG_MAX, hi = LLONG_MIN, nul = 0;
  for (int64_t c = tid; c < C; c += kGbMaxBins) {
    lo = min(lo, part[3 * c]);
    hi = max(hi, part[3 * c + 1]);
    nul |= part[3 * c + 2];
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o));
    hi = max(hi, __shfl_xor(hi, o));
    nul |= __shfl_xor(nul, o);
  }
  const int lane = tid & 63, w = tid >> 6;
  if (lane == 0) {
    wred[0][w] = lo;
    wred[1][w] = hi;
    wred[2][w] = nul;
  }
  // exclusive scans over the digits (events and pass-2 tile counts)
  const unsigned v = tid < R1 ? run : 0u;
  const unsigned tl = (unsigned)((v + kGbTile - 1) / kGbTile);
  unsigned iv = v, it = tl;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned a = __shfl_up(iv, o), b = __shfl_up(it, o);
    if (lane >= o) {
      iv += a;
      it += b;
    }
  }
  if (lane == 63) {
    wsum[w] = iv;
    wt[w] = it;
  }
  __syncthreads();
  unsigned bv = 0, bt = 0;
  for (int i = 0; i < w; ++i) {
    bv += wsum[i];
    bt += wt[i];
  }
  if (tid < R1) {
    binbase[tid] = bv + iv - v;
    tile2start[tid] = (int)(bt + it - tl);
  }
  if (tid == kGbMaxBins - 1) {
    binbase[R1] = bv + iv;
    tile2start[R1] = (int)(bt + it);
    res[3] = bt + it;
    res[4] = bv + iv;
  }
  if (tid == 0) {
    for (int i = 1; i < 8; ++i) {
      lo = min(lo, wred[0][i]);
      hi = max(hi, wred[1][i]);
      nul |= wred[2][i];
    }
    res[0] = tsr ? tsr[0] : lo;
    res[1] = tsr ? tsr[1] : hi;
    res[2] = tsr ? tsr[2] : nul;
  }
}

// Timestamp range of n events (min and max of the non-null ones, any null):
// per-workgroup partials, then one workgroup.
__global__ __launch_bounds__(256) void gb_tsr_part(const long long* __restrict__ ts, int64_t n,
                                                   long long* __restrict__ part) {
  long long lo = LLONG_MAX, hi = LLONG_MIN, nul = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const long long t = ts[i];
    if (t == kTsNullG) {
      nul = 1;
    } else {
      lo = min(lo, t);
      hi = max(hi, t);
    }
  }
  __shared__ long long red[3][4];
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o));
    hi = max(hi, __shfl_xor(hi, o));
    nul |= __shfl_xor(nul, o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = lo;
    red[1][w] = hi;
    red[2][w] = nul;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) {
      lo = min(lo, red[0][i]);
      hi = max(hi, red[1][i]);
      nul |= red[2][i];
    }
    part[3 * blockIdx.x] = lo;
    part[3 * blockIdx.x + 1] = hi;
    part[3 * blockIdx.x + 2] = nul;
  }
}

__global__ __launch_bounds__(64) void gb_tsr_fin(const long long* __restrict__ part, int nb,
                                                 long long* __restrict__ out) {
  long long lo = LLONG_MAX, hi = LLONG_MIN, nul = 0;
  for (int b = threadIdx.x; b < nb; b += 64) {
    lo = min(lo, part[3 * b]);
    hi = max(hi, part[3 * b + 1]);
    nul |= part[3 * b + 2];
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o));
    hi = max(hi, __shfl_xor(hi, o));
    nul |= __shfl_xor(nul, o);
  }
  if (threadIdx.x == 0) {
    out[0] = lo;
    out[1] = hi;
    out[2] = nul;
  }
}

__global__ __launch_bounds__(kGbMaxBins) void gb_scan1c(unsigned* __restrict__ chunk, int64_t C,
                                                        int R1, const unsigned* __restrict__ rbase,
                                                        const unsigned* __restrict__ binbase) {
  const int r = threadIdx.x;
  if (r >= R1) return;
  const int64_t c0 = (int64_t)blockIdx.x * kGbRange;
  unsigned v[kGbRange];
#pragma unroll
  for (int j = 0; j < kGbRange; ++j) v[j] = c0 + j < C ? chunk[(c0 + j) * R1 + r] : 0u;
  unsigned run = binbase[r] + rbase[(int64_t)blockIdx.x * R1 + r];
#pragma unroll
  for (int j = 0; j < kGbRange; ++j) {
    if (c0 + j < C) chunk[(c0 + j) * R1 + r] = run;
    run += v[j];
  }
}

// ---- P1 / P2 ----------------------------------------------------------------
// Tile order: blocks are dealt round-robin over the 8 XCDs, so block b works
// on tile (b % 8) * per + b / 8: each XCD walks one contiguous range of tiles
// and a digit's consecutive runs are written from one L2.
__device__ __forceinline__ int64_t xcd_tile(int64_t per) {
  return (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
}

template <typename T>
struct GbStage {
  T val[kGbTile];
  uint16_t dig[kGbTile];
  unsigned cnt[kGbMaxBins], lp[kGbMaxBins], goff[kGbMaxBins];
  unsigned wsum[8];
};

// Rank the tile's events by digit in LDS, stage them digit-contiguous, and
// write each digit's run to its region (goff[d] = the run's first position).
// dr[j] = digit of event j, or ~0u when the event is not placed.
template <typename T>
__device__ __forceinline__ void gb_place(GbStage<T>& s, const T* val, unsigned* dr, int R,
                                         T* __restrict__ out) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < kGbPer; ++j)
    if (dr[j] != ~0u) dr[j] = (dr[j] << 16) | atomicAdd(&s.cnt[dr[j]], 1u);
  __syncthreads();
  lds_scan(s.cnt, s.lp, R, s.wsum);
#pragma unroll
  for (int j = 0; j < kGbPer; ++j) {
    if (dr[j] != ~0u) {
      const unsigned d = dr[j] >> 16;
      const unsigned slot = s.lp[d] + (dr[j] & 0xFFFFu);
      s.val[slot] = val[j];
      s.dig[slot] = (uint16_t)d;
    }
  }
  __syncthreads();
  const unsigned nv = s.lp[R - 1] + s.cnt[R - 1];
  for (unsigned i = tid; i < nv; i += kGbThreads) {
    const unsigned d = s.dig[i];
    out[s.goff[d] + (i - s.lp[d])] = s.val[i];
  }
}

template <typename T>
__global__ __launch_bounds__(kGbThreads) __attribute__((amdgpu_waves_per_eu(4))) void gb_scatter1(
    const int32_t* __restrict__ file, const uint8_t* __restrict__ op,
    const int32_t* __restrict__ client, const long long* __restrict__ ts, int64_t ne, int64_t nf,
    GbPay p, int shift1, int R1, int64_t T1, int64_t per, const unsigned* __restrict__ tilepref,
    const unsigned* __restrict__ chunkbase, T* __restrict__ out) {
  __shared__ GbStage<T> s;
  const int64_t t = xcd_tile(per);
  if (t >= T1) return;
  const int tid = threadIdx.x;
  const int64_t base = t * kGbTile;
  const int64_t c = t / kGbChunkTiles;
  if (tid < R1) {
    s.cnt[tid] = 0;
    s.goff[tid] = chunkbase[c * R1 + tid] + tilepref[t * R1 + tid];
  }
  // thread tid takes the tile's event quads q = j * 512 + tid (events
  // base + 4 q .. + 3), j = 0..3: every load instruction of a wave reads one
  // contiguous span (file / client ids 1 KiB, timestamps 2 x 1 KiB, op bytes
  // 256 B), so each cache line is used whole by the instruction that brings
  // it in.  (Lane-contiguous runs of 16 events left lines half-read between
  // instructions and, with the tile's working set over the L2, re-fetched:
  // 29.6 B read per 17-B event.)  The order of events inside a tile does not
  // matter to the partition.
  T val[kGbPer];
  unsigned dr[kGbPer];
  const bool full = base + kGbTile <= ne;
#pragma unroll
  for (int j = 0; j < kGbPer / 4; ++j) {
    const int64_t q = (int64_t)j * kGbThreads + tid;
    const int64_t eq = base + 4 * q;
    int fr[4], cv[4];
    long long tv[4];
    uint8_t ov[4];
    if (full) {
      const int4 a = reinterpret_cast<const int4*>(file + base)[q];
      const int4 b = reinterpret_cast<const int4*>(client + base)[q];
      const longlong2 t0 = reinterpret_cast<const longlong2*>(ts + base)[2 * q];
      const longlong2 t1 = reinterpret_cast<const longlong2*>(ts + base)[2 * q + 1];
      const unsigned o4 = reinterpret_cast<const unsigned*>(op + base)[q];
      fr[0] = a.x, fr[1] = a.y, fr[2] = a.z, fr[3] = a.w;
      cv[0] = b.x, cv[1] = b.y, cv[2] = b.z, cv[3] = b.w;
      tv[0] = t0.x, tv[1] = t0.y, tv[2] = t1.x, tv[3] = t1.y;
#pragma unroll
      for (int r = 0; r < 4; ++r) ov[r] = (uint8_t)(o4 >> (8 * r));
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t e = eq + r;
        const bool in = e < ne;
        fr[r] = in ? file[e] : -1;
        tv[r] = in ? ts[e] : 0;
        ov[r] = in ? op[e] : 0;
        cv[r] = in ? client[e] : -1;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = 4 * j + r;
      dr[o] = (fr[r] >= 0 && fr[r] < nf) ? (unsigned)fr[r] >> shift1 : ~0u;
      val[o] = gb_make<T>(p, (unsigned)((unsigned long long)(unsigned)fr[r] & p.low_mask), tv[r],
                          ov[r], cv[r]);
    }
  }
  __syncthreads();
  gb_place<T>(s, val, dr, R1, out);
}

__device__ __forceinline__ int find_digit(const int* __restrict__ start, int R1, int64_t t2) {
  int lo = 0, hi = R1;  // start[lo] <= t2 < start[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (start[mid] <= t2) lo = mid;
    else hi = mid;
  }
  return lo;
}

template <typename T>
__global__ __launch_bounds__(kGbThreads) void gb_hist2(const T* __restrict__ in,
                                                      const unsigned* __restrict__ binbase,
                                                      const int* __restrict__ tile2start, int R1,
                                                      int R2, int shift2,
                                                      unsigned* __restrict__ hist2) {
  __shared__ unsigned h[kGbMaxBins];
  const int64_t t2 = blockIdx.x;
  const int sd = find_digit(tile2start, R1, t2);
  const int64_t beg = binbase[sd] + (t2 - tile2start[sd]) * (int64_t)kGbTile;
  const int64_t end = min((int64_t)binbase[sd + 1], beg + kGbTile);
  if (threadIdx.x < R2) h[threadIdx.x] = 0;
  T v[kGbPer];
#pragma unroll
  for (int j = 0; j < kGbPer; ++j) {
    const int64_t i = beg + j * kGbThreads + threadIdx.x;
    v[j] = i < end ? in[i] : (T)0;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kGbPer; ++j)
    if (beg + j * kGbThreads + threadIdx.x < end)
      atomicAdd(&h[(unsigned)((unsigned long long)v[j] >> shift2) & (R2 - 1)], 1u);
  __syncthreads();
  if (threadIdx.x < R2) hist2[t2 * R2 + threadIdx.x] = h[threadIdx.x];
}

// Pass 3 (large file counts): the R regions of pass 2 (bases bbase[0..R])
// become the regions pass 3 splits; tstart[r] = the 8192-event tiles before
// region r (exclusive scan of ceil(size / tile)), tstart[R] and *tot the
// total.  Two launches of kGbT3Per regions per workgroup, one region per
// thread: gb_tilecount3 sums each workgroup's tile counts, gb_tilestart3 adds
// the earlier workgroups' sums and scans its own regions.  (One workgroup
// walking all 2^18 regions of the 1B-event log took 0.43 ms per step.)
constexpr int kGbT3Per = 1024;
__device__ __forceinline__ unsigned gb_tiles_of(const unsigned* __restrict__ bbase, int r, int R) {
  return r < R ? (bbase[r + 1] - bbase[r] + kGbTile - 1) / kGbTile : 0u;
}
__global__ __launch_bounds__(kGbT3Per) void gb_tilecount3(const unsigned* __restrict__ bbase, int R,
                                                          unsigned* __restrict__ wsum) {
  __shared__ unsigned ws[kGbT3Per / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  unsigned c = gb_tiles_of(bbase, blockIdx.x * kGbT3Per + t, R);
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if (lane == 0) ws[w] = c;
  __syncthreads();
  if (t == 0) {
    unsigned s = 0;
    for (int i = 0; i < kGbT3Per / 64; ++i) s += ws[i];
    wsum[blockIdx.x] = s;
  }
}
__global__ __launch_bounds__(kGbT3Per) void gb_tilestart3(const unsigned* __restrict__ bbase, int R,
                                                          const unsigned* __restrict__ wsum,
                                                          int* __restrict__ tstart,
                                                          long long* __restrict__ tot) {
  __shared__ unsigned wb[kGbT3Per / 64], wi[kGbT3Per / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // this workgroup's base: the earlier workgroups' tile sums (a share per
  // wave, added up below)
  unsigned bs = 0;
  for (int i = t; i < (int)blockIdx.x; i += kGbT3Per) bs += wsum[i];
  for (int o = 32; o > 0; o >>= 1) bs += __shfl_xor(bs, o);
  // its regions' tile counts, scanned by waves and then across them
  const int r = blockIdx.x * kGbT3Per + t;
  const unsigned c = gb_tiles_of(bbase, r, R);
  unsigned inc = c;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 0) wb[w] = bs;
  if (lane == 63) wi[w] = inc;
  __syncthreads();
  unsigned run = inc - c;
  for (int i = 0; i < kGbT3Per / 64; ++i) {
    run += wb[i];             // the earlier workgroups' tiles
    if (i < w) run += wi[i];  // the earlier waves' regions
  }
  if (r < R) tstart[r] = (int)run;
  if (r == R - 1) {
    tstart[R] = (int)(run + c);
    *tot = (long long)(run + c);
  }
}

// Pass 3's scan with few bins (R3 <= 16): one thread per region sd (most
// regions span one or two tiles): running offsets over its tiles per bin,
// then its bucket bases bbase3[sd * R3 + r].
constexpr int kGbScan3Max = 16;
__global__ __launch_bounds__(256) void gb_scan3(unsigned* __restrict__ hist3,
                                                const int* __restrict__ tstart,
                                                const unsigned* __restrict__ bbase, int R12, int R3,
                                                unsigned* __restrict__ bbase3) {
  const int sd = blockIdx.x * 256 + threadIdx.x;
  if (sd >= R12) return;
  const int t0 = tstart[sd], t1 = tstart[sd + 1];
  unsigned base = bbase[sd];
  for (int r = 0; r < R3; ++r) {
    unsigned run = 0;
    for (int tb = t0; tb < t1; ++tb) {
      const unsigned v = hist3[(int64_t)tb * R3 + r];
      hist3[(int64_t)tb * R3 + r] = run;
      run += v;
    }
    bbase3[(int64_t)sd * R3 + r] = base;
    base += run;
  }
  if (sd == R12 - 1) bbase3[(int64_t)R12 * R3] = bbase[R12];
}

// One workgroup per pass-1 digit sd, thread r = pass-2 digit: running offsets
// over the digit's tiles, then the bucket bases bbase[sd * R2 + r].
__global__ __launch_bounds__(kGbMaxBins) void gb_scan2(unsigned* __restrict__ hist2,
                                                       const int* __restrict__ tile2start,
                                                       const unsigned* __restrict__ binbase,
                                                       int R1, int R2,
                                                       unsigned* __restrict__ bbase) {
  __shared__ unsigned cnt[kGbMaxBins], lp[kGbMaxBins], wsum[8];
  const int sd = blockIdx.x, r = threadIdx.x;
  const int t0 = tile2start[sd], t1 = tile2start[sd + 1];
  unsigned run = 0;
  if (r < R2) {
    for (int tb = t0; tb < t1; tb += 16) {
      unsigned v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = tb + j < t1 ? hist2[(int64_t)(tb + j) * R2 + r] : 0u;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (tb + j < t1) hist2[(int64_t)(tb + j) * R2 + r] = run;
        run += v[j];
      }
    }
    cnt[r] = run;
  }
  __syncthreads();
  lds_scan(cnt, lp, R2, wsum);
  if (r < R2) bbase[(int64_t)sd * R2 + r] = binbase[sd] + lp[r];
  if (sd == R1 - 1 && r == 0) bbase[(int64_t)R1 * R2] = binbase[R1];
}

template <typename T>
__global__ __launch_bounds__(kGbThreads) void gb_scatter2(
    const T* __restrict__ in, const unsigned* __restrict__ binbase,
    const int* __restrict__ tile2start, int R1, int R2, int shift2, int64_t T2, int64_t per,
    const unsigned* __restrict__ off2, const unsigned* __restrict__ bbase, T* __restrict__ out) {
  __shared__ GbStage<T> s;
  const int64_t t2 = xcd_tile(per);
  if (t2 >= T2) return;
  const int tid = threadIdx.x;
  const int sd = find_digit(tile2start, R1, t2);
  const int64_t beg = binbase[sd] + (t2 - tile2start[sd]) * (int64_t)kGbTile;
  const int64_t end = min((int64_t)binbase[sd + 1], beg + kGbTile);
  if (tid < R2) {
    s.cnt[tid] = 0;
    s.goff[tid] = bbase[(int64_t)sd * R2 + tid] + off2[t2 * R2 + tid];
  }
  T val[kGbPer];
  unsigned dr[kGbPer];
#pragma unroll
  for (int j = 0; j < kGbPer; ++j) {
    const int64_t i = beg + j * kGbThreads + tid;
    val[j] = i < end ? in[i] : (T)0;
  }
#pragma unroll
  for (int j = 0; j < kGbPer; ++j)
    dr[j] = beg + j * kGbThreads + tid < end
                ? (unsigned)((unsigned long long)val[j] >> shift2) & (R2 - 1)
                : ~0u;
  __syncthreads();
  gb_place<T>(s, val, dr, R2, out);
}

// ---- K4 --------------------------------------------------------------------
struct GbKey {
  int CB;                   // count bits of a hash slot (slot = key << CB | count)
  unsigned long long cmask;
};

__device__ __forceinline__ unsigned gb_hash(unsigned long long key) {
  return (unsigned)((key * 0x9E3779B97F4A7C15ull) >> 32);
}

// Insert one event of (file-local fl, second code sc) into an open-addressing
// table; returns the pair's count after this event.
template <bool LDS>
__device__ __forceinline__ unsigned long long gb_insert(unsigned long long* slots, unsigned size,
                                                        bool pow2, unsigned long long key,
                                                        const GbKey& k) {
  unsigned h = gb_hash(key);
  h = pow2 ? (h & (size - 1)) : (h % size);
  const unsigned long long fresh = (key << k.CB) | 1ull;
  while (true) {
    // one CAS claims an empty slot (the common case: a new (file, second)
    // pair) or returns the occupant
    const unsigned long long v = atomicCAS(&slots[h], kEmpty, fresh);
    if (v == kEmpty) return 1;
    if ((v >> k.CB) == key) return (atomicAdd(&slots[h], 1ull) & k.cmask) + 1;
    h = h + 1 == size ? 0 : h + 1;
  }
}

// Per-file LDS state of a bucket (F = 2^L files), after the hash slots.
struct GbFiles {
  unsigned long long* cw;   // count | writes << 32
  unsigned long long* rl;   // reads | local << 32
  unsigned* conc;
  int* prim;
};

__device__ __forceinline__ GbFiles gb_files(unsigned long long* base, int F) {
  GbFiles g;
  g.cw = base;
  g.rl = base + F;
  g.conc = reinterpret_cast<unsigned*>(base + 2 * F);
  g.prim = reinterpret_cast<int*>(g.conc + F);
  return g;
}

// One event: hash insert, concurrency maximum, and the per-file sums added
// once per group of lanes of one file (ballots over the file-local bits), so
// a bucket's few files do not serialise the LDS atomics.
template <bool LDS>
__device__ __forceinline__ void gb_event(bool act, unsigned long long v, const GbPay& p,
                                         const GbKey& k, unsigned long long* slots,
                                         unsigned size, bool pow2, GbFiles& g) {
  const unsigned fl = (unsigned)(v >> p.fshift) & ((1u << p.L) - 1);
  const unsigned long long sc = (v >> p.sshift) & ((1ull << p.sbits) - 1);
  const unsigned oc = (unsigned)(v >> p.cbits) & 3u;
  const int cl = (int)((unsigned)v & ((1u << p.cbits) - 1)) - 1;
  bool loc = false;
  if (act) {
    const unsigned long long cnt =
        gb_insert<LDS>(slots, size, pow2, ((unsigned long long)fl << p.sbits) | sc, k);
    const unsigned c32 = (unsigned)min(cnt, 0xFFFFFFFFull);
    if (c32 > g.conc[fl]) atomicMax(&g.conc[fl], c32);
    const int pr = g.prim[fl];
    loc = cl >= 0 && pr >= 0 && cl == pr;
  }
  unsigned long long peers = __ballot(act);
  for (int b = 0; b < p.L; ++b) {
    const bool bit = (fl >> b) & 1u;
    const unsigned long long bb = __ballot(act && bit);
    peers &= bit ? bb : ~bb;
  }
  const unsigned long long mw = __ballot(act && oc == 1), mr = __ballot(act && oc == 2);
  const unsigned long long ml = __ballot(act && loc);
  const int lane = threadIdx.x & 63;
  if (act && lane == __ffsll((long long)peers) - 1) {
    atomicAdd(&g.cw[fl], (unsigned long long)__popcll(peers) |
                             ((unsigned long long)__popcll(peers & mw) << 32));
    atomicAdd(&g.rl[fl], (unsigned long long)__popcll(peers & mr) |
                             ((unsigned long long)__popcll(peers & ml) << 32));
  }
}

__device__ __forceinline__ void gb_write_files(const GbFiles& g, int nfl, int64_t f0,
                                               long long* __restrict__ out) {
  for (int f = threadIdx.x; f < nfl; f += kGbBThreads) {
    long long* o = out + (f0 + f) * 6;
    const unsigned long long cw = g.cw[f], rl = g.rl[f];
    o[0] = (long long)(cw & 0xFFFFFFFFull);
    o[1] = (long long)(cw >> 32);
    o[2] = (long long)(rl & 0xFFFFFFFFull);
    o[3] = (long long)(rl >> 32);
    o[4] = (long long)(cw & 0xFFFFFFFFull);
    o[5] = (long long)g.conc[f];
  }
}

// Persistent: workgroup w takes buckets w, w + G, w + 2G, ...; the next
// bucket's payloads and primaries are loaded while the current one is hashed
// (a bucket holds ~1k events, so one global round trip per bucket would
// otherwise dominate).  LDS: kGbSlots hash slots, then the per-file state of
// F = 2^L files.
template <typename T>
__global__ __launch_bounds__(kGbBThreads) void gb_bucket(const T* __restrict__ pb,
                                                        const unsigned* __restrict__ bbase,
                                                        int64_t nbuckets, int64_t nf, GbPay p,
                                                        GbKey k,
                                                        const int32_t* __restrict__ primary,
                                                        long long* __restrict__ out,
                                                        int* __restrict__ big_list,
                                                        int* __restrict__ big_count) {
  extern __shared__ unsigned long long lds[];
  const int tid = threadIdx.x;
  const int F = 1 << p.L;
  constexpr int kPrimReg = (1 << kGbMaxL) / kGbBThreads;
  unsigned long long* slots = lds;
  GbFiles g = gb_files(lds + kGbSlots, F);
  const int64_t G = gridDim.x;
  int64_t b = blockIdx.x;
  if (b >= nbuckets) return;
  // bucket b's bounds, payloads (in registers) and primaries
  int64_t s0 = bbase[b], n = (int64_t)bbase[b + 1] - s0;
  T v[kGbReg];
  int pr[kPrimReg];
  auto fetch = [&](int64_t bb, int64_t ss, int64_t nn, T* vv, int* pp) {
    const bool small = nn <= kGbLdsCap;
#pragma unroll
    for (int j = 0; j < kGbReg; ++j) {
      const int64_t i = tid + j * kGbBThreads;
      vv[j] = small && i < nn ? pb[ss + i] : (T)0;
    }
    const int64_t f0 = bb << p.L;
#pragma unroll
    for (int j = 0; j < kPrimReg; ++j) {
      const int64_t f = tid + j * kGbBThreads;
      pp[j] = f < F && f0 + f < nf ? primary[f0 + f] : -2;
    }
  };
  fetch(b, s0, n, v, pr);
  int64_t s0n = 0, nn = 0;
  if (b + G < nbuckets) {
    s0n = bbase[b + G];
    nn = (int64_t)bbase[b + G + 1] - s0n;
  }
  T v2[kGbReg];
  int pr2[kPrimReg];
  // One bucket: cur holds it (its loads are waited for at the empty asm,
  // before the next bucket's loads go out into nxt); ping-pong buffers
  // instead of copies, so no copy of an in-flight register forces a wait.
  auto step = [&](T (&cur)[kGbReg], int (&cpr)[kPrimReg], T (&nxt)[kGbReg],
                  int (&npr)[kPrimReg]) {
#pragma unroll
    for (int j = 0; j < kGbReg; ++j) asm volatile("" : "+v"(cur[j]));
#pragma unroll
    for (int j = 0; j < kPrimReg; ++j) asm volatile("" : "+v"(cpr[j]));
    const int64_t bn = b + G;
    const int64_t f0 = b << p.L;
    const int nfl = (int)min((int64_t)F, nf - f0);
    const bool over = n > kGbLdsCap;
    unsigned size = 64;
    if (!over) {
      while (size < 2 * n && size < kGbSlots) size <<= 1;
      for (unsigned i = tid; i < size; i += kGbBThreads) slots[i] = kEmpty;
#pragma unroll
      for (int j = 0; j < kPrimReg; ++j) {
        const int f = tid + j * kGbBThreads;
        if (f < nfl) {
          g.cw[f] = 0;
          g.rl[f] = 0;
          g.conc[f] = 0;
          g.prim[f] = cpr[j];
        }
      }
    }
    __syncthreads();
    int64_t s0nn = 0, nnn = 0;
    if (bn < nbuckets) {
      fetch(bn, s0n, nn, nxt, npr);
      if (bn + G < nbuckets) {
        s0nn = bbase[bn + G];
        nnn = (int64_t)bbase[bn + G + 1] - s0nn;
      }
    }
    if (over) {
      if (tid == 0) big_list[atomicAdd(big_count, 1)] = (int)b;
    } else {
#pragma unroll
      for (int j = 0; j < kGbReg; ++j) {
        const bool act = tid + j * kGbBThreads < n;
        if (__ballot(act) == 0) break;
        gb_event<true>(act, (unsigned long long)cur[j], p, k, slots, size, true, g);
      }
      __syncthreads();
      gb_write_files(g, nfl, f0, out);
    }
    __syncthreads();  // the LDS is cleared for the next bucket
    s0 = s0n;
    n = nn;
    s0n = s0nn;
    nn = nnn;
    b = bn;
  };
  while (true) {
    step(v, pr, v2, pr2);
    if (b >= nbuckets) break;
    step(v2, pr2, v, pr);
    if (b >= nbuckets) break;
  }
}

// Dense variant (2^(L + sbits) <= 2^kGbDenseBits): the bucket's (file, second)
// grid of u16 counts is the table (two per u32 word; bucket events < 2^16, so
// no count overflows), one non-returning LDS add per event; count / writes /
// reads / local per file are added once per group of lanes of one file
// (ballots, as gb_event), and the concurrency maximum is a max over the file's
// row at the end.  Persistent like gb_bucket.
constexpr int kGbDenseBits = 12;
constexpr int kGbDenseCap = 65535;

template <typename T>
__global__ __launch_bounds__(kGbBThreads) void gb_bucket_dense(
    const T* __restrict__ pb, const unsigned* __restrict__ bbase, int64_t nbuckets, int64_t nf,
    GbPay p, const int32_t* __restrict__ primary, long long* __restrict__ out,
    int* __restrict__ big_list, int* __restrict__ big_count) {
  extern __shared__ unsigned long long lds[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int F = 1 << p.L;
  const int S = 1 << p.sbits;
  const int KW = (F * S + 1) >> 1;  // u32 words of the count grid
  constexpr int kPrimReg = (1 << kGbMaxL) / kGbBThreads;
  GbFiles g = gb_files(lds, F);
  unsigned* grid = reinterpret_cast<unsigned*>(g.prim + F);
  const int64_t G = gridDim.x;
  int64_t b = blockIdx.x;
  if (b >= nbuckets) return;
  const unsigned lmask = (1u << p.L) - 1;
  const unsigned smask = (1u << p.sbits) - 1;
  const unsigned ccmask = (1u << p.cbits) - 1;
  int64_t s0 = bbase[b], n = (int64_t)bbase[b + 1] - s0;
  T v[kGbReg];
  int pr[kPrimReg];
  auto fetch = [&](int64_t bb, int64_t ss, int64_t nn, T* vv, int* pp) {
    const bool ok = nn <= kGbDenseCap;
#pragma unroll
    for (int j = 0; j < kGbReg; ++j) {
      const int64_t i = tid + j * kGbBThreads;
      vv[j] = ok && i < nn ? pb[ss + i] : (T)0;
    }
    const int64_t f0 = bb << p.L;
#pragma unroll
    for (int j = 0; j < kPrimReg; ++j) {
      const int64_t f = tid + j * kGbBThreads;
      pp[j] = f < F && f0 + f < nf ? primary[f0 + f] : -2;
    }
  };
  // the file's sums once per group of lanes of one file (ballots over the
  // file-local bits); fl / oc / loc of this lane's event, act: it holds one
  auto file_sums = [&](bool act, unsigned fl, unsigned oc, bool loc) {
    unsigned long long peers = __ballot(act);
    for (int bt = 0; bt < p.L; ++bt) {
      const bool bit = (fl >> bt) & 1u;
      const unsigned long long bb = __ballot(act && bit);
      peers &= bit ? bb : ~bb;
    }
    const unsigned long long mw = __ballot(act && oc == 1), mr = __ballot(act && oc == 2);
    const unsigned long long ml = __ballot(act && loc);
    if (act && lane == __ffsll((long long)peers) - 1) {
      atomicAdd(&g.cw[fl], (unsigned long long)__popcll(peers) |
                               ((unsigned long long)__popcll(peers & mw) << 32));
      atomicAdd(&g.rl[fl], (unsigned long long)__popcll(peers & mr) |
                               ((unsigned long long)__popcll(peers & ml) << 32));
    }
  };
  // one event's pair count (a non-returning add) and its fields
  auto pair = [&](unsigned long long x, int pf_sel_unused, unsigned& fl, unsigned& oc, int& cl) {
    fl = (unsigned)(x >> p.fshift) & lmask;
    const unsigned sc = (unsigned)(x >> p.sshift) & smask;
    oc = (unsigned)(x >> p.cbits) & 3u;
    cl = (int)((unsigned)x & ccmask) - 1;
    const unsigned key = (fl << p.sbits) | sc;
    atomicAdd(&grid[key >> 1], 1u << ((key & 1u) << 4));
  };
  auto add = [&](bool act, unsigned long long x) {
    unsigned fl = 0, oc = 0;
    int cl = -1;
    if (act) pair(x, 0, fl, oc, cl);
    const int pf = g.prim[fl];
    file_sums(act, fl, oc, act && cl >= 0 && pf >= 0 && cl == pf);
  };
  fetch(b, s0, n, v, pr);
  int64_t s0n = 0, nn = 0;
  if (b + G < nbuckets) {
    s0n = bbase[b + G];
    nn = (int64_t)bbase[b + G + 1] - s0n;
  }
  T v2[kGbReg];
  int pr2[kPrimReg];
  // ping-pong like gb_bucket
  auto step = [&](T (&cur)[kGbReg], int (&cpr)[kPrimReg], T (&nxt)[kGbReg],
                  int (&npr)[kPrimReg]) {
#pragma unroll
    for (int j = 0; j < kGbReg; ++j) asm volatile("" : "+v"(cur[j]));
#pragma unroll
    for (int j = 0; j < kPrimReg; ++j) asm volatile("" : "+v"(cpr[j]));
    const int64_t bn = b + G;
    const int64_t f0 = b << p.L;
    const int nfl = (int)min((int64_t)F, nf - f0);
    const bool over = n > kGbDenseCap;
    if (!over) {
      for (int i = tid; i < KW; i += kGbBThreads) grid[i] = 0;
#pragma unroll
      for (int j = 0; j < kPrimReg; ++j) {
        const int f = tid + j * kGbBThreads;
        if (f < F) {
          g.cw[f] = 0;
          g.rl[f] = 0;
          g.prim[f] = cpr[j];
        }
      }
    }
    __syncthreads();
    // the next bucket's loads fly while this one is counted
    int64_t s0nn = 0, nnn = 0;
    if (bn < nbuckets) {
      fetch(bn, s0n, nn, nxt, npr);
      if (bn + G < nbuckets) {
        s0nn = bbase[bn + G];
        nnn = (int64_t)bbase[bn + G + 1] - s0nn;
      }
    }
    if (over) {
      if (tid == 0) big_list[atomicAdd(big_count, 1)] = (int)b;
    } else {
#pragma unroll
      for (int j = 0; j < kGbReg; ++j) {
        const bool act = tid + j * kGbBThreads < n;
        if (__ballot(act) == 0) break;
        add(act, (unsigned long long)cur[j]);
      }
      for (int64_t i0 = kGbReg * kGbBThreads; i0 < n; i0 += kGbBThreads) {
        const int64_t i = i0 + tid;
        add(i < n, i < n ? (unsigned long long)pb[s0 + i] : 0ull);
      }
      __syncthreads();
      // one wave per file: the maximum count over the file's seconds
      for (int f = wv; f < nfl; f += kGbBThreads / 64) {
        const unsigned* row = grid + (((unsigned)f << p.sbits) >> 1);
        const int words = S >= 2 ? S >> 1 : 1;
        unsigned mx = 0;
        for (int w = lane; w < words; w += 64) {
          const unsigned e = row[w];
          const unsigned lo = S >= 2 ? (e & 0xFFFFu) : ((f & 1) ? (e >> 16) : (e & 0xFFFFu));
          const unsigned hi = S >= 2 ? (e >> 16) : 0u;
          mx = max(mx, max(lo, hi));
        }
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, o));
        if (lane == 0) g.conc[f] = mx;
      }
      __syncthreads();
      gb_write_files(g, nfl, f0, out);
    }
    __syncthreads();  // the grid is cleared for the next bucket
    s0 = s0n;
    n = nn;
    s0n = s0nn;
    nn = nnn;
    b = bn;
  };
  while (true) {
    step(v, pr, v2, pr2);
    if (b >= nbuckets) break;
    step(v2, pr2, v, pr);
    if (b >= nbuckets) break;
  }
}

// Dense variant, one WAVE per bucket (2^L <= 2^kGwMaxL files): each wave of
// the workgroup owns a private LDS slice [u16 grid of F x S counts | per-file
// state] and takes every (grid waves)-th bucket, so no workgroup barrier
// and no end-of-bucket row scan sits between two buckets: the wave clears
// its grid (ds_write_b128), adds each event with a RETURNING u16 add (the
// returned count + 1 is the pair's running count, so the concurrency
// maximum is tracked as it grows; counts of 1 need no atomic since every
// file with an event has concurrency >= 1), sums count / writes / reads /
// local per group of lanes of one file (ballots), and writes the bucket's
// (F, 6) int64 rows as one contiguous run.  LDS instructions of one wave run
// in order, so the clear, the adds and the reads need no barrier.
constexpr int kGwMaxL = 8;
constexpr int kGwWaves = 4;   // waves per workgroup
constexpr int kGwUnroll = 8;  // payload loads in flight per lane

__host__ __device__ inline int gw_grid_words(int L, int sbits) {
  return ((((1 << (L + sbits)) + 1) >> 1) + 3) & ~3;  // u32 words, multiple of 4
}
__host__ __device__ inline int gw_wave_bytes(int L, int sbits) {
  return (4 * gw_grid_words(L, sbits) + 24 * (1 << L) + 15) & ~15;  // 16-byte aligned slices
}

template <typename T>
__global__ __launch_bounds__(64 * kGwWaves) void gb_bucket_wave(
    const T* __restrict__ pb, const unsigned* __restrict__ bbase, int64_t nbuckets, int64_t nf,
    GbPay p, const int32_t* __restrict__ primary, long long* __restrict__ out,
    int* __restrict__ big_list, int* __restrict__ big_count) {
  extern __shared__ unsigned long long lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int F = 1 << p.L;
  const int KW = gw_grid_words(p.L, p.sbits);
  unsigned char* mine =
      reinterpret_cast<unsigned char*>(lds) + (size_t)wv * gw_wave_bytes(p.L, p.sbits);
  unsigned* grid = reinterpret_cast<unsigned*>(mine);
  GbFiles g = gb_files(reinterpret_cast<unsigned long long*>(mine + 4 * KW), F);
  const unsigned lmask = (1u << p.L) - 1;
  const unsigned smask = (1u << p.sbits) - 1;
  const unsigned ccmask = (1u << p.cbits) - 1;
  // buckets strided over the waves of the grid (a dynamic atomic counter
  // here miscompiled into a loop that never exits)
  const int64_t nw = (int64_t)gridDim.x * kGwWaves;
  for (int64_t b = (int64_t)blockIdx.x * kGwWaves + wv; b < nbuckets; b += nw) {
    const int b32 = (int)b;
    const int64_t s0 = bbase[b], n = (int64_t)bbase[b + 1] - s0;
    if (n > kGbDenseCap) {
      if (lane == 0) big_list[atomicAdd(big_count, 1)] = b32;
    } else {
      const int64_t f0 = b << p.L;
      const int nfl = (int)min((int64_t)F, nf - f0);
      // the first payloads go out before the clear
      T v[kGwUnroll];
  #pragma unroll
      for (int u = 0; u < kGwUnroll; ++u) {
        const int64_t i = u * 64 + lane;
        v[u] = i < n ? pb[s0 + i] : (T)0;
      }
      const uint4 z = {0u, 0u, 0u, 0u};
      for (int i = lane * 4; i < KW; i += 256) *reinterpret_cast<uint4*>(grid + i) = z;
      for (int f = lane; f < F; f += 64) {
        g.cw[f] = 0;
        g.rl[f] = 0;
        g.conc[f] = 0;
        g.prim[f] = f < nfl ? primary[f0 + f] : -2;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int64_t i0 = 0; i0 < n; i0 += 64 * kGwUnroll) {
        if (i0 > 0) {
  #pragma unroll
          for (int u = 0; u < kGwUnroll; ++u) {
            const int64_t i = i0 + u * 64 + lane;
            v[u] = i < n ? pb[s0 + i] : (T)0;
          }
        }
  #pragma unroll
        for (int u = 0; u < kGwUnroll; ++u) {
          const bool act = i0 + u * 64 + lane < n;
          if (__ballot(act) == 0) break;
          const unsigned long long x = (unsigned long long)v[u];
          unsigned fl = 0, oc = 0;
          bool loc = false;
          if (act) {
            fl = (unsigned)(x >> p.fshift) & lmask;
            const unsigned sc = (unsigned)(x >> p.sshift) & smask;
            oc = (unsigned)(x >> p.cbits) & 3u;
            const int cl = (int)((unsigned)x & ccmask) - 1;
            const unsigned key = (fl << p.sbits) | sc;
            const unsigned sh = (key & 1u) << 4;
            const unsigned old = atomicAdd(&grid[key >> 1], 1u << sh);
            const unsigned cnt = ((old >> sh) & 0xFFFFu) + 1u;
            if (cnt > 1u && cnt > g.conc[fl]) atomicMax(&g.conc[fl], cnt);
            const int pf = g.prim[fl];
            loc = cl >= 0 && pf >= 0 && cl == pf;
          }
          unsigned long long peers = __ballot(act);
          for (int bt = 0; bt < p.L; ++bt) {
            const bool bit = (fl >> bt) & 1u;
            const unsigned long long bb = __ballot(act && bit);
            peers &= bit ? bb : ~bb;
          }
          const unsigned long long mw = __ballot(act && oc == 1), mr = __ballot(act && oc == 2);
          const unsigned long long ml = __ballot(act && loc);
          if (act && lane == __ffsll((long long)peers) - 1) {
            atomicAdd(&g.cw[fl], (unsigned long long)__popcll(peers) |
                                     ((unsigned long long)__popcll(peers & mw) << 32));
            atomicAdd(&g.rl[fl], (unsigned long long)__popcll(peers & mr) |
                                     ((unsigned long long)__popcll(peers & ml) << 32));
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // rows f0 .. f0 + nfl, six fields each: one contiguous run of the output
      long long* o = out + f0 * 6;
      for (int t = lane; t < 6 * nfl; t += 64) {
        const int f = t / 6, fld = t - 6 * f;
        const unsigned long long cw = g.cw[f], rl = g.rl[f];
        const long long cntf = (long long)(cw & 0xFFFFFFFFull);
        long long val;
        switch (fld) {
          case 0: val = cntf; break;
          case 1: val = (long long)(cw >> 32); break;
          case 2: val = (long long)(rl & 0xFFFFFFFFull); break;
          case 3: val = (long long)(rl >> 32); break;
          case 4: val = cntf; break;
          default: val = cntf > 0 ? (long long)max(g.conc[f], 1u) : 0; break;
        }
        o[t] = val;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// The same for buckets of at most 4 files (L <= 2, config 4's shape): the
// per-file count / writes / reads / local and the concurrency maximum are
// kept in each lane's registers (select by the event's file, no ballots and
// no per-file LDS atomics), the payload is decoded with 32-bit field
// extracts, and the bucket's rows come from one wave reduction per value at
// the end.  The (file, second) counts stay in the wave's LDS grid.  The
// ballot kernel above spent ~165 instructions per 64 events here.
template <typename T>
__global__ __launch_bounds__(64 * kGwWaves) void gb_bucket_wave4(
    const T* __restrict__ pb, const unsigned* __restrict__ bbase, int64_t nbuckets, int64_t nf,
    GbPay p, const int32_t* __restrict__ primary, long long* __restrict__ out,
    int* __restrict__ big_list, int* __restrict__ big_count) {
  extern __shared__ unsigned long long lds[];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int KW = gw_grid_words(p.L, p.sbits);
  unsigned* grid = reinterpret_cast<unsigned*>(reinterpret_cast<unsigned char*>(lds) +
                                               (size_t)wv * gw_wave_bytes(p.L, p.sbits));
  const int F = 1 << p.L;
  const int sb = p.sbits;
  const int nw = gridDim.x * kGwWaves;
  for (int b = blockIdx.x * kGwWaves + wv; b < nbuckets; b += nw) {
    const int s0 = (int)bbase[b];
    const int n = (int)bbase[b + 1] - s0;
    if (n > kGbDenseCap) {
      if (lane == 0) big_list[atomicAdd(big_count, 1)] = b;
      continue;
    }
    const int64_t f0 = (int64_t)b << p.L;
    const int nfl = (int)min((int64_t)F, nf - f0);
    T v[kGwUnroll];
#pragma unroll
    for (int u = 0; u < kGwUnroll; ++u) {
      const int i = u * 64 + lane;
      v[u] = i < n ? pb[s0 + i] : (T)0;
    }
    const int pl = lane < nfl ? primary[f0 + lane] : -2;
    const uint4 z = {0u, 0u, 0u, 0u};
    for (int i = lane * 4; i < KW; i += 256) *reinterpret_cast<uint4*>(grid + i) = z;
    // the bucket's primaries (client code = client + 1; -1: none)
    int pc[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) pc[f] = __builtin_amdgcn_readlane(pl, f) + 1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    unsigned A[4] = {0u, 0u, 0u, 0u}, B[4] = {0u, 0u, 0u, 0u}, M[4] = {0u, 0u, 0u, 0u};
    for (int i0 = 0; i0 < n; i0 += 64 * kGwUnroll) {
      if (i0 > 0) {
#pragma unroll
        for (int u = 0; u < kGwUnroll; ++u) {
          const int i = i0 + u * 64 + lane;
          v[u] = i < n ? pb[s0 + i] : (T)0;
        }
      }
#pragma unroll
      for (int u = 0; u < kGwUnroll; ++u) {
        if (i0 + u * 64 >= n) break;  // wave-uniform
        if (i0 + u * 64 + lane < n) {
          const unsigned long long x = (unsigned long long)v[u];
          const unsigned lo = (unsigned)x;  // op, client and (4-byte payloads) all fields
          const unsigned fl = (unsigned)(x >> p.fshift) & (unsigned)(F - 1);
          const unsigned sc = (unsigned)(x >> p.sshift) & ((1u << sb) - 1u);
          const unsigned oc = __builtin_amdgcn_ubfe(lo, p.cbits, 2);
          const int cc = (int)__builtin_amdgcn_ubfe(lo, 0, p.cbits);
          const unsigned key = (fl << sb) | sc;
          const unsigned sh = (key & 1u) << 4;
          const unsigned old = atomicAdd(&grid[key >> 1], 1u << sh);
          const unsigned cnt = __builtin_amdgcn_ubfe(old, sh, 16) + 1u;
          const int pf = fl == 0 ? pc[0] : fl == 1 ? pc[1] : fl == 2 ? pc[2] : pc[3];
          const unsigned loc = (cc != 0 && pf > 0 && cc == pf) ? 1u : 0u;
          const unsigned va = 1u | ((oc == 1u) ? 0x10000u : 0u);
          const unsigned vb = ((oc == 2u) ? 1u : 0u) | (loc << 16);
#pragma unroll
          for (int f = 0; f < 4; ++f) {
            const bool m = fl == (unsigned)f;
            A[f] += m ? va : 0u;
            B[f] += m ? vb : 0u;
            M[f] = max(M[f], m ? cnt : 0u);
          }
        }
      }
    }
    // wave sums / maxima of the lanes' per-file values by halving exchanges:
    // at each xor step a lane keeps half of its values and adds the
    // partner's copy of that half (sums: A0..3 B0..3 over xor 32, 16, 8 ->
    // lane bits 5..3 name the value, then xor 4, 2, 1; maxima: M0..3 over
    // xor 32, 16 -> lane bits 5..4, then xor 8..1): 17 exchanges instead of
    // 72 (3 values x 4 files x 6 levels)
    const int h5 = (lane >> 5) & 1, h4 = (lane >> 4) & 1, h3 = (lane >> 3) & 1;
    unsigned s4[4], s2[2], s1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned send = h5 ? A[i] : B[i];
      s4[i] = (h5 ? B[i] : A[i]) + (unsigned)__shfl_xor((int)send, 32);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const unsigned send = h4 ? s4[i] : s4[2 + i];
      s2[i] = (h4 ? s4[2 + i] : s4[i]) + (unsigned)__shfl_xor((int)send, 16);
    }
    {
      const unsigned send = h3 ? s2[0] : s2[1];
      s1 = (h3 ? s2[1] : s2[0]) + (unsigned)__shfl_xor((int)send, 8);
    }
    for (int o = 4; o > 0; o >>= 1) s1 += (unsigned)__shfl_xor((int)s1, o);
    unsigned m2[2], m1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const unsigned send = h5 ? M[i] : M[2 + i];
      m2[i] = max(h5 ? M[2 + i] : M[i], (unsigned)__shfl_xor((int)send, 32));
    }
    {
      const unsigned send = h4 ? m2[0] : m2[1];
      m1 = max(h4 ? m2[1] : m2[0], (unsigned)__shfl_xor((int)send, 16));
    }
    for (int o = 8; o > 0; o >>= 1) m1 = max(m1, (unsigned)__shfl_xor((int)m1, o));
    // lane 8 f holds A[f], lane 32 + 8 f B[f], lane 16 f M[f]
    const int fo = lane / 6;
    const unsigned a_f = (unsigned)__shfl((int)s1, (8 * fo) & 63);
    const unsigned b_f = (unsigned)__shfl((int)s1, (32 + 8 * fo) & 63);
    const unsigned m_f = (unsigned)__shfl((int)m1, (16 * fo) & 63);
    // rows f0 .. f0 + nfl, six fields each: one contiguous run of the output
    long long* o = out + f0 * 6;
    if (lane < 6 * nfl) {
      const int f = fo, fld = lane - 6 * f;
      const unsigned a = a_f;
      const unsigned bb = b_f;
      const unsigned mm = m_f;
      long long val;
      switch (fld) {
        case 0: val = a & 0xFFFFu; break;
        case 1: val = a >> 16; break;
        case 2: val = bb & 0xFFFFu; break;
        case 3: val = bb >> 16; break;
        case 4: val = a & 0xFFFFu; break;
        default: val = mm; break;
      }
      o[lane] = val;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// Buckets over the LDS capacity: the hash lives in global memory (2 n slots
// from gslots + 2 * s0, so buckets never overlap).
template <typename T>
__global__ __launch_bounds__(kGbBThreads) void gb_bucket_big(
    const T* __restrict__ pb, const unsigned* __restrict__ bbase, const int* __restrict__ list,
    int64_t nf, GbPay p, GbKey k, const int32_t* __restrict__ primary,
    unsigned long long* __restrict__ gslots, long long* __restrict__ out) {
  extern __shared__ unsigned long long lds[];
  const int64_t b = list[blockIdx.x];
  const int tid = threadIdx.x;
  const int64_t s0 = bbase[b], n = (int64_t)bbase[b + 1] - s0;
  const int F = 1 << p.L;
  const int64_t f0 = b << p.L;
  const int nfl = (int)min((int64_t)F, nf - f0);
  unsigned long long* slots = gslots + 2 * s0;
  const unsigned size = (unsigned)(2 * n);
  GbFiles g = gb_files(lds, F);
  for (unsigned i = tid; i < size; i += kGbBThreads) slots[i] = kEmpty;
  for (int f = tid; f < nfl; f += kGbBThreads) {
    g.cw[f] = 0;
    g.rl[f] = 0;
    g.conc[f] = 0;
    g.prim[f] = primary[f0 + f];
  }
  __syncthreads();
  for (int64_t i0 = 0; i0 < n; i0 += kGbBThreads) {
    const int64_t i = i0 + tid;
    const bool act = i < n;
    gb_event<false>(act, act ? (unsigned long long)pb[s0 + i] : 0ull, p, k, slots, size, false,
                    g);
  }
  __syncthreads();
  gb_write_files(g, nfl, f0, out);
}

// forget the profile triple of a step that returns before its last event
void prof_drop(Ctx& c) {
  if (c.prof_cur >= 0) {
    c.prof_used -= 4;
    c.prof_cur = -1;
  }
}

int bitlen(unsigned long long v) {  // bits to hold v (0 -> 0)
  int b = 0;
  while (b < 64 && (v >> b) != 0) ++b;
  return b;
}

template <typename T>
void gb_run(Ctx& c, int64_t ne, int64_t nf, int fbits, int L, int B1, int B2, int B3, bool dense,
            GbPay p, int64_t T1, int64_t* out, const long long* res) {
  const int R1 = 1 << B1, R2 = 1 << B2;
  const int shift1 = fbits - B1;
  const int64_t nb = ceil_div(nf, (int64_t)1 << L);
  const int64_t nvalid = res[4];
  T* p1 = c.gb_p1.as<T>();
  unsigned* binbase = c.gb_small.as<unsigned>();
  int* tile2start = reinterpret_cast<int*>(binbase + kGbMaxBins + 1);
  unsigned* tilepref = c.gb_tilepref.as<unsigned>();
  unsigned* chunkbase = c.gb_chunk.as<unsigned>();
  const int64_t per1 = ceil_div(T1, 8);
  if (nvalid > 0) {
    hipLaunchKernelGGL(gb_scatter1<T>, dim3(8 * per1), dim3(kGbThreads), 0, c.stream,
                       c.ev_file.as<int32_t>(), c.ev_op.as<uint8_t>(), c.ev_client.as<int32_t>(),
                       c.ev_ts.as<long long>(), ne, nf, p, shift1, R1, T1, per1, tilepref,
                       chunkbase, p1);
    HIP_CHECK(hipGetLastError());
  }
  const T* pb = p1;
  unsigned* bbase = binbase;  // one pass: the buckets are the pass-1 digits
  if (B2 > 0) {
    const int64_t T2 = res[3];
    bbase = c.gb_bbase.as<unsigned>();
    c.gb_hist2.ensure(sizeof(unsigned) * (size_t)std::max<int64_t>(T2, 1) * R2);
    unsigned* hist2 = c.gb_hist2.as<unsigned>();
    const int shift2 = p.fshift + L + B3;
    if (T2 > 0)
      hipLaunchKernelGGL(gb_hist2<T>, dim3(T2), dim3(kGbThreads), 0, c.stream, p1, binbase,
                         tile2start, R1, R2, shift2, hist2);
    hipLaunchKernelGGL(gb_scan2, dim3(R1), dim3(kGbMaxBins), 0, c.stream, hist2, tile2start,
                       binbase, R1, R2, bbase);
    HIP_CHECK(hipGetLastError());
    if (T2 > 0) {
      const int64_t per2 = ceil_div(T2, 8);
      hipLaunchKernelGGL(gb_scatter2<T>, dim3(8 * per2), dim3(kGbThreads), 0, c.stream, p1,
                         binbase, tile2start, R1, R2, shift2, T2, per2, hist2, bbase,
                         c.gb_p2.as<T>());
      HIP_CHECK(hipGetLastError());
    }
    pb = c.gb_p2.as<T>();
  }
  if (B3 > 0) {
    // pass 3 within each of the R1 R2 pass-2 regions (the same kernels: its
    // regions take the place of pass 1's digits); output into p1's buffer
    const int R12 = R1 * R2, R3 = 1 << B3;
    const int shift3 = p.fshift + L;
    const int g3 = (R12 + kGbT3Per - 1) / kGbT3Per;
    c.gb_t3.ensure(sizeof(int) * ((size_t)R12 + 1 + g3) + 64);
    int* tstart3 = c.gb_t3.as<int>();
    unsigned* wsum3 = reinterpret_cast<unsigned*>(tstart3 + R12 + 1);  // (after the starts)
    long long* tot3 = reinterpret_cast<long long*>(c.gb_res.as<long long>() + 6);
    hipLaunchKernelGGL(gb_tilecount3, dim3(g3), dim3(kGbT3Per), 0, c.stream, bbase, R12, wsum3);
    hipLaunchKernelGGL(gb_tilestart3, dim3(g3), dim3(kGbT3Per), 0, c.stream, bbase, R12, wsum3,
                       tstart3, tot3);
    HIP_CHECK(hipGetLastError());
    long long T3 = 0;
    HIP_CHECK(hipMemcpyAsync(&T3, tot3, sizeof(T3), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    c.gb_hist2.ensure(sizeof(unsigned) * (size_t)std::max<long long>(T3, 1) * R3);
    unsigned* hist3 = c.gb_hist2.as<unsigned>();
    c.gb_bbase3.ensure(sizeof(unsigned) * ((size_t)R12 * R3 + 1) + 64);
    unsigned* bbase3 = c.gb_bbase3.as<unsigned>();
    if (T3 > 0)
      hipLaunchKernelGGL(gb_hist2<T>, dim3((unsigned)T3), dim3(kGbThreads), 0, c.stream, pb, bbase,
                         tstart3, R12, R3, shift3, hist3);
    if (R3 <= kGbScan3Max)
      hipLaunchKernelGGL(gb_scan3, dim3((R12 + 255) / 256), dim3(256), 0, c.stream, hist3, tstart3,
                         bbase, R12, R3, bbase3);
    else
      hipLaunchKernelGGL(gb_scan2, dim3(R12), dim3(kGbMaxBins), 0, c.stream, hist3, tstart3, bbase,
                         R12, R3, bbase3);
    HIP_CHECK(hipGetLastError());
    if (T3 > 0) {
      const int64_t per3 = ceil_div((int64_t)T3, 8);
      hipLaunchKernelGGL(gb_scatter2<T>, dim3(8 * per3), dim3(kGbThreads), 0, c.stream, pb, bbase,
                         tstart3, R12, R3, shift3, (int64_t)T3, per3, hist3, bbase3, p1);
      HIP_CHECK(hipGetLastError());
    }
    pb = p1;
    bbase = bbase3;
  }
  prof_mark(c, 1);  // partition done
  GbKey k;
  k.CB = 64 - (L + p.sbits);
  k.cmask = k.CB >= 64 ? ~0ull : ((1ull << k.CB) - 1);
  int* big = reinterpret_cast<int*>(tile2start + kGbMaxBins + 1);  // count, then the list
  HIP_CHECK(hipMemsetAsync(big, 0, 4, c.stream));
  c.gb_list.ensure(sizeof(int) * (size_t)std::max<int64_t>(nb, 1));
  const size_t files_lds = (size_t)24 << L;
  // persistent grids: exactly the workgroups that stay resident together (a
  // second round of late workgroups would double the tail)
  const size_t lds_b = dense ? files_lds + ((size_t)4 << std::max(0, L + p.sbits - 1)) + 16
                             : 8 * kGbSlots + files_lds;
  const bool wave = dense && L <= kGwMaxL && !getenv("CDR_GB_BLOCK");
  int per_cu = 0;
  if (wave) {
    const size_t lds_w = (size_t)kGwWaves * gw_wave_bytes(L, p.sbits);
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, reinterpret_cast<const void*>(gb_bucket_wave<T>), 64 * kGwWaves, lds_w));
    per_cu = std::max(1, per_cu);
    const int64_t wgrid = std::min<int64_t>(ceil_div(nb, (int64_t)kGwWaves),
                                            (int64_t)lloyd_num_cus(c.device) * per_cu);
    c.gb_last_grid = wgrid;
    if (L <= 2 && !getenv("CDR_GB_BALLOT"))
      hipLaunchKernelGGL(gb_bucket_wave4<T>, dim3(wgrid), dim3(64 * kGwWaves), lds_w, c.stream,
                         pb, bbase, nb, nf, p, c.ev_primary.as<int32_t>(),
                         c.ev_out.as<long long>(), c.gb_list.as<int>(), big);
    else
      hipLaunchKernelGGL(gb_bucket_wave<T>, dim3(wgrid), dim3(64 * kGwWaves), lds_w, c.stream,
                         pb, bbase, nb, nf, p, c.ev_primary.as<int32_t>(),
                         c.ev_out.as<long long>(), c.gb_list.as<int>(), big);
  } else {
    if (dense)
      HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, reinterpret_cast<const void*>(gb_bucket_dense<T>), kGbBThreads, lds_b));
    else
      HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, reinterpret_cast<const void*>(gb_bucket<T>), kGbBThreads, lds_b));
    per_cu = std::max(1, per_cu);
    const int64_t gb_grid = std::min<int64_t>(nb, (int64_t)lloyd_num_cus(c.device) * per_cu);
    c.gb_last_grid = gb_grid;
    if (dense)
      hipLaunchKernelGGL(gb_bucket_dense<T>, dim3(gb_grid), dim3(kGbBThreads), lds_b, c.stream,
                         pb, bbase, nb, nf, p, c.ev_primary.as<int32_t>(),
                         c.ev_out.as<long long>(), c.gb_list.as<int>(), big);
    else
      hipLaunchKernelGGL(gb_bucket<T>, dim3(gb_grid), dim3(kGbBThreads), lds_b, c.stream, pb,
                         bbase, nb, nf, p, k, c.ev_primary.as<int32_t>(),
                         c.ev_out.as<long long>(), c.gb_list.as<int>(), big);
  }
  HIP_CHECK(hipGetLastError());
  prof_mark(c, 2);
  int nbig = 0;
  HIP_CHECK(hipMemcpyAsync(&nbig, big, 4, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  if (nbig > 0) {
    c.gb_slots.ensure(sizeof(unsigned long long) * 2 * (size_t)std::max<int64_t>(nvalid, 1));
    hipLaunchKernelGGL(gb_bucket_big<T>, dim3(nbig), dim3(kGbBThreads), files_lds, c.stream, pb,
                       bbase, c.gb_list.as<int>(), nf, p, k, c.ev_primary.as<int32_t>(),
                       c.gb_slots.as<unsigned long long>(), c.ev_out.as<long long>());
    HIP_CHECK(hipGetLastError());
    prof_mark(c, 2);
  }
  c.gb_last_big = nbig;
  if (out)
    HIP_CHECK(hipMemcpyAsync(out, c.ev_out.p, 8 * 6 * nf, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
}

}  // namespace

// The resident events' timestamp range, computed once by their producer (the
// group-by's partition then reads 4 B per event in its histogram pass
// instead of 12).  Every writer of c.ev_ts calls this or clears
// c.ev_tsr_valid.
void events_ts_range(Ctx& c, int64_t ne) {
  c.ev_tsr.ensure(sizeof(long long) * 4);
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(2048, ceil_div(ne, 256 * 16)));
  c.gb_part.ensure(sizeof(long long) * 3 * (size_t)nb + 64);
  hipLaunchKernelGGL(gb_tsr_part, dim3(nb), dim3(256), 0, c.stream, c.ev_ts.as<long long>(), ne,
                     c.gb_part.as<long long>());
  hipLaunchKernelGGL(gb_tsr_fin, dim3(1), dim3(64), 0, c.stream, c.gb_part.as<long long>(), nb,
                     c.ev_tsr.as<long long>());
  HIP_CHECK(hipGetLastError());
  c.ev_tsr_valid = true;
  c.ev_tsr_n = ne;
}

// The group-by of the events resident in c.ev_* (features_aggregate_resident's
// hand-written path).  Returns false (nothing computed) when the shape is
// outside what the packed payload and bucket tables can hold; the caller then
// takes the sort-based path.
//
// Layout: fbits = bits of the file id; the top B1 = min(9, fbits) bits are the
// pass-1 digit; the remaining rem bits split into the pass-2 digit (B2 <= 9)
// and the file-local bits L (2^L files per bucket), chosen once the second
// range is known: the dense (file, second) grid when 2^(L + sbits) <= 4096,
// else the hash with about 1024 events per bucket.
bool groupby_resident(Ctx& c, int64_t ne, int64_t nf, int64_t* out, int64_t* max_ts) {
  c.gb_last_hand = 0;
  if (nf < 1 || ne < 0 || ne >= (1ll << 31) || nf >= (1ll << 31)) return false;
  if (getenv("CDR_GROUPBY_SORT")) return false;  // the sort-based path, for comparisons
  const int cmax = c.ev_cmax;
  const int cbits = std::max(1, bitlen((unsigned long long)std::max(cmax, 0) + 1));
  const int fbits = bitlen((unsigned long long)(nf - 1));
  const int B1 = std::min(kGbMaxDigit, fbits);
  const int rem = fbits - B1;
  const int Lmin = std::max(0, rem - kGbMaxDigit), Lmax = std::min(rem, kGbMaxL);
  if (Lmin > Lmax) return false;
  const int R1 = 1 << B1;
  const int64_t T1 = std::max<int64_t>(1, ceil_div(ne, kGbTile));
  const int64_t C = ceil_div(T1, kGbChunkTiles);
  // K1 + S1
  c.gb_tilepref.ensure(sizeof(unsigned) * (size_t)T1 * R1);
  c.gb_chunk.ensure(sizeof(unsigned) * (size_t)C * R1);
  c.gb_part.ensure(sizeof(long long) * 3 * (size_t)C + 64);
  c.gb_small.ensure(sizeof(int) * (3 * (kGbMaxBins + 1) + 8));
  c.gb_res.ensure(sizeof(long long) * 8);  // (res[6]: pass 3's tile total)
  c.gb_bbase.ensure(sizeof(unsigned) * ((size_t)R1 << kGbMaxDigit) + 64);
  const size_t ne1 = ne > 0 ? (size_t)ne : 1;
  c.ev_out.ensure(8 * 6 * (size_t)nf + 64);
  // profiling: events 0 (start), 1 (partition done), 2 (buckets done)
  prof_step_begin(c);
  prof_mark(c, 0);
  // the producer's timestamp range, when it computed one for these events
  const bool tsr = c.ev_tsr_valid && c.ev_tsr_n == ne && !exp_env("CDR_GB_TSRANGE");
  hipLaunchKernelGGL(tsr ? gb_hist1<false> : gb_hist1<true>, dim3(C), dim3(kGbThreads), 0,
                     c.stream, c.ev_file.as<int32_t>(), c.ev_ts.as<long long>(), ne, nf,
                     fbits - B1, R1, c.gb_tilepref.as<unsigned>(), c.gb_chunk.as<unsigned>(),
                     c.gb_part.as<long long>());
  HIP_CHECK(hipGetLastError());
  unsigned* binbase = c.gb_small.as<unsigned>();
  int* tile2start = reinterpret_cast<int*>(binbase + kGbMaxBins + 1);
  const int64_t G = ceil_div(C, kGbRange);
  c.gb_rsum.ensure(sizeof(unsigned) * (size_t)G * R1);
  hipLaunchKernelGGL(gb_scan1a, dim3(G), dim3(kGbMaxBins), 0, c.stream, c.gb_chunk.as<unsigned>(),
                     C, R1, c.gb_rsum.as<unsigned>());
  hipLaunchKernelGGL(gb_scan1b, dim3(1), dim3(kGbMaxBins), 0, c.stream, c.gb_rsum.as<unsigned>(),
                     G, R1, c.gb_part.as<long long>(), C, binbase, tile2start,
                     c.gb_res.as<long long>(), tsr ? c.ev_tsr.as<long long>() : nullptr);
  hipLaunchKernelGGL(gb_scan1c, dim3(G), dim3(kGbMaxBins), 0, c.stream, c.gb_chunk.as<unsigned>(),
                     C, R1, c.gb_rsum.as<unsigned>(), binbase);
  HIP_CHECK(hipGetLastError());
  long long res[5];
  HIP_CHECK(hipMemcpyAsync(res, c.gb_res.p, sizeof(res), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  // payload layout from the timestamp range
  *max_ts = LLONG_MIN;
  long long sec_min = 0, sec_max = 0;
  if (ne > 0 && res[0] <= res[1]) {
    *max_ts = res[1];
    sec_min = (long long)std::floor((double)res[0] / 1000000.0);
    sec_max = (long long)std::floor((double)res[1] / 1000000.0);
  }
  if (sec_max - sec_min >= (1ll << 40)) {
    prof_drop(c);
    return false;
  }
  const int sbits = std::max(1, bitlen((unsigned long long)(sec_max - sec_min) + 1));
  const double a = (double)std::max<int64_t>(res[4], 1) / (double)nf;  // events per file
  // the bucket shape from the smallest file-local width the passes allow
  auto shape = [&](int lmin, bool& dn) -> int {
    dn = sbits + lmin <= kGbDenseBits && !exp_env("CDR_GB_HASH");
    if (dn) {
      const int Lt = (int)std::floor(std::log2(2048.0 / a));
      return std::max(lmin, std::min({Lt, Lmax, kGbDenseBits - sbits}));
    }
    const int Lt = (int)std::floor(std::log2(1024.0 / a));
    return std::max(lmin, std::min(Lt, Lmax));
  };
  bool dense;
  int L = shape(Lmin, dense);
  int B2 = rem - L, B3 = 0;
  // Two passes leave buckets over the LDS tables (about 3 million files and
  // more: the one-GPU 1B-event log's 5.95M files gave 32-file buckets of ~5400
  // events, every one through the global-memory hash): a third pass
  // (9 + 9 + B3 bits) brings the buckets back to the LDS shapes.
  // (CDR_GB_PASS3=1, tests: the third pass whenever the file bits allow it)
  const bool force3 = getenv("CDR_GB_PASS3") != nullptr;
  if (rem > kGbMaxDigit && (a * std::ldexp(1.0, L) > 0.5 * kGbLdsCap || force3)) {
    bool dn3;
    const int lmin3 = std::max(0, rem - 2 * kGbMaxDigit);
    int L3 = shape(lmin3, dn3);
    if (force3) L3 = std::max(lmin3, std::min(L3, rem - kGbMaxDigit - 1));
    if (rem - kGbMaxDigit - L3 >= 1 && L3 < L) {
      L = L3;
      dense = dn3;
      B2 = kGbMaxDigit;
      B3 = rem - kGbMaxDigit - L;
    }
  }
  if (!dense && L + sbits > 40) {  // hash key + count in 64 bits
    prof_drop(c);
    return false;
  }
  GbPay p;
  p.cbits = cbits;
  p.sshift = 2 + cbits;
  p.sbits = sbits;
  p.fshift = p.sshift + sbits;
  p.L = L;
  p.sec_min = sec_min;
  const int lowbits = fbits - B1;
  p.low_mask = lowbits >= 64 ? ~0ull : ((1ull << lowbits) - 1);
  const int pbits = p.fshift + lowbits;
  if (pbits > 64) {
    prof_drop(c);
    return false;
  }
  // pass-2 tiles per digit were counted by S1 for the same tile size
  c.gb_last_hand = 1;
  c.gb_last_L = L;
  c.gb_last_passes = B3 > 0 ? 3 : (B2 > 0 ? 2 : 1);
  c.gb_last_pbytes = pbits <= 32 ? 4 : 8;
  c.gb_last_dense = dense ? 1 : 0;
  const size_t pay = pbits <= 32 ? 4 : 8;
  c.gb_p1.ensure(pay * ne1);
  if (B2 > 0) c.gb_p2.ensure(pay * ne1);
  if (pbits <= 32)
    gb_run<unsigned>(c, ne, nf, fbits, L, B1, B2, B3, dense, p, T1, out, res);
  else
    gb_run<unsigned long long>(c, ne, nf, fbits, L, B1, B2, B3, dense, p, T1, out, res);
  return true;
}

}  // namespace cdr
