// ingest.hip — access-log CSV ingest on the device.
//
// Replaces the host tokeniser in front of the group-by: the reference reads the
// header-less log `ts,path,op,client_node,pid` (src/access_simulator.py:61-63)
// with spark.read.csv + to_timestamp (src/compute_features.py:19-29) and joins
// `path` against the manifest (:37-41).  The build's host restatement of that
// read is compute_features.load_access_log + encode (python csv.reader, the
// ISO regex of parse_ts_us); this file produces the same encoded events,
// directly into the resident event buffers of features.hip (c.ev_*), so
// cdr_features_aggregate_resident runs next without a host round trip.
//
// Pipeline (all byte work, HBM-bound, no MFMA):
//   K8a  nl_count   one uint4 per lane, 4 KiB tiles: count record terminators
//   K8b  exclusive scan of the tile counts (tile_scan_part / _mid / _out,
//        4096 counts per workgroup) + tile_total (tail record)
//   K8c  nl_write   K8a's per-lane masks (2 B per 16 log bytes), workgroup scan,
//                   write each record's end index
//   K8d  parse      64 records per workgroup (one wave; measured best of
//                   64/128/256 records and 5/6/8 KiB stages): their span is staged
//                   into LDS with coalesced 16-byte loads, then one lane per
//                   record splits fields, parses the timestamp, and looks the
//                   path / client up in device hash tables of the manifest.
// Dictionary build (once per manifest): tab_insert (64-bit CAS, first row
// wins via atomicMin, like dict.setdefault) + tab_verify (a distinct string
// with an equal 64-bit hash is reported, never merged silently).
//
// Record semantics (python csv.reader, default dialect, on unquoted input):
//   * records end at '\n'; a '\r' right before it is dropped; a line that is
//     empty (or only "\r") yields no record (csv gives [] and load_access_log
//     skips it); a last line without '\n' is still a record;
//   * fields split at ','; missing fields are empty; an empty field is None:
//     ts -> error, path -> -1 (no manifest row), op -> 0, client -> -1;
//   * a '"', a NUL byte, a '\r' elsewhere, or a non-ASCII byte in the ts
//     field is "unsupported": csv quoting / csv errors / Unicode digits are
//     left to the host tokeniser (the caller is told, nothing is guessed).
// Timestamps follow parse_ts_us (the regex in compute_features.py): greedy
// digit groups are the regex's only possible match, so a left-to-right scan
// decides it exactly.
#include <climits>
#include <cstring>

#include "cdr_internal.h"

namespace cdr {

namespace {

constexpr int kTile = 4096;       // bytes per K8a/K8c workgroup (256 lanes x 16)
#ifndef CDR_ING_REC
#define CDR_ING_REC 64
#endif
#ifndef CDR_ING_STAGE
#define CDR_ING_STAGE 6144
#endif
constexpr int kRecPerWG = CDR_ING_REC;  // records (lanes) per K8d workgroup
constexpr int kStage = CDR_ING_STAGE;   // LDS bytes staged per K8d workgroup
constexpr int kNodeMissing = -3;  // a client that is no manifest primary node

__device__ __forceinline__ bool is_rec_end(const uint8_t* b, int64_t p, uint8_t c1, uint8_t c2) {
  // '\n' at p closes a non-blank line: c1 = b[p-1], c2 = b[p-2] (0 if absent)
  if (p == 0 || c1 == '\n') return false;
  if (c1 == '\r' && (p == 1 || c2 == '\n')) return false;
  return true;
}

// Terminator mask of the 16 bytes at tile lane t (bit j = record ends at byte j).
__device__ __forceinline__ unsigned lane_mask(const uint8_t* __restrict__ b, int64_t base,
                                              uint4 v) {
  uint8_t by[16];
  memcpy(by, &v, 16);
  unsigned m = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (by[j] != '\n') continue;
    const int64_t p = base + j;
    const uint8_t c1 = j >= 1 ? by[j - 1] : (p >= 1 ? b[p - 1] : 0);
    const uint8_t c2 = j >= 2 ? by[j - 2] : (p >= 2 ? b[p - 2] : 0);
    if (is_rec_end(b, p, c1, c2)) m |= 1u << j;
  }
  return m;
}

// Exclusive scan of one value per thread over a 256-thread workgroup (4
// waves: shuffles inside each wave, the wave totals through LDS); *total =
// the workgroup's sum.  Every thread of the workgroup calls it.
__device__ __forceinline__ long long wg256_exscan(long long v, long long* total) {
  __shared__ long long sw[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  long long inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const long long t = __shfl_up(inc, o);
    if (lane >= o) inc += t;
  }
  if (lane == 63) sw[w] = inc;
  __syncthreads();
  long long base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < w) base += sw[i];
    tot += sw[i];
  }
  __syncthreads();  // sw is reused by the next call
  *total = tot;
  return base + inc - v;
}

// Exclusive scan of n counts (the tile counts): per 4096-count part the sum
// (tile_scan_part), the parts' exclusive scan in one workgroup
// (tile_scan_mid), then every count's offset (tile_scan_out).
constexpr int kScanPer = 16;                // counts per thread
constexpr int kScanPart = 256 * kScanPer;   // counts per workgroup
__global__ __launch_bounds__(256) void tile_scan_part(const long long* __restrict__ cnt,
                                                      int64_t n, long long* __restrict__ part) {
  const int64_t lo = (int64_t)blockIdx.x * kScanPart + (int64_t)threadIdx.x * kScanPer;
  long long s = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j)
    if (lo + j < n) s += cnt[lo + j];
  long long tot;
  wg256_exscan(s, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void tile_scan_mid(long long* __restrict__ part, int64_t np) {
  const int64_t per = (np + 255) / 256;
  const int64_t lo = (int64_t)threadIdx.x * per;
  long long s = 0;
  for (int64_t i = lo; i < lo + per && i < np; ++i) s += part[i];
  long long tot;
  long long o = wg256_exscan(s, &tot);
  for (int64_t i = lo; i < lo + per && i < np; ++i) {
    const long long v = part[i];
    part[i] = o;
    o += v;
  }
}

__global__ __launch_bounds__(256) void tile_scan_out(const long long* __restrict__ cnt, int64_t n,
                                                     const long long* __restrict__ part,
                                                     long long* __restrict__ out) {
  const int64_t lo = (int64_t)blockIdx.x * kScanPart + (int64_t)threadIdx.x * kScanPer;
  long long v[kScanPer];
  long long s = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    v[j] = lo + j < n ? cnt[lo + j] : 0;
    s += v[j];
  }
  long long tot;
  long long o = part[blockIdx.x] + wg256_exscan(s, &tot);
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    if (lo + j < n) out[lo + j] = o;
    o += v[j];
  }
}

__global__ __launch_bounds__(256) void nl_count(const uint8_t* __restrict__ b,
                                                long long* __restrict__ tile_cnt,
                                                uint16_t* __restrict__ masks) {
  const int64_t base = (int64_t)blockIdx.x * kTile + threadIdx.x * 16;
  const uint4 v = *reinterpret_cast<const uint4*>(b + base);
  const unsigned m = lane_mask(b, base, v);
  masks[(int64_t)blockIdx.x * 256 + threadIdx.x] = (uint16_t)m;  // nl_write reads these
  long long tot;
  wg256_exscan(__popc(m), &tot);
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

// Record count after the scan of the tile counts: sc[0] = records
// (terminators + the tail record), sc[5] = 1 if the last record is a last
// line without '\n' (its end index nbytes is then written last).
__global__ void tile_total(const long long* __restrict__ cnt, const long long* __restrict__ off,
                           int64_t ntiles, const uint8_t* __restrict__ b, int64_t nbytes,
                           long long* __restrict__ sc) {
  long long tail = 0;
  if (nbytes > 0 && b[nbytes - 1] != '\n') {
    const uint8_t c1 = b[nbytes - 1], c2 = nbytes >= 2 ? b[nbytes - 2] : '\n';
    tail = !(c1 == '\r' && c2 == '\n');
  }
  sc[0] = off[ntiles - 1] + cnt[ntiles - 1] + tail;
  sc[5] = tail;
}

// From nl_count's per-lane terminator masks (1/8 of the log's bytes) instead
// of a second read of the log.
__global__ __launch_bounds__(256) void nl_write(const uint16_t* __restrict__ masks,
                                                const long long* __restrict__ tile_off,
                                                long long* __restrict__ ends) {
  const int64_t base = (int64_t)blockIdx.x * kTile + threadIdx.x * 16;
  unsigned m = masks[(int64_t)blockIdx.x * 256 + threadIdx.x];
  long long tot;
  long long o = tile_off[blockIdx.x] + wg256_exscan(__popc(m), &tot);
  while (m) {
    const int j = __ffs(m) - 1;
    m &= m - 1;
    ends[o++] = base + j;
  }
}

// ---- hashing ---------------------------------------------------------------
// Strings are read 4 bytes at a time: two aligned dword loads and a
// v_alignbyte, so one code path reads the LDS stage (ds_read_b32) and global
// memory.  Every buffer read this way carries >= 8 bytes past its end.
__device__ __forceinline__ unsigned ld4(const uint8_t* p) {
  const unsigned sh = (unsigned)reinterpret_cast<uintptr_t>(p) & 3u;
  const unsigned* w = reinterpret_cast<const unsigned*>(p - sh);
  return __builtin_amdgcn_alignbyte(w[1], w[0], sh);
}
__device__ __forceinline__ unsigned tail_mask(int64_t rem) {
  return rem >= 4 ? ~0u : (1u << (8 * rem)) - 1u;
}

__host__ __device__ __forceinline__ unsigned long long fin64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z ? z : 1ull;  // 0 marks an empty slot
}

// Word-wise: each step is a bijection of the state for a fixed word and
// injective in the word, so equal-length strings that differ in one word
// never collide; the length seeds the state.
__device__ __forceinline__ unsigned long long hash_bytes(const uint8_t* p, int64_t n) {
  unsigned long long h = 0x9E3779B97F4A7C15ull ^ (unsigned long long)n;
  for (int64_t k = 0; k < n; k += 4) {
    h = (h ^ (ld4(p + k) & tail_mask(n - k))) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
  }
  return fin64(h);
}

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, int64_t n) {
  unsigned diff = 0;
#pragma unroll 4
  for (int64_t k = 0; k < n; k += 4) diff |= (ld4(a + k) ^ ld4(b + k)) & tail_mask(n - k);
  return diff == 0;
}

// Open-addressing table: slot s = {key, meta} at tab[2s], tab[2s + 1] (one
// 16-byte load per probe), meta = byte offset << 24 | length of the owning
// string; idx[s] = its row (the first row with that string).
struct Dict {
  const unsigned long long* tab;
  const int32_t* idx;
  unsigned long long mask;
  const uint8_t* bytes;
};

__global__ void fill_i32(int32_t* __restrict__ a, int64_t n, int32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    a[i] = v;
}

__global__ void tab_insert(const uint8_t* __restrict__ bytes, const long long* __restrict__ off,
                           int64_t n, unsigned long long* __restrict__ tab,
                           int32_t* __restrict__ idx, unsigned long long mask) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const long long s = off[i], len = off[i + 1] - s;
    if (len <= 0) continue;  // an empty manifest string never matches a log field
    const unsigned long long h = hash_bytes(bytes + s, len);
    for (unsigned long long slot = h & mask;; slot = (slot + 1) & mask) {
      const unsigned long long old = atomicCAS(&tab[2 * slot], 0ull, h);
      if (old == 0ull || old == h) {
        atomicMin(&idx[slot], (int32_t)i);
        break;
      }
    }
  }
}

__global__ void tab_meta(const long long* __restrict__ off, unsigned long long* __restrict__ tab,
                         const int32_t* __restrict__ idx, unsigned long long nslots) {
  for (unsigned long long s = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
       s < nslots; s += (unsigned long long)gridDim.x * blockDim.x) {
    if (tab[2 * s] == 0ull) continue;
    const int32_t j = idx[s];
    tab[2 * s + 1] = ((unsigned long long)off[j] << 24) | (unsigned long long)(off[j + 1] - off[j]);
  }
}

// Row owning string (p, len), or -1.
__device__ __forceinline__ int32_t tab_find(const uint8_t* p, int64_t len, const Dict& d) {
  const unsigned long long h = hash_bytes(p, len);
  for (unsigned long long slot = h & d.mask;; slot = (slot + 1) & d.mask) {
    const ulonglong2 km = reinterpret_cast<const ulonglong2*>(d.tab)[slot];
    if (km.x == 0ull) return -1;
    if (km.x == h) {
      const int32_t j = d.idx[slot];
      return ((int64_t)(km.y & 0xFFFFFFull) == len && bytes_eq(d.bytes + (km.y >> 24), p, len))
                 ? j : -1;
    }
  }
}

// Split lookup: probe_begin hashes and issues the first slot load, so the
// caller can overlap two lookups and the timestamp parse with its latency.
struct Probe {
  unsigned long long h, slot;
  ulonglong2 km;
};
__device__ __forceinline__ void probe_begin(const uint8_t* p, int64_t len, const Dict& d,
                                            Probe& q) {
  q.h = hash_bytes(p, len);
  q.slot = q.h & d.mask;
  q.km = reinterpret_cast<const ulonglong2*>(d.tab)[q.slot];
}
__device__ __forceinline__ int32_t probe_end(const uint8_t* p, int64_t len, const Dict& d,
                                             Probe& q) {
  while (q.km.x != 0ull && q.km.x != q.h) {
    q.slot = (q.slot + 1) & d.mask;
    q.km = reinterpret_cast<const ulonglong2*>(d.tab)[q.slot];
  }
  if (q.km.x == 0ull) return -1;
  const int32_t j = d.idx[q.slot];
  return ((int64_t)(q.km.y & 0xFFFFFFull) == len && bytes_eq(d.bytes + (q.km.y >> 24), p, len))
             ? j : -1;
}

__global__ void tab_verify(const uint8_t* __restrict__ bytes, const long long* __restrict__ off,
                           int64_t n, Dict d, long long* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const long long s = off[i], len = off[i + 1] - s;
    if (len <= 0) continue;
    // -1 here means another string with the same 64-bit hash owns the slot
    if (tab_find(bytes + s, len, d) < 0) atomicMin(bad, (long long)i);
  }
}

// ---- timestamps: compute_features.parse_ts_us ------------------------------
__device__ __forceinline__ bool dig(uint8_t c) { return c >= '0' && c <= '9'; }
__device__ __forceinline__ bool wsp(uint8_t c) {
  // python str \s over ASCII: \t \n \v \f \r, 0x1c-0x1f, space
  return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f);
}

// 0 = parsed, 1 = no match / invalid date (None), 2 = unsupported (non-ASCII)
__device__ __forceinline__ int ts_finish(int y, int mo, int d, int hh, int mi, int ss, int us,
                                         long long off, long long* out) {
  // _days_from_civil with its validation
  if (mo < 1 || mo > 12) return 1;
  const bool leap = (y % 4 == 0) && (y % 100 != 0 || y % 400 == 0);
  const int mdays = mo == 2 ? 28 + leap : 30 + ((mo + (mo >> 3)) & 1);
  if (d < 1 || d > mdays) return 1;
  if (hh > 23 || mi > 59 || ss > 59) return 1;
  // 32-bit day arithmetic (|y| <= 9999: every term fits; constant divisions
  // become multiply-high sequences, not 64-bit division loops)
  const int y2 = y - (mo <= 2);
  const int era = (y2 >= 0 ? y2 : y2 - 399) / 400;
  const int yoe = y2 - era * 400;
  const int doy = (153 * (mo + (mo > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  const int days = era * 146097 + doe - 719468;
  *out = (((long long)days * 86400 + hh * 3600ll + mi * 60ll + ss) - off) * 1000000ll + us;
  return 0;
}

__device__ int parse_ts(const uint8_t* p, int n, long long* out) {
  if (n == 24) {
    // fast path for the simulator's own layout "YYYY-MM-DDTHH:MM:SS.fffZ"
    // (src/access_simulator.py:61): six word loads, straight-line digits;
    // any other string takes the general scan below (same result).
    unsigned w[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) w[k] = ld4(p + 4 * k);
    auto B = [&](int i) -> unsigned { return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu; };
    auto D = [&](int i) -> int { return (int)B(i) - '0'; };
    bool ok = B(4) == '-' && B(7) == '-' && B(10) == 'T' && B(13) == ':' && B(16) == ':' &&
              B(19) == '.' && B(23) == 'Z';
#pragma unroll
    for (int i = 0; i < 23; ++i) {
      if (i == 4 || i == 7 || i == 10 || i == 13 || i == 16 || i == 19) continue;
      ok &= (unsigned)D(i) <= 9u;
    }
    if (ok)
      return ts_finish(D(0) * 1000 + D(1) * 100 + D(2) * 10 + D(3), D(5) * 10 + D(6),
                       D(8) * 10 + D(9), D(11) * 10 + D(12), D(14) * 10 + D(15),
                       D(17) * 10 + D(18), (D(20) * 100 + D(21) * 10 + D(22)) * 1000, 0, out);
  }
  for (int i = 0; i < n; ++i)
    if (p[i] >= 0x80) return 2;
  int i = 0;
  auto num = [&](int lo, int hi, int* v) -> bool {  // greedy lo..hi digits
    int k = 0, x = 0;
    while (k < hi && i < n && dig(p[i])) x = x * 10 + (p[i++] - '0'), ++k;
    *v = x;
    return k >= lo;
  };
  while (i < n && wsp(p[i])) ++i;
  int y, mo, d, hh = 0, mi = 0, ss = 0, us = 0;
  if (!num(4, 4, &y)) return 1;
  if (i >= n || p[i] != '-') return 1;
  ++i;
  if (!num(1, 2, &mo)) return 1;
  if (i >= n || p[i] != '-') return 1;
  ++i;
  if (!num(1, 2, &d)) return 1;
  if (i + 1 < n && (p[i] == 'T' || p[i] == ' ') && dig(p[i + 1])) {
    ++i;
    num(1, 2, &hh);
    if (i >= n || p[i] != ':') return 1;
    ++i;
    if (!num(1, 2, &mi)) return 1;
    if (i + 1 < n && p[i] == ':' && dig(p[i + 1])) {
      ++i;
      num(1, 2, &ss);
      if (i + 1 < n && p[i] == '.' && dig(p[i + 1])) {
        ++i;
        int k = 0;
        while (k < 9 && i < n && dig(p[i])) {
          if (k < 6) us = us * 10 + (p[i] - '0');
          ++i, ++k;
        }
        for (; k < 6; ++k) us *= 10;
      }
    }
  }
  while (i < n && wsp(p[i])) ++i;
  long long off = 0;
  if (i < n && p[i] == 'Z') {
    ++i;
  } else if (i < n && (p[i] == '+' || p[i] == '-')) {
    const int sign = p[i] == '-' ? -1 : 1;
    ++i;
    int zh, zm = 0;
    if (!num(2, 2, &zh)) return 1;
    if (i < n && p[i] == ':') {
      ++i;
      if (!num(2, 2, &zm)) return 1;
    } else if (i < n && dig(p[i])) {
      if (!num(2, 2, &zm)) return 1;
    }
    off = sign * (zh * 3600ll + zm * 60ll);
  }
  while (i < n && wsp(p[i])) ++i;
  if (i != n) return 1;
  return ts_finish(y, mo, d, hh, mi, ss, us, off, out);
}

// One record: buf = the bytes from a0 on (LDS stage or global), st = byte
// position (relative to a0) just after the previous record, e0 = position of
// this record's terminator.
__device__ __forceinline__ void parse_record(const uint8_t* buf, int64_t st, int64_t e0,
                                             const Dict& paths, const Dict& nodes, int64_t r,
                                             int32_t* __restrict__ o_file,
                                             uint8_t* __restrict__ o_op,
                                             int32_t* __restrict__ o_client,
                                             long long* __restrict__ o_ts,
                                             long long* __restrict__ sc) {
  int64_t s = st;  // skip the blank lines before the record ("\n", "\r\n")
  for (;;) {
    const uint8_t c = buf[s];
    if (c == '\n') ++s;
    else if (c == '\r' && buf[s + 1] == '\n') s += 2;
    else break;
  }
  int64_t e = e0;
  if (e > s && buf[e - 1] == '\r') --e;
  // field f spans [c_{f-1} + 1, c_f) with c_{-1} = s - 1 and c_f = e past the
  // last comma (the commas after the fourth one are irrelevant)
  int64_t c0 = e, c1 = e, c2 = e, c3 = e;
  int fi = 0;
  unsigned bad = 0;
  // four bytes at a time: exact per-byte flags (no borrow between bytes) of
  // ',' and of the bytes the host tokeniser must take ('"', NUL, '\r')
  auto zb = [](unsigned x) {
    const unsigned t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    return ~(t | x | 0x7F7F7F7Fu);  // 0x80 in each zero byte of x
  };
  for (int64_t k = s; k < e; k += 4) {
    const unsigned w = ld4(buf + k);
    const int64_t rem = e - k;
    const unsigned live = rem >= 4 ? 0x80808080u : (0x80808080u & ((1u << (8 * rem)) - 1u));
    bad |= (zb(w ^ 0x22222222u) | zb(w) | zb(w ^ 0x0D0D0D0Du)) & live;
    unsigned cm = zb(w ^ 0x2C2C2C2Cu) & live;
    while (cm && fi < 4) {
      const int64_t at = k + (__builtin_ctz(cm) >> 3);
      if (fi == 0) c0 = at;
      else if (fi == 1) c1 = at;
      else if (fi == 2) c2 = at;
      else c3 = at;
      ++fi;
      cm &= cm - 1u;
    }
  }
  bool unsup = bad != 0;
  const int64_t f1 = min(c0 + 1, e), f2 = min(c1 + 1, e), f3 = min(c2 + 1, e);
  // both dictionary probes go out first; the timestamp parse overlaps them
  const bool has_path = c1 > f1, has_client = c3 > f3 && nodes.mask;
  Probe qp, qc;
  if (has_path) probe_begin(buf + f1, c1 - f1, paths, qp);
  if (has_client) probe_begin(buf + f3, c3 - f3, nodes, qc);
  long long ts = LLONG_MIN;
  int stt = 1;
  if (c0 > s) stt = parse_ts(buf + s, (int)(c0 - s), &ts);
  if (stt == 2) unsup = true;
  if (stt != 0) ts = LLONG_MIN;
  uint8_t op = 0;
  const int64_t ol = c2 - f2;
  const unsigned ow = ld4(buf + f2);
  if (ol == 5 && ow == 0x54495257u && buf[f2 + 4] == 'E') op = 1;  // "WRIT" + 'E'
  if (ol == 4 && ow == 0x44414552u) op = 2;                         // "READ"
  const int32_t file = has_path ? probe_end(buf + f1, c1 - f1, paths, qp) : -1;
  int32_t client = -1;
  if (c3 > f3) {
    client = has_client ? probe_end(buf + f3, c3 - f3, nodes, qc) : -1;
    if (client < 0) client = kNodeMissing;
  }
  o_file[r] = file;
  o_op[r] = op;
  o_client[r] = client;
  o_ts[r] = ts;
  if (stt != 0 && !unsup) {
    atomicMin(&sc[1], (long long)r);
    atomicAdd(reinterpret_cast<unsigned long long*>(&sc[3]), 1ull);
  }
  if (unsup) atomicMin(&sc[2], (long long)r);
}

// sc[1] = first record with an unparseable / null timestamp, sc[2] = first
// unsupported record, sc[3] = number of unparseable timestamps (all LLONG_MAX /
// 0 initially).  Unparseable timestamps are stored as LLONG_MIN.
__global__ __launch_bounds__(kRecPerWG) void parse(const uint8_t* __restrict__ b,
                                             const long long* __restrict__ ends, int64_t nrec,
                                             Dict paths, Dict nodes,
                                             int32_t* __restrict__ o_file,
                                             uint8_t* __restrict__ o_op,
                                             int32_t* __restrict__ o_client,
                                             long long* __restrict__ o_ts,
                                             long long* __restrict__ sc) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[kStage + 16];
  const int64_t r0 = (int64_t)blockIdx.x * kRecPerWG;
  const int64_t r1 = min<int64_t>(nrec, r0 + kRecPerWG);
  const int64_t lo = r0 == 0 ? 0 : ends[r0 - 1] + 1;
  const int64_t hi = ends[r1 - 1];
  const int64_t a0 = lo & ~(int64_t)15;
  const int64_t r = r0 + threadIdx.x;
  // byte positions are relative to a0 (an LDS pointer offset by -a0 would
  // wrap in 32 bits)
  const int64_t e0 = r < r1 ? ends[r] - a0 : 0;
  const int64_t st = r < r1 ? (r == r0 ? lo : ends[r - 1] + 1) - a0 : 0;
  if (hi - a0 <= kStage) {
    const int nvec = (int)((hi - a0 + 15) >> 4);
    for (int v = threadIdx.x; v < nvec; v += kRecPerWG)
      reinterpret_cast<uint4*>(stage)[v] = reinterpret_cast<const uint4*>(b + a0)[v];
    __syncthreads();
    if (r < r1) parse_record(stage, st, e0, paths, nodes, r, o_file, o_op, o_client, o_ts, sc);
  } else if (r < r1) {
    parse_record(b + a0, st, e0, paths, nodes, r, o_file, o_op, o_client, o_ts, sc);
  }
}

int gsz(int64_t work, int threads, int cap) {
  int64_t g = (work + threads - 1) / threads;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

uint64_t table_mask(int64_t n) {
  uint64_t cap = 64;
  while (cap < (uint64_t)(2 * n)) cap <<= 1;
  return cap - 1;
}

// Builds (tab, idx) for n strings given as bytes + offsets already on the device.
void build_table(Ctx& c, DevBuf& key, DevBuf& idx, const uint8_t* bytes, const long long* off,
                 int64_t n, uint64_t mask, const char* what) {
  key.ensure(16 * (mask + 1));
  idx.ensure(4 * (mask + 1));
  HIP_CHECK(hipMemsetAsync(key.p, 0, 16 * (mask + 1), c.stream));
  hipLaunchKernelGGL(fill_i32, dim3(gsz(mask + 1, 256, 8192)), dim3(256), 0, c.stream,
                     idx.as<int32_t>(), (int64_t)(mask + 1), INT_MAX);
  hipLaunchKernelGGL(tab_insert, dim3(gsz(n, 256, 8192)), dim3(256), 0, c.stream, bytes, off, n,
                     key.as<unsigned long long>(), idx.as<int32_t>(), (unsigned long long)mask);
  hipLaunchKernelGGL(tab_meta, dim3(gsz(mask + 1, 256, 8192)), dim3(256), 0, c.stream, off,
                     key.as<unsigned long long>(), idx.as<int32_t>(),
                     (unsigned long long)(mask + 1));
  long long* bad = c.ing_scalar.as<long long>() + 4;
  const long long init = LLONG_MAX;
  HIP_CHECK(hipMemcpyAsync(bad, &init, 8, hipMemcpyHostToDevice, c.stream));
  const Dict d{key.as<unsigned long long>(), idx.as<int32_t>(), (unsigned long long)mask, bytes};
  hipLaunchKernelGGL(tab_verify, dim3(gsz(n, 256, 8192)), dim3(256), 0, c.stream, bytes, off, n,
                     d, bad);
  HIP_CHECK(hipGetLastError());
  long long hb = 0;
  HIP_CHECK(hipMemcpyAsync(&hb, bad, 8, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  if (hb != LLONG_MAX)
    CDR_FAIL(CDR_ERR_UNSUPPORTED, std::string("64-bit hash collision between two distinct ") +
                                      what + " (row " + std::to_string(hb) + ")");
}

void upload_strings(Ctx& c, DevBuf& bytes, DevBuf& off, const char* h_bytes,
                    const int64_t* h_off, int64_t n) {
  const int64_t nb = h_off[n];
  if (h_off[0] != 0 || nb < 0) CDR_FAIL(CDR_ERR_ARG, "string offsets must start at 0");
  for (int64_t i = 0; i < n; ++i) {
    if (h_off[i + 1] < h_off[i]) CDR_FAIL(CDR_ERR_ARG, "string offsets must be non-decreasing");
    if (h_off[i + 1] - h_off[i] >= (1 << 24))
      CDR_FAIL(CDR_ERR_UNSUPPORTED, "string of 16 MiB or more in the manifest");
  }
  if (nb >= (1ll << 40)) CDR_FAIL(CDR_ERR_UNSUPPORTED, "manifest strings of 1 TiB or more");
  bytes.ensure(nb + 16);  // ld4 reads up to 7 bytes past a string
  off.ensure(8 * (n + 1));
  if (nb > 0) HIP_CHECK(hipMemcpyAsync(bytes.p, h_bytes, nb, hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipMemcpyAsync(off.p, h_off, 8 * (n + 1), hipMemcpyHostToDevice, c.stream));
}

}  // namespace

void ingest_manifest(Ctx& c, int64_t n_files, const char* pbytes, const int64_t* poff,
                     const int32_t* primary, int32_t n_nodes, const char* nbytes,
                     const int64_t* noff) {
  if (n_files < 1) CDR_FAIL(CDR_ERR_ARG, "need n_files >= 1");
  if (n_files >= (1ll << 31) - 1) CDR_FAIL(CDR_ERR_UNSUPPORTED, "n_files >= 2^31 - 1");
  if (n_nodes < 0) CDR_FAIL(CDR_ERR_ARG, "negative n_nodes");
  c.ing_scalar.ensure(8 * 16);
  upload_strings(c, c.ing_pbytes, c.ing_poff, pbytes, poff, n_files);
  c.ing_pmask = table_mask(n_files);
  build_table(c, c.ing_pkey, c.ing_pidx, c.ing_pbytes.as<uint8_t>(),
              c.ing_poff.as<long long>(), n_files, c.ing_pmask, "manifest paths");
  c.ing_nnodes = n_nodes;
  c.ing_nmask = 0;
  if (n_nodes > 0) {
    upload_strings(c, c.ing_nbytes, c.ing_noff, nbytes, noff, n_nodes);
    c.ing_nmask = table_mask(n_nodes);
    build_table(c, c.ing_nkey, c.ing_nidx, c.ing_nbytes.as<uint8_t>(),
                c.ing_noff.as<long long>(), n_nodes, c.ing_nmask, "node names");
  }
  c.ev_primary.ensure(4 * n_files);
  HIP_CHECK(hipMemcpyAsync(c.ev_primary.p, primary, 4 * n_files, hipMemcpyHostToDevice,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.ing_nfiles = n_files;
  c.ev_n = 0;
  c.ev_tsr_valid = false;
  c.ev_nf = 0;
}

// Parses the resident log bytes (c.ing_log, c.ing_nbytes_log) into c.ev_*.
// status[0] = records, [1] = first bad-timestamp record (-1 none),
// [2] = first unsupported record (-1 none), [3] = bad-timestamp count,
// [4]/[5] = byte span [start, end) of the record in [1] (or [2]).
void ingest_parse(Ctx& c, int64_t* status) {
  const int64_t nbytes = c.ing_nbytes_log;
  const int64_t ntiles = nbytes > 0 ? ceil_div(nbytes, kTile) : 0;
  long long* sc = c.ing_scalar.as<long long>();
  const long long init[4] = {0, LLONG_MAX, LLONG_MAX, 0};
  HIP_CHECK(hipMemcpyAsync(sc, init, sizeof(init), hipMemcpyHostToDevice, c.stream));
  long long nrec = 0;
  bool tail = false;
  if (ntiles > 0) {
    c.ing_blk.ensure(16 * ntiles);
    long long* cnt = c.ing_blk.as<long long>();
    long long* toff = cnt + ntiles;
    c.ing_mask.ensure(2 * 256 * ntiles);
    hipLaunchKernelGGL(nl_count, dim3(ntiles), dim3(256), 0, c.stream, c.ing_log.as<uint8_t>(),
                       cnt, c.ing_mask.as<uint16_t>());
    const int64_t nparts = ceil_div(ntiles, kScanPart);
    c.ing_tmp.ensure(sizeof(long long) * nparts);
    long long* part = c.ing_tmp.as<long long>();
    hipLaunchKernelGGL(tile_scan_part, dim3(nparts), dim3(256), 0, c.stream, cnt, ntiles, part);
    hipLaunchKernelGGL(tile_scan_mid, dim3(1), dim3(256), 0, c.stream, part, nparts);
    hipLaunchKernelGGL(tile_scan_out, dim3(nparts), dim3(256), 0, c.stream, cnt, ntiles, part,
                       toff);
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(tile_total, dim3(1), dim3(1), 0, c.stream, cnt, toff, ntiles,
                       c.ing_log.as<uint8_t>(), nbytes, sc);
    HIP_CHECK(hipGetLastError());
    long long r6[6];
    HIP_CHECK(hipMemcpyAsync(r6, sc, sizeof(r6), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    nrec = r6[0];
    tail = r6[5] != 0;
  }
  const int64_t ne1 = nrec > 0 ? nrec : 1;
  c.ing_ends.ensure(8 * ne1);
  c.ev_file.ensure(4 * ne1);
  c.ev_op.ensure(ne1);
  c.ev_client.ensure(4 * ne1);
  c.ev_ts.ensure(8 * ne1);
  c.ev_out.ensure(8 * 6 * (c.ing_nfiles > 0 ? c.ing_nfiles : 1) + 64);
  if (nrec > 0) {
    // the tail record's end goes last
    hipLaunchKernelGGL(nl_write, dim3(ntiles), dim3(256), 0, c.stream, c.ing_mask.as<uint16_t>(),
                       c.ing_blk.as<long long>() + ntiles, c.ing_ends.as<long long>());
    if (tail) {
      c.h_small.ensure(64);
      *c.h_small.as<long long>() = nbytes;
      HIP_CHECK(hipMemcpyAsync(c.ing_ends.as<long long>() + nrec - 1, c.h_small.p, 8,
                               hipMemcpyHostToDevice, c.stream));
    }
    const Dict pd{c.ing_pkey.as<unsigned long long>(), c.ing_pidx.as<int32_t>(), c.ing_pmask,
                  c.ing_pbytes.as<uint8_t>()};
    const Dict nd{c.ing_nkey.as<unsigned long long>(), c.ing_nidx.as<int32_t>(), c.ing_nmask,
                  c.ing_nbytes.as<uint8_t>()};
    hipLaunchKernelGGL(parse, dim3(ceil_div(nrec, kRecPerWG)), dim3(kRecPerWG), 0, c.stream,
                       c.ing_log.as<uint8_t>(), c.ing_ends.as<long long>(), (int64_t)nrec, pd, nd,
                       c.ev_file.as<int32_t>(), c.ev_op.as<uint8_t>(), c.ev_client.as<int32_t>(),
                       c.ev_ts.as<long long>(), sc);
    HIP_CHECK(hipGetLastError());
  }
  long long r[4];
  HIP_CHECK(hipMemcpyAsync(r, sc, sizeof(r), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  status[0] = nrec;
  status[1] = r[1] == LLONG_MAX ? -1 : r[1];
  status[2] = r[2] == LLONG_MAX ? -1 : r[2];
  status[3] = r[3];
  status[4] = status[5] = -1;
  const long long which = status[2] >= 0 ? status[2] : status[1];
  if (which >= 0) {
    long long e[2] = {-1, 0};
    if (which > 0)
      HIP_CHECK(hipMemcpyAsync(e, c.ing_ends.as<long long>() + which - 1, 16,
                               hipMemcpyDeviceToHost, c.stream));
    else
      HIP_CHECK(hipMemcpyAsync(e + 1, c.ing_ends.as<long long>(), 8, hipMemcpyDeviceToHost,
                               c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    status[4] = e[0] + 1;  // the record starts after the last '\n' before it
    status[5] = e[1];
  }
  c.ev_n = nrec;
  events_ts_range(c, nrec);
  c.ev_nf = c.ing_nfiles;
  c.ev_cmax = std::max(0, c.ing_nnodes - 1);  // client ids are node ids (or < 0)
}

void ingest_log(Ctx& c, const char* bytes, int64_t nbytes, int64_t* status) {
  if (c.ing_nfiles < 1) CDR_FAIL(CDR_ERR_STATE, "no manifest (cdr_ingest_manifest)");
  if (nbytes < 0) CDR_FAIL(CDR_ERR_ARG, "negative nbytes");
  const int64_t ntiles = nbytes > 0 ? ceil_div(nbytes, kTile) : 0;
  const size_t padded = (size_t)(ntiles + 1) * kTile;  // a zero tile after the last
  c.ing_log.ensure(padded);
  HIP_CHECK(hipMemsetAsync(c.ing_log.as<uint8_t>() + nbytes, 0, padded - nbytes, c.stream));
  if (nbytes > 0)
    HIP_CHECK(hipMemcpyAsync(c.ing_log.p, bytes, nbytes, hipMemcpyHostToDevice, c.stream));
  c.ing_nbytes_log = nbytes;
  ingest_parse(c, status);
}

}  // namespace cdr

using namespace cdr;

extern "C" {

int cdr_ingest_manifest(cdr_ctx* h, int64_t n_files, const char* path_bytes,
                        const int64_t* path_off, const int32_t* primary, int32_t n_nodes,
                        const char* node_bytes, const int64_t* node_off) {
  CDR_TRY
  if (!h || !path_off || !primary || (n_nodes > 0 && !node_off)) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  ingest_manifest(h->c, n_files, path_bytes, path_off, primary, n_nodes, node_bytes, node_off);
  CDR_CATCH
}

int cdr_ingest_log(cdr_ctx* h, const char* bytes, int64_t nbytes, int64_t* status) {
  CDR_TRY
  if (!h || !status || (nbytes > 0 && !bytes)) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  ingest_log(h->c, bytes, nbytes, status);
  CDR_CATCH
}

int cdr_ingest_reparse(cdr_ctx* h, int64_t* status) {
  CDR_TRY
  if (!h || !status) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  if (c.ing_nfiles < 1) CDR_FAIL(CDR_ERR_STATE, "no manifest (cdr_ingest_manifest)");
  HIP_CHECK(hipSetDevice(c.device));
  ingest_parse(c, status);
  CDR_CATCH
}

}  // extern "C"
