// lloyd.hip — one Lloyd iteration (reference src/kmeans_plusplus.py:31-43).
//
//   labels = argmin_j sqrt(pw_d((x - c_j)^2))          (:33-34, first index on ties)
//   new_c[j] = mean(X[labels == j])                     (:37-41; host divides)
//
// F32X mode (grid data, fp32 storage) runs three kernels per step:
//   1. screen_kernel — fp16 hi/lo split MFMA (v_mfma_f32_16x16x32_f16) screen of
//      T_j ~ ||xhat - chat_j||^2 for every centroid, a wave-level certified
//      argmin (best and runner-up keys), and — for certified points — the
//      exact int64 fixed-point centroid sums/counts privatised in LDS.
//      Uncertified points are appended to a fallback list.
//   2. reduce_partials — sums the per-workgroup LDS tables (no float atomics,
//      integer sums are order independent, hence bit-reproducible).
//   3. fallback_exact — NumPy-order fp64 distances + correctly rounded sqrt for
//      the listed points, then integer atomics into the totals.
// The certification bound makes the labels identical to the
// fp64 reference: a point is certified only when its runner-up screen value
// exceeds the best by more than twice the rigorous screen error plus the
// reference's own rounding slack.
//
// F64 mode (arbitrary fp64 data): exact fp64 assignment for every point and a
// row-ordered fp64 sum per (cluster, feature) — NumPy's X[mask].mean(axis=0)
// is a sequential row-order sum for d >= 2 and the blocked pairwise sum for
// d == 1 (oracle/kmeans_oracle.py pins both against NumPy).
#include <cstdio>
#include <cmath>
#include <cstring>

#include "cdr_internal.h"
#include "exact_math.h"

namespace cdr {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

struct ScreenArgs {
  const float* X;
  int64_t n, n_pad;
  int d, k, KT;
  const h8* frag;
  const float* mu_s;  // -mu_f * 2^sigma
  float sig;          // 2^sigma
  float fx;           // 2^S (fixed-point scale)
  float thrA0, thrA1;
  int32_t* labels;
  unsigned long long* partials;
  int32_t* fb_list;   // per-wave regions of fb_cap entries
  int32_t* fb_count;  // [waves] entries per region, [waves] = total
  int fb_cap;
  float* dbg;  // optional: screen values (n_pad x KT*16) for tests
  int ablate;  // timing experiments only (CDR_SCREEN_ABLATE): 1 no update,
               // 2 no argmin, 4 no MFMA, 8 no loads; results are garbage
};

// Running (best, runner-up) of unsigned keys: second = med3(best, v, second)
// holds because best <= second.
__device__ __forceinline__ void push_key(unsigned& bk, unsigned& sk, unsigned v) {
  sk = max(min(bk, v), min(max(bk, v), sk));  // v_med3_u32
  bk = min(bk, v);
}

template <int DCH, bool PACK6, bool DBG>
__global__ __launch_bounds__(256) void screen_kernel(ScreenArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int nfrag = a.KT * DCH * 2 * 64;
  h8* sfrag = reinterpret_cast<h8*>(smem);
  unsigned long long* tbl =
      reinterpret_cast<unsigned long long*>(smem + (size_t)nfrag * sizeof(h8));
  const int d = a.d;
  const int kd1 = d + 1;
  for (int i = threadIdx.x; i < nfrag; i += blockDim.x) sfrag[i] = a.frag[i];
  for (int i = threadIdx.x; i < a.k * kd1; i += blockDim.x) tbl[i] = 0ull;
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;    // lane group: k-slots 8g..8g+7, centroid rows 4g..4g+3
  const int col = lane & 15;  // point column of the 16x16 tile
  float ms[DCH][4];
  bool fok[DCH][4];
#pragma unroll
  for (int c = 0; c < DCH; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = 16 * c + 4 * g + i;
      fok[c][i] = f < d;
      ms[c][i] = fok[c][i] ? a.mu_s[f] : 0.0f;
    }
  const unsigned kmask = PACK6 ? 63u : 15u;
  const int wpb = blockDim.x >> 6;
  const int64_t ngroups = a.n_pad >> 6;
  const int wave_id = blockIdx.x * wpb + (threadIdx.x >> 6);
  int32_t* fb_region = a.fb_list + (size_t)wave_id * a.fb_cap;
  int fb_used = 0;
  for (int64_t G = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); G < ngroups;
       G += (int64_t)gridDim.x * wpb) {
    const int64_t base = G << 6;
    if (base >= a.n) continue;  // wave-uniform: padding groups
    float xr[4][DCH][4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int c = 0; c < DCH; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int f = 16 * c + 4 * g + i;
          xr[p][c][i] = fok[c][i] ? a.X[xidx(a.X, f, base + 16 * p + col, a.n_pad)] : 0.0f;
        }
    if (a.ablate & 8) {
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int c = 0; c < DCH; ++c)
#pragma unroll
          for (int i = 0; i < 4; ++i) xr[p][c][i] = (float)((int)(base + p * 16 + col + i) & 255) * 0x1p-8f;
    }
    h8 b1[4][DCH], b2[4][DCH];
    float xx[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float s = 0.0f;
#pragma unroll
      for (int c = 0; c < DCH; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float xt = fmaf(xr[p][c][i], a.sig, ms[c][i]);  // (x - mu) 2^sigma
          const _Float16 hi = (_Float16)xt;
          const _Float16 lo = (_Float16)(xt - (float)hi);
          s = fmaf(xt, xt, s);
          b1[p][c][2 * i] = hi;
          b1[p][c][2 * i + 1] = lo;
          b2[p][c][2 * i] = hi;
          b2[p][c][2 * i + 1] = (_Float16)0.0f;
        }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      xx[p] = s;
      // chunk-0 spare slots: lane group 0 carries ||xhat||^2 (3-way fp16
      // split, paired with 1.0 in A), group 1 carries 1.0 (paired with the
      // 3-way split of ||chat_j||^2 + eps in A).
      _Float16 e0, e1, e2;
      if (g == 0) {
        e0 = (_Float16)s;
        float r = s - (float)e0;
        e1 = (_Float16)r;
        r = r - (float)e1;
        e2 = (_Float16)r;
      } else if (g == 1) {
        e0 = e1 = e2 = (_Float16)1.0f;
      } else {
        e0 = e1 = e2 = (_Float16)0.0f;
      }
      b2[p][0][1] = e0;
      b2[p][0][3] = e1;
      b2[p][0][5] = e2;
    }

    unsigned bk[4], sk[4];
    int bt[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      bk[p] = 0xFFFFFFFFu;
      sk[p] = 0xFFFFFFFFu;
      bt[p] = 0;
    }
    for (int t = 0; t < a.KT; ++t) {
      h8 A1[DCH], A2[DCH];
#pragma unroll
      for (int c = 0; c < DCH; ++c) {
        A1[c] = sfrag[((t * DCH + c) * 2 + 0) * 64 + lane];
        A2[c] = sfrag[((t * DCH + c) * 2 + 1) * 64 + lane];
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
        if (a.ablate & 4) {
          acc[0] = (float)b1[p][0][0] + (float)A1[0][1];
          acc[1] = (float)b2[p][0][1] + (float)A2[0][2];
          acc[2] = (float)b1[p][0][2] + t;
          acc[3] = xx[p];
        } else {
#pragma unroll
          for (int c = 0; c < DCH; ++c) {
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1[c], b1[p][c], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(A2[c], b2[p][c], acc, 0, 0, 0);
          }
        }
        if (a.ablate & 2) {
          bk[p] ^= __float_as_uint(acc[0] + acc[1] + acc[2] + acc[3]);
          continue;
        }
        if constexpr (DBG) {
          const int64_t pt = base + 16 * p + col;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            a.dbg[pt * (int64_t)(a.KT * 16) + 16 * t + 4 * g + r] = acc[r];
        }
        if constexpr (PACK6) {
          const unsigned jb = 16u * (unsigned)t;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            push_key(bk[p], sk[p], (__float_as_uint(acc[r]) & ~63u) | (jb + r));
        } else {
          unsigned tb = (__float_as_uint(acc[0]) & ~15u) | 0u, ts = 0xFFFFFFFFu;
          push_key(tb, ts, (__float_as_uint(acc[1]) & ~15u) | 1u);
          push_key(tb, ts, (__float_as_uint(acc[2]) & ~15u) | 2u);
          push_key(tb, ts, (__float_as_uint(acc[3]) & ~15u) | 3u);
          const bool take = tb < bk[p];
          const unsigned nsk = min(max(bk[p], tb), min(sk[p], ts));
          bt[p] = take ? t : bt[p];
          bk[p] = min(bk[p], tb);
          sk[p] = nsk;
        }
      }
    }

#pragma unroll
    for (int p = 0; p < 4; ++p) {
      unsigned b = bk[p] | ((unsigned)g << 2), s = sk[p] | ((unsigned)g << 2);
      int tsel = bt[p];
#pragma unroll
      for (int m = 16; m <= 32; m <<= 1) {
        const unsigned ob = (unsigned)__shfl_xor((int)b, m);
        const unsigned os = (unsigned)__shfl_xor((int)s, m);
        const int ot = PACK6 ? 0 : __shfl_xor(tsel, m);
        const unsigned ns = min(max(b, ob), min(s, os));
        if (!PACK6) tsel = ob < b ? ot : tsel;
        b = min(b, ob);
        s = ns;
      }
      const int label = PACK6 ? (int)(b & 63u) : tsel * 16 + (int)(b & 15u);
      const float vb = __uint_as_float(b & ~kmask);
      const float vs = __uint_as_float(s & ~kmask);
      const float lim = fmaf(vb, 1.0f + 0x1p-15f, fmaf(a.thrA1, xx[p], a.thrA0));
      const bool cert = (a.ablate & 2) ? true : vs > lim;  // NaN: never certifies
      const int64_t pt = base + 16 * p + col;
      const bool real = pt < a.n;
      if (g == 0 && real) a.labels[pt] = label;
      const bool need = (g == 0) && real && !cert;
      const unsigned long long m = __ballot(need);
      if (m) {
        const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        if (need) fb_region[fb_used + rank] = (int32_t)pt;
        fb_used += __popcll(m);
      }
      if (a.ablate & 1) {
        asm volatile("" ::"v"(xr[p][0][0]), "v"(xr[p][0][3]), "v"(label));
        continue;
      }
      if (real && cert) {
        unsigned long long* row = tbl + (size_t)((unsigned)label < (unsigned)a.k ? label : 0) * kd1;
#pragma unroll
        for (int c = 0; c < DCH; ++c)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (fok[c][i]) {
              const long long u = (long long)(int)(xr[p][c][i] * a.fx);
              atomicAdd(&row[16 * c + 4 * g + i], (unsigned long long)u);
            }
        if (g == 0) atomicAdd(&row[d], 1ull);
      }
    }
  }
  if (lane == 0) {
    a.fb_count[wave_id] = fb_used;
    if (fb_used) atomicAdd(a.fb_count + (int64_t)gridDim.x * wpb, fb_used);
  }
  __syncthreads();
  unsigned long long* dst = a.partials + (size_t)blockIdx.x * a.k * kd1;
  for (int i = threadIdx.x; i < a.k * kd1; i += blockDim.x) dst[i] = tbl[i];
}


// ---------------------------------------------------------------------------
// screen_fast: the k*d <= 64*16 regime (KT*DCH <= 4), the BASELINE configs.
// A fragments live in registers for the whole kernel; one wave processes a
// 64-point group per iteration as four 16-point tiles and prefetches the
// next group's quads while it computes.  Per tile and lane: one 16-byte load
// per 16 features, packed fp32->fp16 hi/lo split, 2*KT*DCH MFMAs whose first
// C operand is the point norm ||xhat||^2, 2.5 VALU ops per screen value for
// the running (best, runner-up) keys.  Per group: the four tiles' (best,
// runner-up) pairs are reduced across the lane groups by a 4x4 permlane
// transpose, after which lane group g owns tile g's points — one coalesced
// label store, one certification test, one fallback ballot — and the
// per-point verdicts are broadcast back for the LDS u64 adds (4 per 16
// features, +1 count) of the certified points.
// Fragment k-slot order (must match build_screen_plan):
//   B1 = [hi0..3, lo0..3]      B2 = [hi0..3, (g==1: 1, 1, 1, 0)]
//   A1 = [-2chi0..3, -2chi0..3]  A2 = [-2clo0..3, (g==1: cc parts p0, p1, p2, 0)]
// ---------------------------------------------------------------------------
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned pack_h2(float a, float b) {
  h2v h = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(unsigned, h);
}

__device__ __forceinline__ unsigned umed3(unsigned a, unsigned b, unsigned c) {
  return max(min(a, b), min(max(a, b), c));  // v_med3_u32
}

// (best, runner-up) of two (best, runner-up) pairs
__device__ __forceinline__ void merge_top2(unsigned& b, unsigned& s, unsigned b2, unsigned s2) {
  const unsigned nb = min(b, b2);
  s = min(max(b, b2), min(s, s2));
  b = nb;
}

// Exchange halves between x and y: permlane32 pairs lane L < 32 with L + 32,
// permlane16 pairs row 2r with row 2r + 1 (rows of 16 lanes).
__device__ __forceinline__ void swap32(unsigned& x, unsigned& y) {
  auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}
__device__ __forceinline__ void swap16(unsigned& x, unsigned& y) {
  auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}

template <int DCH, int KT, bool NONNEG, bool FULL, int ABL = 0, int WAVES = 4>
__global__ __launch_bounds__(256, WAVES) void screen_fast(ScreenArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long* tbl = reinterpret_cast<unsigned long long*>(smem);
  const int d = a.d;
  const int d4 = (d + 3) & ~3;
  const int KS = d4 + 1;  // table row: d4 sums (padding features add 0) + count
  for (int i = threadIdx.x; i < a.k * KS; i += blockDim.x) tbl[i] = 0ull;

  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int col = lane & 15;
  h8 A1[KT][DCH], A2[KT][DCH];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int c = 0; c < DCH; ++c) {
      A1[t][c] = a.frag[((t * DCH + c) * 2 + 0) * 64 + lane];
      A2[t][c] = a.frag[((t * DCH + c) * 2 + 1) * 64 + lane];
    }
  f4v ms[DCH];
  bool qok[DCH];
  const f4v* Xq = reinterpret_cast<const f4v*>(a.X);
#pragma unroll
  for (int c = 0; c < DCH; ++c) {
    const int f0 = 16 * c + 4 * g;
    qok[c] = FULL || f0 < d4;
#pragma unroll
    for (int i = 0; i < 4; ++i) ms[c][i] = (f0 + i < d) ? a.mu_s[f0 + i] : 0.0f;
  }
  // chunk-0 spare k-slots: lane group 1 holds the 1.0 multipliers of the
  // three fp16 parts of ||c_j||^2 + eps (constants, no per-tile work)
  const unsigned one01 = g == 1 ? pack_h2(1.0f, 1.0f) : 0u;
  const unsigned one2 = g == 1 ? pack_h2(1.0f, 0.0f) : 0u;
  const float sig = a.sig, fx = a.fx, thrA0 = a.thrA0, thrA1 = a.thrA1;
  const int wpb = blockDim.x >> 6;
  const int64_t ngroups = a.n_pad >> 6;
  const int64_t gstride = (int64_t)gridDim.x * wpb;
  int64_t G = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6);
  const int wave_id = (int)G;
  int32_t* fb_region = a.fb_list + (size_t)wave_id * a.fb_cap;
  int fb_used = 0;
  constexpr int ablate = ABL;  // timing experiments only (separate instances)
  __syncthreads();

  auto load = [&](f4v (&buf)[4][DCH], int64_t grp) {
    if constexpr ((ablate & 8) != 0) {  // synthetic points, no HBM reads
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int c = 0; c < DCH; ++c)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            buf[p][c][i] = (float)(((int)grp + 7 * p + 3 * i + col) & 255) * 0x1p-8f;
      return;
    }
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int c = 0; c < DCH; ++c) {
        if (FULL) {
          buf[p][c] = Xq[(int64_t)(4 * c + g) * a.n_pad + (grp << 6) + 16 * p + col];
        } else {
          f4v v = {0.f, 0.f, 0.f, 0.f};
          if (qok[c]) v = Xq[(int64_t)(4 * c + g) * a.n_pad + (grp << 6) + 16 * p + col];
          buf[p][c] = v;
        }
      }
  };

  // B fragments + MFMAs of one 16-point tile; the point norm (summed over the
  // four lane groups) enters as the first MFMA's C operand.  Returns it.
  auto screen_tile = [&](const f4v (&xq)[DCH], f4 (&acc)[KT]) -> float {
    h8 b1[DCH], b2[DCH];
    float xxp = 0.0f;
#pragma unroll
    for (int c = 0; c < DCH; ++c) {
      f4v xt;
#pragma unroll
      for (int i = 0; i < 4; ++i) xt[i] = fmaf(xq[c][i], sig, ms[c][i]);
      const unsigned h01 = pack_h2(xt[0], xt[1]), h23 = pack_h2(xt[2], xt[3]);
      const h2v hh01 = __builtin_bit_cast(h2v, h01), hh23 = __builtin_bit_cast(h2v, h23);
      // residual x - hi straight from the packed halves (v_fma_mix_f32)
      const unsigned l01 = pack_h2(fmaf((float)hh01[0], -1.0f, xt[0]),
                                   fmaf((float)hh01[1], -1.0f, xt[1]));
      const unsigned l23 = pack_h2(fmaf((float)hh23[0], -1.0f, xt[2]),
                                   fmaf((float)hh23[1], -1.0f, xt[3]));
      xxp = fmaf(xt[0], xt[0], xxp);
      xxp = fmaf(xt[1], xt[1], xxp);
      xxp = fmaf(xt[2], xt[2], xxp);
      xxp = fmaf(xt[3], xt[3], xxp);
      u4v w1 = {h01, h23, l01, l23};
      u4v w2 = {h01, h23, c == 0 ? one01 : 0u, c == 0 ? one2 : 0u};
      b1[c] = __builtin_bit_cast(h8, w1);
      b2[c] = __builtin_bit_cast(h8, w2);
    }
    {
      auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(xxp), __float_as_uint(xxp),
                                                  false, false);
      xxp = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
      auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(xxp), __float_as_uint(xxp),
                                                  false, false);
      xxp = __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
    }
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      acc[t] = f4{xxp, xxp, xxp, xxp};
#pragma unroll
      for (int c = 0; c < DCH; ++c) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1[t][c], b1[c], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A2[t][c], b2[c], acc[t], 0, 0, 0);
      }
    }
    return xxp;
  };

  // (best, runner-up) keys of the lane's 4*KT screen values: value bits with
  // the low 6 replaced by the row index 16t + r (the lane group's 4g is added
  // once per group); values taken in pairs, b = min3, s = min(s, med3)
  auto tile_top2 = [&](const f4 (&acc)[KT], unsigned& bk, unsigned& sk) {
    auto key = [&](int t, int r) {
      return (__float_as_uint(acc[t][r]) & ~63u) | (unsigned)(16 * t + r);
    };
    auto chain = [&](int t0, int t1, unsigned& b, unsigned& s) {
      const unsigned k0 = key(t0, 0), k1 = key(t0, 1);
      b = min(k0, k1);
      s = max(k0, k1);
#pragma unroll
      for (int q = 2; q < 4 * (t1 - t0); q += 2) {
        const unsigned x = key(t0 + q / 4, q & 3), y = key(t0 + q / 4, (q & 3) + 1);
        s = min(s, umed3(b, x, y));
        b = min(min(b, x), y);
      }
    };
    if constexpr (KT >= 2) {  // two independent chains, one merge
      unsigned b2, s2;
      chain(0, KT / 2, bk, sk);
      chain(KT / 2, KT, b2, s2);
      merge_top2(bk, sk, b2, s2);
    } else {
      chain(0, 1, bk, sk);
    }
  };

  auto process = [&](const f4v (&buf)[4][DCH], int64_t grp) {
    const int64_t base = grp << 6;
    if (base >= a.n) return;  // wave-uniform: padding group
    unsigned bk[4], sk[4];
    float xx[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      f4 acc[KT];
      xx[p] = screen_tile(buf[p], acc);
      if constexpr ((ablate & 2) != 0) {  // no argmin / update
        float z = xx[p];
#pragma unroll
        for (int t = 0; t < KT; ++t) z += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
        asm volatile("" ::"v"(z));
      } else {
        tile_top2(acc, bk[p], sk[p]);
        bk[p] |= (unsigned)g << 2;
      }
    }
    if constexpr ((ablate & 2) != 0) return;
    // 4x4 transpose-reduce across lane groups: afterwards lane group g holds
    // the (best, runner-up) of tile g's point `col` (merges are symmetric,
    // so the swap orientation does not matter here)
    swap32(bk[0], bk[2]);
    swap32(sk[0], sk[2]);
    merge_top2(bk[0], sk[0], bk[2], sk[2]);
    swap32(bk[1], bk[3]);
    swap32(sk[1], sk[3]);
    merge_top2(bk[1], sk[1], bk[3], sk[3]);
    swap16(bk[0], bk[1]);
    swap16(sk[0], sk[1]);
    merge_top2(bk[0], sk[0], bk[1], sk[1]);
    const float xxg = g == 0 ? xx[0] : g == 1 ? xx[1] : g == 2 ? xx[2] : xx[3];
    const int64_t pt = base + 16 * g + col;  // < n_pad
    const int label = (int)(bk[0] & 63u);
    const float vb = __uint_as_float(bk[0] & ~63u);
    const float vs = __uint_as_float(sk[0] & ~63u);
    const bool cert = vs > fmaf(vb, 1.0f + 0x1p-15f, fmaf(thrA1, xxg, thrA0));
    a.labels[pt] = label;  // one coalesced 256-byte store per group
    const bool real = pt < a.n;
    const unsigned long long need = __ballot(real && !cert);
    if (need) {  // private region: no returning atomic, no vmcnt(0) stall
      const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(need >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((unsigned)need, 0u));
      if (real && !cert) fb_region[fb_used + rank] = (int32_t)pt;
      fb_used += __popcll(need);
    }
    if constexpr ((ablate & 1) != 0) return;  // no update
    // broadcast each tile's verdict (label, or -1) to all four lane groups
    unsigned v0 = (cert && real) ? (unsigned)label : 0xFFFFFFFFu;
    unsigned v1 = v0;
    swap16(v0, v1);  // rows (0,1): v0 = tile 0, v1 = tile 1; rows (2,3): tiles 2, 3
    unsigned v2 = v0, v3 = v1;
    swap32(v0, v2);  // v0 = tile 0, v2 = tile 2 in every lane
    swap32(v1, v3);  // v1 = tile 1, v3 = tile 3
    const unsigned vt[4] = {v0, v1, v2, v3};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int lp = (int)vt[p];
      if (lp >= 0) {
        unsigned long long* row = tbl + (size_t)lp * KS;
#pragma unroll
        for (int c = 0; c < DCH; ++c)
          if (qok[c]) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int u = (int)(buf[p][c][i] * fx);
              const unsigned long long v =
                  NONNEG ? (unsigned long long)(unsigned)u : (unsigned long long)(long long)u;
              atomicAdd(&row[16 * c + 4 * g + i], v);
            }
          }
        if (g == 0) atomicAdd(&row[d4], 1ull);
      }
    }
  };

  // one group in flight ahead of the one being processed
  f4v cur[4][DCH], nxt[4][DCH];
  if (G < ngroups) load(cur, G);
  // drain before the loop: otherwise the waitcnt pass merges this load into
  // the loop header state and puts a vmcnt wait for the freshly issued
  // prefetch in front of every tile (vmcnt(0), lgkmcnt/expcnt untouched)
  __builtin_amdgcn_s_waitcnt(0x0F70);
  for (; G < ngroups; G += gstride) {
    const int64_t Gn = G + gstride;
    if (Gn < ngroups) load(nxt, Gn);
    process(cur, G);
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int c = 0; c < DCH; ++c) cur[p][c] = nxt[p][c];
  }
  if (lane == 0) {
    a.fb_count[wave_id] = fb_used;
    if (fb_used) atomicAdd(a.fb_count + (int64_t)gstride, fb_used);
  }
  __syncthreads();
  unsigned long long* dst = a.partials + (size_t)blockIdx.x * a.k * KS;
  for (int i = threadIdx.x; i < a.k * KS; i += blockDim.x) dst[i] = tbl[i];
}

// Sum the per-workgroup tables: block (x, y) covers 64 entries and the y-th
// slice of the workgroups; 4 waves split that slice, combine in LDS and add
// into the (zeroed) output with one integer atomic per entry and slice.
constexpr int kReduceSlices = 16;
__global__ __launch_bounds__(256) void reduce_partials(const long long* __restrict__ part,
                                                       int nwg, int len, int d, int KS,
                                                       unsigned long long* __restrict__ out) {
  __shared__ long long red[4][64];
  const int e = blockIdx.x * 64 + (threadIdx.x & 63);  // (j, f) of the (k, d+1) output
  const int sub = threadIdx.x >> 6;
  const int per = (nwg + kReduceSlices - 1) / kReduceSlices;
  const int w0 = blockIdx.y * per, w1 = min(nwg, w0 + per);
  const int j = e / (d + 1), f = e % (d + 1);
  const int src = j * KS + (f < d ? f : KS - 1);
  const int slen = (len / (d + 1)) * KS;
  long long s = 0;
  if (e < len)
    for (int w = w0 + sub; w < w1; w += 4) s += part[(size_t)w * slen + src];
  red[sub][threadIdx.x & 63] = s;
  __syncthreads();
  if (sub == 0 && e < len) {
    const long long t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                        red[3][threadIdx.x];
    if (t) atomicAdd(&out[e], (unsigned long long)t);
  }
}

// Exact NumPy-order argmin over k centroids (row-major fp64 C).  sqrt is only
// evaluated when the squared distance drops, which keeps first-index ties of
// the *square roots* exactly as np.argmin(np.linalg.norm(...)) sees them.

// Wave-wide minimum, result in every lane: row_ror 8/4/2/1 inside each row of
// 16 lanes (DPP), then the permlane16 / permlane32 swaps across rows.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xF, 0xF, false);
  const unsigned hi =
      (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double wave_min_f64(double v) {
  v = fmin(v, dpp_f64<0x128>(v));
  v = fmin(v, dpp_f64<0x124>(v));
  v = fmin(v, dpp_f64<0x122>(v));
  v = fmin(v, dpp_f64<0x121>(v));
  auto mk = [](unsigned lo, unsigned hi) {
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
  };
  unsigned long long u = (unsigned long long)__double_as_longlong(v);
  auto l16 = __builtin_amdgcn_permlane16_swap((unsigned)u, (unsigned)u, false, false);
  auto h16 = __builtin_amdgcn_permlane16_swap((unsigned)(u >> 32), (unsigned)(u >> 32), false, false);
  v = fmin(mk(l16[0], h16[0]), mk(l16[1], h16[1]));
  u = (unsigned long long)__double_as_longlong(v);
  auto l32 = __builtin_amdgcn_permlane32_swap((unsigned)u, (unsigned)u, false, false);
  auto h32 = __builtin_amdgcn_permlane32_swap((unsigned)(u >> 32), (unsigned)(u >> 32), false, false);
  return fmin(mk(l32[0], h32[0]), mk(l32[1], h32[1]));
}
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
  v = min(v, (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false));
  v = min(v, (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false));
  v = min(v, (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x122, 0xF, 0xF, false));
  v = min(v, (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x121, 0xF, 0xF, false));
  auto r16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = min(r16[0], r16[1]);
  auto r32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return min(r32[0], r32[1]);
}

// Exact assignment of the points the screen did not certify: one wave per
// point, lane j computes the NumPy-order fp64 distance to centroids j, j+64,
// ... and its correctly rounded sqrt; first index on ties of the roots, as
// np.argmin sees them (reference src/kmeans_plusplus.py:33-34).  Workgroup b's
// waves take the screen's fallback regions 4b..4b+3, so the grid equals the
// screen's; lane f holds feature f of the point (prefetched one point ahead)
// and broadcasts it with readlane.  Sums go to an LDS table laid out like the
// screen's (row stride KS, count at KS-1), which is then added into the
// screen's partial row b — reduce_partials runs afterwards, so there are no
// global atomics.  CLDS: centroids staged transposed ([d][k]) in LDS.
// Requires d <= 64.
template <bool CLDS>
__global__ __launch_bounds__(256) void fallback_exact_wave(
    const float* __restrict__ X, int64_t n_pad, int d, const double* __restrict__ C, int k,
    const int32_t* __restrict__ list, const int32_t* __restrict__ count, int cap, int KS,
    int32_t* __restrict__ labels, unsigned long long* __restrict__ partials, float fx) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long* tbl = reinterpret_cast<unsigned long long*>(smem);
  double* ct = reinterpret_cast<double*>(tbl + (size_t)k * KS);
  const int tk = k * KS;
  for (int i = threadIdx.x; i < tk; i += blockDim.x) tbl[i] = 0ull;
  if (CLDS)
    for (int i = threadIdx.x; i < k * d; i += blockDim.x) {
      const int j = i / d, f = i - j * d;
      ct[f * k + j] = C[i];
    }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int reg = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int cnt = count[reg];
  const int32_t* lst = list + (size_t)reg * cap;
  auto cval = [&](int f, int j) -> double { return CLDS ? ct[f * k + j] : C[(size_t)j * d + f]; };
  int chunk = 0;  // list entries 64m .. 64m+63, one per lane
  int64_t pt = 0;
  float xf = 0.0f;
  if (cnt > 0) {
    chunk = lst[lane < cnt ? lane : 0];
    pt = __builtin_amdgcn_readfirstlane(chunk);
    if (lane < d) xf = X[xidx(X, lane, pt, n_pad)];
  }
  for (int e = 0; e < cnt; ++e) {
    const int64_t cpt = pt;
    const int cx = __float_as_int(xf);
    if (e + 1 < cnt) {  // prefetch the next point
      const int e1 = e + 1;
      if ((e1 & 63) == 0) chunk = lst[e1 + lane < cnt ? e1 + lane : e1];
      pt = __builtin_amdgcn_readlane(chunk, e1 & 63);
      if (lane < d) xf = X[xidx(X, lane, pt, n_pad)];
    }
    auto xv = [&](int f) { return (double)__int_as_float(__builtin_amdgcn_readlane(cx, f)); };
    double rb = INFINITY;
    int jb = k;
    for (int j = lane; j < k; j += 64) {
      const double r = sqrt(np_sqdist(xv, [&](int f) { return cval(f, j); }, d));
      if (r < rb) {  // j increases per lane: strict < keeps the first index
        rb = r;
        jb = j;
      }
    }
    const double m = wave_min_f64(rb);
    int jmin;
    if (k <= 64) {
      jmin = (int)__builtin_ctzll(__ballot(rb == m));  // lane == j
    } else {
      jmin = (int)wave_min_u32(rb == m ? (unsigned)jb : 0xFFFFFFFFu);
    }
    if (lane == 0) labels[cpt] = jmin;
    if (lane < d)
      atomicAdd(&tbl[(size_t)jmin * KS + lane],
                (unsigned long long)(long long)(int)(__int_as_float(cx) * fx));
    if (lane == 0) atomicAdd(&tbl[(size_t)jmin * KS + KS - 1], 1ull);  // d may be 64
  }
  __syncthreads();
  unsigned long long* dst = partials + (size_t)blockIdx.x * tk;
  for (int i = threadIdx.x; i < tk; i += blockDim.x) {
    const unsigned long long v = tbl[i];
    if (v) dst[i] += v;
  }
}

// Exact assignment of every point (F64 mode, or shapes the screen does not
// cover).  T = float (F32X storage) or double (F64 storage).
template <typename T>
__global__ void assign_exact_all(const T* __restrict__ X, int64_t n, int64_t n_pad, int d,
                                 const double* __restrict__ C, int k,
                                 int32_t* __restrict__ labels) {
  for (int64_t pt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; pt < n;
       pt += (int64_t)gridDim.x * blockDim.x) {
    auto xv = [&](int f) { return (double)X[xidx(X, f, pt, n_pad)]; };
    labels[pt] = exact_argmin(xv, C, k, d);
  }
}

// The same with the point's d <= 16 features loaded into registers once
// (assign_exact_all re-reads them from memory for every centroid) and the
// NumPy-order distance unrolled for that d; the centroid values are uniform
// (scalar) loads.
template <typename T, int D>
__global__ __launch_bounds__(256) void assign_exact_d(const T* __restrict__ X, int64_t n,
                                                      int64_t n_pad,
                                                      const double* __restrict__ C, int k,
                                                      int32_t* __restrict__ labels) {
  for (int64_t pt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; pt < n;
       pt += (int64_t)gridDim.x * blockDim.x) {
    double xr[D];
#pragma unroll
    for (int f = 0; f < D; ++f) xr[f] = (double)X[xidx(X, f, pt, n_pad)];
    labels[pt] = exact_argmin([&](int f) { return xr[f]; }, C, k, D);
  }
}

template <typename T>
static void launch_assign_exact(const T* X, int64_t n, int64_t n_pad, int d, const double* C,
                                int k, int32_t* labels, int cus, hipStream_t st) {
  typedef void (*Fn)(const T*, int64_t, int64_t, const double*, int, int32_t*);
#define CDR_AE(D_) assign_exact_d<T, D_>
  static const Fn fns[17] = {nullptr,     CDR_AE(1),  CDR_AE(2),  CDR_AE(3),  CDR_AE(4),
                             CDR_AE(5),   CDR_AE(6),  CDR_AE(7),  CDR_AE(8),  CDR_AE(9),
                             CDR_AE(10),  CDR_AE(11), CDR_AE(12), CDR_AE(13), CDR_AE(14),
                             CDR_AE(15),  CDR_AE(16)};
#undef CDR_AE
  const dim3 grid(std::max(1, (int)std::min<int64_t>(ceil_div(n, 256), (int64_t)cus * 8)));
  if (d >= 1 && d <= 16)
    hipLaunchKernelGGL(fns[d], grid, dim3(256), 0, st, X, n, n_pad, C, k, labels);
  else
    hipLaunchKernelGGL(assign_exact_all<T>, grid, dim3(256), 0, st, X, n, n_pad, d, C, k, labels);
  HIP_CHECK(hipGetLastError());
}

// Fixed-point sums from labels (F32X shapes without the screen): LDS table per
// workgroup, plain stores of the table, reduce_partials afterwards.
__global__ __launch_bounds__(256) void update_from_labels_f32x(
    const float* __restrict__ X, int64_t n, int64_t n_pad, int d, int k,
    const int32_t* __restrict__ labels, float fx, unsigned long long* __restrict__ partials) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long* tbl = reinterpret_cast<unsigned long long*>(smem);
  const int kd1 = d + 1;
  for (int i = threadIdx.x; i < k * kd1; i += blockDim.x) tbl[i] = 0ull;
  __syncthreads();
  for (int64_t pt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; pt < n;
       pt += (int64_t)gridDim.x * blockDim.x) {
    const int j = labels[pt];
    unsigned long long* row = tbl + (size_t)j * kd1;
    for (int f = 0; f < d; ++f)
      atomicAdd(&row[f], (unsigned long long)(long long)(int)(X[xidx(X, f, pt, n_pad)] * fx));
    atomicAdd(&row[d], 1ull);
  }
  __syncthreads();
  unsigned long long* dst = partials + (size_t)blockIdx.x * k * kd1;
  for (int i = threadIdx.x; i < k * kd1; i += blockDim.x) dst[i] = tbl[i];
}

// F64 mode: sums[j][f] = row-ordered fp64 sum of X[labels == j][:, f] and
// counts[j].  One thread per (j, f); f == d counts.  d == 1 follows NumPy's
// contiguous reduction instead: blocked (8192) pairwise over the selection.
__global__ void seq_sums_f64(const double* __restrict__ X, int64_t n, int64_t n_pad, int d,
                             int k, const int32_t* __restrict__ labels,
                             const long long* __restrict__ counts_in,
                             double* __restrict__ sums, long long* __restrict__ counts) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= k * (d + 1)) return;
  const int j = t / (d + 1), f = t % (d + 1);
  if (f == d) {
    long long c = 0;
    for (int64_t i = 0; i < n; ++i) c += (labels[i] == j);
    counts[j] = c;
    return;
  }
  auto col = [&](int64_t i) { return X[xidx(X, f, i, n_pad)]; };
  if (d >= 2) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i)
      if (labels[i] == j) s = s + col(i);
    sums[(size_t)j * d + f] = s;
    return;
  }
  // d == 1: res = 0; res += pairwise(block) for each 8192-block of the selection.
  const long long m = counts_in[j];
  int64_t cursor = 0;
  auto next = [&](int64_t) -> double {
    while (labels[cursor] != j) ++cursor;
    return col(cursor++);
  };
  double res = 0.0;
  for (long long done = 0; done < m; done += kSeedBlock) {
    const long long blk = (m - done) < kSeedBlock ? (m - done) : kSeedBlock;
    res = res + np_pairwise(next, blk);
  }
  sums[j] = res;
}

// Cluster sizes of the labels: one LDS histogram per wave (k <= kCountLds),
// added into the global counts once per (workgroup, cluster).  (One global
// atomic per point serialised on the k addresses: 28 ms at 10M points, k = 16.)
constexpr int kCountLds = 4096;
__global__ __launch_bounds__(256) void count_labels(const int32_t* __restrict__ labels, int64_t n,
                                                    int k, unsigned long long* __restrict__ counts) {
  extern __shared__ unsigned hist[];  // [4 waves][k] when k <= kCountLds
  const bool lds = k <= kCountLds;
  if (lds) {
    for (int i = threadIdx.x; i < 4 * k; i += blockDim.x) hist[i] = 0u;
    __syncthreads();
  }
  unsigned* wh = hist + (threadIdx.x >> 6) * k;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int l = labels[i];
    if (lds) atomicAdd(&wh[l], 1u);
    else atomicAdd(&counts[l], 1ull);
  }
  if (!lds) return;
  __syncthreads();
  for (int j = threadIdx.x; j < k; j += blockDim.x) {
    const unsigned long long v = (unsigned long long)hist[j] + hist[k + j] + hist[2 * k + j] +
                                 hist[3 * k + j];
    if (v) atomicAdd(&counts[j], v);
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
int lloyd_num_cus(int device) {
  static int cached[64] = {0};
  if (device >= 0 && device < 64 && cached[device]) return cached[device];
  int v = 0;
  HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device));
  if (device >= 0 && device < 64) cached[device] = v;
  return v;
}

struct ScreenPlan {
  int DCH, KT;
  bool pack6, fast;
  float thrA0, thrA1;
  std::vector<h8> frag;
};

// Build the fp16 A-operand fragments and the certification constants
// (derivation: DESIGN.md §3 "screen error bound").
static void build_screen_plan(const Ctx& c, const double* C, int k, ScreenPlan& pl,
                              bool allow_fast = true) {
  const int d = c.d;
  pl.DCH = (d + 15) / 16;
  pl.KT = (k + 15) / 16;
  pl.pack6 = pl.KT <= 4;
  const double sc = std::ldexp(1.0, c.sigma);
  std::vector<double> ch((size_t)k * d);
  double ccmax = 0.0;
  std::vector<double> cc(k, 0.0);
  for (int j = 0; j < k; ++j) {
    double s = 0.0;
    for (int f = 0; f < d; ++f) {
      const double v = (C[(size_t)j * d + f] - (double)c.mu[f]) * sc;
      ch[(size_t)j * d + f] = v;
      s += v * v;
    }
    cc[j] = s;
    ccmax = std::fmax(ccmax, s);
  }
  const double u = std::ldexp(1.0, -24);
  const double N = 64.0 * pl.DCH + 1.0;
  // factor 2 on the accumulation term: no assumption on the MFMA's internal
  // rounding beyond "each of its N additions errs by at most 2u".
  const double a = (2.0 * 2.02 * N + 14.0) * u;
  const double b = (4.04 * d + 8.0) * u + std::ldexp(1.0, -30);
  const double xxmax = d * (1.0 + 1e-6);
  const double eps = a * (ccmax + xxmax) + b;
  const double ccp = ccmax + eps;
  pl.thrA0 = (float)(2.02 * (a * ccp + b) + std::ldexp(ccp, -40));
  pl.thrA1 = (float)(2.02 * a * (1.0 + std::ldexp(1.0, -10)) + std::ldexp(1.0, -40));
  pl.thrA0 *= 1.0001f;
  pl.thrA1 *= 1.0001f;

  pl.fast = allow_fast && pl.KT * pl.DCH <= 4;
  pl.frag.assign((size_t)pl.KT * pl.DCH * 2 * 64, h8{});
  for (int t = 0; t < pl.KT; ++t)
    for (int cch = 0; cch < pl.DCH; ++cch)
      for (int lane = 0; lane < 64; ++lane) {
        const int j = 16 * t + (lane & 15);
        const int g = lane >> 4;
        h8 A1 = {}, A2 = {};
        // k-slot of (feature i, part): fast kernel [hi0..3 | lo0..3],
        // generic kernel interleaved [hi0, lo0, hi1, lo1, ...]
        auto slot_hi = [&](int i) { return pl.fast ? i : 2 * i; };
        auto slot_lo = [&](int i) { return pl.fast ? 4 + i : 2 * i + 1; };
        auto slot_ex = [&](int e) { return pl.fast ? 4 + e : 2 * e + 1; };
        for (int i = 0; i < 4; ++i) {
          const int f = 16 * cch + 4 * g + i;
          if (j < k && f < d) {
            const double v = ch[(size_t)j * d + f];
            const _Float16 hi = (_Float16)v;
            const _Float16 lo = (_Float16)(v - (double)hi);
            A1[slot_hi(i)] = (_Float16)(-2.0 * (double)hi);
            A1[slot_lo(i)] = (_Float16)(-2.0 * (double)hi);
            A2[slot_hi(i)] = (_Float16)(-2.0 * (double)lo);
          }
        }
        if (cch == 0) {
          if (g == 0) {
            A2[slot_ex(0)] = A2[slot_ex(1)] = A2[slot_ex(2)] = (_Float16)1.0f;
          } else if (g == 1) {
            if (j < k) {
              const double v = cc[j] + eps;
              const _Float16 p0 = (_Float16)v;
              const double r1 = v - (double)p0;
              const _Float16 p1 = (_Float16)r1;
              const double r2 = r1 - (double)p1;
              const _Float16 p2 = (_Float16)r2;
              A2[slot_ex(0)] = p0;
              A2[slot_ex(1)] = p1;
              A2[slot_ex(2)] = p2;
            } else {
              A2[slot_ex(0)] = (_Float16)30000.0f;  // padding centroid: never the best
            }
          }
        }
        pl.frag[(((size_t)t * pl.DCH + cch) * 2 + 0) * 64 + lane] = A1;
        pl.frag[(((size_t)t * pl.DCH + cch) * 2 + 1) * 64 + lane] = A2;
      }
}

template <int DCH, int KT>
static void launch_fast(bool nonneg, bool full, dim3 grid, size_t lds, hipStream_t s,
                        const ScreenArgs& a) {
  if (nonneg) {
    if (full) hipLaunchKernelGGL((screen_fast<DCH, KT, true, true>), grid, dim3(256), lds, s, a);
    else hipLaunchKernelGGL((screen_fast<DCH, KT, true, false>), grid, dim3(256), lds, s, a);
  } else {
    if (full) hipLaunchKernelGGL((screen_fast<DCH, KT, false, true>), grid, dim3(256), lds, s, a);
    else hipLaunchKernelGGL((screen_fast<DCH, KT, false, false>), grid, dim3(256), lds, s, a);
  }
}

static int fast_blocks_per_cu(int DCH, int KT, size_t lds) {
  int nb = 0;
  hipError_t e = hipErrorInvalidValue;
#define CDR_OCC(D, K)                                                                      \
  if (DCH == D && KT == K)                                                                  \
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, screen_fast<D, K, true, true>, 256, \
                                                     lds);
  CDR_OCC(1, 1) CDR_OCC(1, 2) CDR_OCC(1, 3) CDR_OCC(1, 4) CDR_OCC(2, 1) CDR_OCC(2, 2)
  CDR_OCC(3, 1) CDR_OCC(4, 1)
#undef CDR_OCC
  if (e != hipSuccess || nb < 1) nb = 2;
  return nb > 8 ? 8 : nb;
}

static void dispatch_fast(int DCH, int KT, bool nonneg, bool full, dim3 grid, size_t lds,
                          hipStream_t s, const ScreenArgs& a) {
#ifdef CDR_EXPERIMENTS
  if (a.ablate && DCH == 1 && KT == 4 && nonneg && full) {  // timing experiments
    switch (a.ablate) {
      case 1: hipLaunchKernelGGL((screen_fast<1, 4, true, true, 1>), grid, dim3(256), lds, s, a); return;
      case 2: hipLaunchKernelGGL((screen_fast<1, 4, true, true, 2>), grid, dim3(256), lds, s, a); return;
      case 8: hipLaunchKernelGGL((screen_fast<1, 4, true, true, 8>), grid, dim3(256), lds, s, a); return;
      case 9: hipLaunchKernelGGL((screen_fast<1, 4, true, true, 9>), grid, dim3(256), lds, s, a); return;
      case 10: hipLaunchKernelGGL((screen_fast<1, 4, true, true, 10>), grid, dim3(256), lds, s, a); return;
      case 16: hipLaunchKernelGGL((screen_fast<1, 4, true, true, 0, 2>), grid, dim3(256), lds, s, a); return;
      case 18: hipLaunchKernelGGL((screen_fast<1, 4, true, true, 0, 1>), grid, dim3(256), lds, s, a); return;
      default: break;
    }
  }
#endif
  if (DCH == 1 && KT == 1) launch_fast<1, 1>(nonneg, full, grid, lds, s, a);
  else if (DCH == 1 && KT == 2) launch_fast<1, 2>(nonneg, full, grid, lds, s, a);
  else if (DCH == 1 && KT == 3) launch_fast<1, 3>(nonneg, full, grid, lds, s, a);
  else if (DCH == 1 && KT == 4) launch_fast<1, 4>(nonneg, full, grid, lds, s, a);
  else if (DCH == 2 && KT == 1) launch_fast<2, 1>(nonneg, full, grid, lds, s, a);
  else if (DCH == 2 && KT == 2) launch_fast<2, 2>(nonneg, full, grid, lds, s, a);
  else if (DCH == 3 && KT == 1) launch_fast<3, 1>(nonneg, full, grid, lds, s, a);
  else launch_fast<4, 1>(nonneg, full, grid, lds, s, a);
}

template <int DCH>
static void launch_screen(bool pack6, bool dbg, dim3 grid, size_t lds, hipStream_t s,
                          const ScreenArgs& a) {
  if (dbg) {
    if (pack6) hipLaunchKernelGGL((screen_kernel<DCH, true, true>), grid, dim3(256), lds, s, a);
    else hipLaunchKernelGGL((screen_kernel<DCH, false, true>), grid, dim3(256), lds, s, a);
  } else {
    if (pack6) hipLaunchKernelGGL((screen_kernel<DCH, true, false>), grid, dim3(256), lds, s, a);
    else hipLaunchKernelGGL((screen_kernel<DCH, false, false>), grid, dim3(256), lds, s, a);
  }
}

static size_t screen_lds_bytes(int KT, int DCH, int k, int d) {
  return (size_t)KT * DCH * 2 * 64 * sizeof(h8) + (size_t)k * (d + 1) * 8;
}

bool screen_supported(const Ctx& c, int k) {
  const int DCH = (c.d + 15) / 16, KT = (k + 15) / 16;
  return c.d <= 64 && DCH <= 4 && screen_lds_bytes(KT, DCH, k, c.d) <= 64 * 1024;
}

// Upload centroids (row-major fp64) for the exact kernels.
static void upload_centroids(Ctx& c, const double* C, int k) {
  c.cent64.ensure(sizeof(double) * (size_t)k * c.d);
  HIP_CHECK(hipMemcpyAsync(c.cent64.p, C, sizeof(double) * (size_t)k * c.d,
                           hipMemcpyHostToDevice, c.stream));
}

static void check_k(const Ctx& c, int k) {
  if (c.mode == 0) CDR_FAIL(CDR_ERR_STATE, "no points loaded");
  if (k < 1) CDR_FAIL(CDR_ERR_ARG, "k must be >= 1");
  if (c.d > 128) CDR_FAIL(CDR_ERR_UNSUPPORTED, "d > 128 is not supported yet");
}

float* g_dbg_ptr = nullptr;  // set by cdr_debug_screen (tests only)
float g_dbg_thr[2] = {0.f, 0.f};

bool screen32_supported(const Ctx& c, int k);
bool big_step(Ctx& c, const double* C, int k, long long* dout, bool prof);
bool screen32_step(Ctx& c, const double* C, int k, long long* dout, long long* hout, bool prof,
                   float* dbg, float* thr_out, long long* gate);

// Adds a screen's published fallback total to the profiling accumulator.
__global__ void fb_accumulate(const int32_t* __restrict__ total, long long* __restrict__ acc) {
  if (threadIdx.x == 0) acc[0] += total[0];
}

bool prof_step_begin(Ctx& c) {
  c.prof_cur = -1;
  if (!c.prof_on) return false;
  if (c.prof_seen++ % c.prof_period != 0) return false;
  if (c.prof_used + 4 > (size_t)(4 << 16)) return false;  // session cap: 65536 steps
  while (c.prof_pool.size() < c.prof_used + 4) {
    hipEvent_t e = nullptr;
    HIP_CHECK(hipEventCreate(&e));
    c.prof_pool.push_back(e);
  }
  c.prof_cur = (int64_t)c.prof_used;
  c.prof_used += 4;
  c.prof_sub.resize(c.prof_used / 4);
  c.prof_sub[c.prof_used / 4 - 1] = 0;
  return true;
}

void prof_mark(Ctx& c, int i) {
  if (c.prof_cur >= 0) HIP_CHECK(hipEventRecord(c.prof_pool[(size_t)c.prof_cur + i], c.stream));
}

void prof_mark_sub(Ctx& c) {
  if (c.prof_cur < 0) return;
  HIP_CHECK(hipEventRecord(c.prof_pool[(size_t)c.prof_cur + 3], c.stream));
  c.prof_sub[(size_t)c.prof_cur / 4] = 1;
}

// End of a profiled screened step whose fallback total sits in fb_count
// (screen_big levels): fold it into the profile, then the closing mark.
void prof_end_screened(Ctx& c) {
  if (c.prof_cur < 0) return;
  c.fb_accum.ensure(2 * sizeof(long long));
  hipLaunchKernelGGL(fb_accumulate, dim3(1), dim3(64), 0, c.stream,
                     c.fb_count.as<int32_t>() + c.fb_total_slot, c.fb_accum.as<long long>());
  HIP_CHECK(hipGetLastError());
  prof_mark(c, 2);
}

// Fold every recorded step's events into the profile accumulators (waits
// for the last one).
void prof_collect(Ctx& c) {
  if (c.prof_used == 0) return;
  HIP_CHECK(hipEventSynchronize(c.prof_pool[c.prof_used - 2]));  // (the last step's end)
  for (size_t t = 0; t + 4 <= c.prof_used; t += 4) {
    float a = 0.f, b = 0.f;
    HIP_CHECK(hipEventElapsedTime(&a, c.prof_pool[t], c.prof_pool[t + 1]));
    HIP_CHECK(hipEventElapsedTime(&b, c.prof_pool[t], c.prof_pool[t + 2]));
    c.prof_screen_ms += a;
    c.prof_step_ms += b;
    c.prof_launches += 1;
    if (c.prof_sub[t / 4]) {
      float s = 0.f;
      HIP_CHECK(hipEventElapsedTime(&s, c.prof_pool[t], c.prof_pool[t + 3]));
      c.prof_sub_ms += s;
      c.prof_sub_launches += 1;
    }
  }
  c.prof_used = 0;
  c.prof_cur = -1;
}

void lloyd_step_f32x(Ctx& c, const double* C, int32_t k, int64_t* out, bool out_dev) {
  check_k(c, k);
  if (c.mode != CDR_MODE_F32X) CDR_FAIL(CDR_ERR_STATE, "lloyd_step: points are not F32X");
  const int d = c.d, kd1 = d + 1, len = k * kd1;
  long long* dout;
  if (out_dev) {
    dout = reinterpret_cast<long long*>(out);
  } else {
    c.out_sums.ensure(sizeof(long long) * len);
    dout = c.out_sums.as<long long>();
  }
  const float fx = (float)std::ldexp(1.0, c.scale_bits);
  const int cus = lloyd_num_cus(c.device);

  const bool prof = prof_step_begin(c);
  bool screened = false;
  // screen32 uploads its own operands (one pinned copy) and leaves the totals
  // in c.run_sums; it copies them to a device `out` itself
  // host path: screen32 publishes the sums and the fallback total straight
  // into mapped pinned memory (h_small)
  if (!out_dev) c.h_small.ensure(sizeof(long long) * (len + 1) + 64);
  // CDR_EXACT_ASSIGN=1 (read per step; tests): the exact fp64 NumPy-order
  // assignment of every point (assign_exact_all), no screen
  const bool exact_only = std::getenv("CDR_EXACT_ASSIGN") && std::atoi(std::getenv("CDR_EXACT_ASSIGN"));
  bool s32 = !exact_only && screen32_supported(c, k) &&
             screen32_step(c, C, k, out_dev ? dout : nullptr,
                           out_dev ? nullptr : c.h_small.as<long long>(), prof, g_dbg_ptr,
                           g_dbg_ptr ? g_dbg_thr : nullptr, nullptr);
  if (!s32) {
    upload_centroids(c, C, k);
    HIP_CHECK(hipMemsetAsync(dout, 0, sizeof(long long) * len, c.stream));
    c.fb_list.ensure(sizeof(int32_t) * (c.n > 0 ? c.n : 1));
  }
  if (s32) {
    screened = true;
  } else if (!exact_only && screen_supported(c, k)) {
    c.run_valid = false;  // the screen_fast / screen_kernel path keeps no running sums
    c.lab8_valid = false;
    c.zb_valid = false;
    c.big_valid = false;
    screened = true;
    ScreenPlan pl;
    build_screen_plan(c, C, k, pl, g_dbg_ptr == nullptr);
    c.frag.ensure(pl.frag.size() * sizeof(h8));
    HIP_CHECK(hipMemcpyAsync(c.frag.p, pl.frag.data(), pl.frag.size() * sizeof(h8),
                             hipMemcpyHostToDevice, c.stream));
    const int d4 = d4_of(d);
    const int KS = pl.fast ? d4 + 1 : kd1;
    const size_t lds = pl.fast ? (size_t)k * KS * 8 : screen_lds_bytes(pl.KT, pl.DCH, k, d);
    const int64_t groups = c.n_pad / 64;
    int nwg;
    if (pl.fast) {
      int bpc = fast_blocks_per_cu(pl.DCH, pl.KT, lds);
      nwg = (int)std::min<int64_t>(ceil_div(groups, 4), (int64_t)cus * bpc);
    } else {
      nwg = (int)std::min<int64_t>(ceil_div(groups, 4), (int64_t)cus * 4);
    }
    if (nwg < 1) nwg = 1;
    c.partials.ensure(sizeof(long long) * (size_t)nwg * k * KS);
    const int nwaves = nwg * 4;
    const int cap = (int)(ceil_div(groups, nwaves) * 64);
    c.fb_list.ensure(sizeof(int32_t) * (size_t)nwaves * cap);
    c.fb_count.ensure(sizeof(int32_t) * (nwaves + 1));
    HIP_CHECK(hipMemsetAsync(c.fb_count.p, 0, sizeof(int32_t) * (nwaves + 1), c.stream));
    c.fb_regions = nwaves;
    c.fb_total_slot = nwaves;
    c.fb_layout = -1;  // screen32 must re-zero its counter layout
    ScreenArgs a;
    a.X = c.x32.as<float>();
    a.n = c.n;
    a.n_pad = c.n_pad;
    a.d = d;
    a.k = k;
    a.KT = pl.KT;
    a.frag = c.frag.as<h8>();
    a.mu_s = c.mu_s.as<float>();
    a.sig = (float)std::ldexp(1.0, c.sigma);
    a.fx = fx;
    a.thrA0 = pl.thrA0;
    a.thrA1 = pl.thrA1;
    a.labels = c.labels.as<int32_t>();
    a.partials = c.partials.as<unsigned long long>();
    a.fb_list = c.fb_list.as<int32_t>();
    a.fb_count = c.fb_count.as<int32_t>();
    a.fb_cap = cap;
    a.dbg = g_dbg_ptr;
#ifdef CDR_EXPERIMENTS
    a.ablate = c.screen_ablate;
#else
    a.ablate = 0;
#endif
    const bool dbg = g_dbg_ptr != nullptr;
    if (pl.fast)
      snprintf(c.prof_kernel, sizeof(c.prof_kernel), "screen_fast<%d,%d>", pl.DCH, pl.KT);
    else
      snprintf(c.prof_kernel, sizeof(c.prof_kernel), "screen_kernel<%d>", pl.DCH);
    if (prof) prof_mark(c, 0);
    if (pl.fast) {
      bool nonneg = true;
      for (int f = 0; f < d; ++f) nonneg = nonneg && c.fmin[f] >= 0.0;
      dispatch_fast(pl.DCH, pl.KT, nonneg, d4 == 16 * pl.DCH, dim3(nwg), lds, c.stream, a);
    } else {
      switch (pl.DCH) {
        case 1: launch_screen<1>(pl.pack6, dbg, dim3(nwg), lds, c.stream, a); break;
        case 2: launch_screen<2>(pl.pack6, dbg, dim3(nwg), lds, c.stream, a); break;
        case 3: launch_screen<3>(pl.pack6, dbg, dim3(nwg), lds, c.stream, a); break;
        default: launch_screen<4>(pl.pack6, dbg, dim3(nwg), lds, c.stream, a); break;
      }
    }
    HIP_CHECK(hipGetLastError());
    if (prof) prof_mark(c, 1);
    // fallback first: it adds into the screen's partial rows
    const size_t fb_lds = (size_t)k * KS * 8;
    const size_t fb_lds_c = fb_lds + (size_t)k * d * 8;
    if (fb_lds_c <= 64 * 1024)
      hipLaunchKernelGGL(fallback_exact_wave<true>, dim3(nwg), dim3(256), fb_lds_c, c.stream,
                         c.x32.as<float>(), c.n_pad, d, c.cent64.as<double>(), k,
                         c.fb_list.as<int32_t>(), c.fb_count.as<int32_t>(), cap, KS,
                         c.labels.as<int32_t>(), c.partials.as<unsigned long long>(), fx);
    else
      hipLaunchKernelGGL(fallback_exact_wave<false>, dim3(nwg), dim3(256), fb_lds, c.stream,
                         c.x32.as<float>(), c.n_pad, d, c.cent64.as<double>(), k,
                         c.fb_list.as<int32_t>(), c.fb_count.as<int32_t>(), cap, KS,
                         c.labels.as<int32_t>(), c.partials.as<unsigned long long>(), fx);
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(reduce_partials, dim3((len + 63) / 64, kReduceSlices), dim3(256), 0,
                       c.stream, c.partials.as<long long>(), nwg, len, d,
                       KS, reinterpret_cast<unsigned long long*>(dout));
    HIP_CHECK(hipGetLastError());
  } else if (!exact_only && big_step(c, C, k, dout, prof)) {
    screened = true;  // large k / d: screen_big levels + update_big
  } else {
    c.run_valid = false;
    c.lab8_valid = false;
    c.zb_valid = false;
    c.big_valid = false;
    // exact assignment for every point, then fixed-point sums from labels
    launch_assign_exact<float>(c.x32.as<float>(), c.n, c.n_pad, d, c.cent64.as<double>(), k,
                               c.labels.as<int32_t>(), cus, c.stream);
    const size_t lds = (size_t)len * 8;
    if (lds > 64 * 1024) CDR_FAIL(CDR_ERR_UNSUPPORTED, "k*(d+1) too large for the update table");
    int nwg = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(c.n, 256), cus * 2));
    c.partials.ensure(sizeof(long long) * (size_t)nwg * len);
    hipLaunchKernelGGL(update_from_labels_f32x, dim3(nwg), dim3(256), lds, c.stream,
                       c.x32.as<float>(), c.n, c.n_pad, d, k, c.labels.as<int32_t>(), fx,
                       c.partials.as<unsigned long long>());
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(reduce_partials, dim3((len + 63) / 64, kReduceSlices), dim3(256), 0,
                       c.stream, c.partials.as<long long>(), nwg, len, d, kd1,
                       reinterpret_cast<unsigned long long*>(dout));
    HIP_CHECK(hipGetLastError());
  }
  c.last_screened = screened;
  if (prof) {
    if (!screened) {  // no screen kernel: an empty triple keeps the pairing
      prof_mark(c, 0);
      prof_mark(c, 1);
    } else if (!s32) {  // screen32's publish32 sums its fallback total itself
      c.fb_accum.ensure(2 * sizeof(long long));
      hipLaunchKernelGGL(fb_accumulate, dim3(1), dim3(64), 0, c.stream,
                         c.fb_count.as<int32_t>() + c.fb_total_slot, c.fb_accum.as<long long>());
      HIP_CHECK(hipGetLastError());
    }
    prof_mark(c, 2);
  }
  c.last_k = k;
  c.have_labels = true;
  if (!out_dev) {
    int32_t fb = 0;
    if (s32) {
      HIP_CHECK(hipStreamSynchronize(c.stream));
      fb = (int32_t)c.h_small.as<long long>()[len];
    } else {
      HIP_CHECK(hipMemcpyAsync(c.h_small.p, dout, sizeof(long long) * len,
                               hipMemcpyDeviceToHost, c.stream));
      int32_t* hfb = reinterpret_cast<int32_t*>(c.h_small.as<long long>() + len);
      *hfb = 0;
      if (screened)
        HIP_CHECK(hipMemcpyAsync(hfb, c.fb_count.as<int32_t>() + c.fb_total_slot,
                                 sizeof(int32_t), hipMemcpyDeviceToHost, c.stream));
      HIP_CHECK(hipStreamSynchronize(c.stream));
      fb = *hfb;
    }
    memcpy(out, c.h_small.p, sizeof(long long) * len);
    c.last_fallback = screened ? fb : c.n;
  } else {
    c.last_fallback = -1;  // unknown until cdr_lloyd_stats synchronises
  }
}

// The device-resident F64 run's update (one workgroup, after each fused
// step): means = sums / counts (np.mean's true division), shift =
// ||means - C|| (src/kmeans_plusplus.py:37-48).  The step is applied on the
// device when every cluster has members and the shift is clear of tol: C =
// means, and the run stops once shift < tol.  An empty cluster (the reference
// reseeds it from np.random) or a shift within 2^-36 of tol (the reference's
// BLAS summation order is not ours) stops the run WITHOUT applying the step:
// the host finishes that step from the kept means and counts.  The shift's
// square is summed in a fixed tree: <= 1024 non-negative terms, within 2^-42
// of any other order's, so the margin decides both sides rigorously.
constexpr int kF64RunThreads = 1024;
__global__ __launch_bounds__(kF64RunThreads) void f64_run_update(
    const double* __restrict__ sums, unsigned long long* __restrict__ counts,
    double* __restrict__ C, double* __restrict__ keep, int k, int d, double tol,
    long long* __restrict__ st) {
  __shared__ double red[kF64RunThreads / 64];
  __shared__ int empty_any;
  if (st[0] == 0) return;  // (uniform) stopped: this step's kernels ran for nothing
  const int t = threadIdx.x, kd = k * d;
  if (t == 0) empty_any = 0;
  __syncthreads();
  double m = 0.0, sq = 0.0;
  if (t < kd) {
    const unsigned long long cnt = counts[t / d];
    m = sums[t] / (double)cnt;
    if (cnt == 0) {
      empty_any = 1;
    } else {
      const double df = m - C[t];
      sq = df * df;
    }
    keep[t] = m;
    if (t % d == 0) reinterpret_cast<long long*>(keep + kd)[t / d] = (long long)cnt;
  }

#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
  if ((t & 63) == 0) red[t >> 6] = sq;
  __syncthreads();
  double ss = 0.0;
#pragma unroll
  for (int w = 0; w < kF64RunThreads / 64; ++w) ss += red[w];
  const double sh = sqrt(ss);
  const double mg = 0x1p-36;
  long long reason = 0;  // 0: applied, go on; 1: applied, converged; 2: the host's step
  if (empty_any) reason = 2;
  else if (tol > 0.0 && !(sh > tol * (1.0 + mg))) reason = sh < tol * (1.0 - mg) ? 1 : 2;
  if (reason != 2 && t < kd) C[t] = m;
  if (t == 0) {
    if (reason != 2) st[1] += 1;
    st[2] = reason;
    st[3] = __double_as_longlong(ss);
    if (reason != 0) st[0] = 0;
  }
}

// cdr_lloyd_f64_run: up to max_steps fused F64 steps (f64sum.hip) with the
// update above on the device; one synchronisation at the end.
void lloyd_run_f64(Ctx& c, const double* C, int32_t k, int32_t max_steps, double tol,
                   double* C_out, double* means_out, int64_t* counts_out, int32_t* info) {
  check_k(c, k);
  if (c.mode != CDR_MODE_F64) CDR_FAIL(CDR_ERR_STATE, "lloyd_run_f64: points are not F64");
  const int d = c.d;
  if (d < 2 || d > 16 || k > 64 || k * d > kF64RunThreads)
    CDR_FAIL(CDR_ERR_UNSUPPORTED, "device F64 run: needs 2 <= d <= 16 and k <= 64");
  if (max_steps < 0) CDR_FAIL(CDR_ERR_ARG, "max_steps < 0");
  c.run_valid = false;
  c.lab8_valid = false;
  c.zb_valid = false;
  c.big_valid = false;
  upload_centroids(c, C, k);
  const size_t kd = (size_t)k * d;
  c.f64_sums.ensure(sizeof(double) * kd);
  c.f64_counts.ensure(sizeof(long long) * k * 2);
  c.f64r_state.ensure(sizeof(long long) * 4);
  c.f64r_keep.ensure(sizeof(double) * kd + sizeof(long long) * k);
  c.h_small.ensure(sizeof(long long) * 4);
  long long* hst = c.h_small.as<long long>();
  hst[0] = 1;
  hst[1] = hst[2] = hst[3] = 0;
  long long* st = c.f64r_state.as<long long>();
  HIP_CHECK(hipMemcpyAsync(st, hst, sizeof(long long) * 4, hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipMemsetAsync(c.f64r_keep.p, 0, c.f64r_keep.bytes, c.stream));
  snprintf(c.prof_kernel, sizeof(c.prof_kernel), "f64_assign_block<%d>", d);
  // Steps are queued in chunks (4, 8, then 16 at a time) with the state word
  // read back between chunks: only f64_assign_block and f64_run_update test
  // it, so a run that stopped (converged, or handed to the host) would still
  // run the rest of every queued step's kernels.  One host sync
  // per chunk costs ~20 us against ~0.5 ms per step.
  int chunk = 4, queued = 0;
  // the transfer cache across the run's steps (f64_step_fused; the first step
  // forms every transfer).  CDR_F64_TCACHE=0 forms every transfer every step
  // (tests/test_gpu_f64_update.py compares the two).
  const char* tce = getenv("CDR_F64_TCACHE");
  const bool tc_on = !tce || std::atoi(tce) != 0;
  for (int s = 0; s < max_steps; ++s) {
    if (queued == chunk) {
      HIP_CHECK(hipMemcpyAsync(hst, st, sizeof(long long), hipMemcpyDeviceToHost, c.stream));
      HIP_CHECK(hipStreamSynchronize(c.stream));
      if (hst[0] == 0) break;
      queued = 0;
      chunk = chunk < 16 ? 2 * chunk : 16;
    }
    ++queued;
    const bool prof = prof_step_begin(c);
    if (prof) prof_mark(c, 0);
    if (!f64_step_fused(c, k, c.cent64.as<double>(), c.f64_sums.as<double>(),
                        reinterpret_cast<unsigned long long*>(c.f64_counts.as<long long>()), prof,
                        st, tc_on ? (s == 0 ? 1 : 2) : 0))
      CDR_FAIL(CDR_ERR_UNSUPPORTED, "device F64 run: shape not covered");
    hipLaunchKernelGGL(f64_run_update, dim3(1), dim3(kF64RunThreads), 0, c.stream,
                       c.f64_sums.as<double>(),
                       reinterpret_cast<unsigned long long*>(c.f64_counts.as<long long>()),
                       c.cent64.as<double>(), c.f64r_keep.as<double>(), k, d, tol, st);
    HIP_CHECK(hipGetLastError());
    if (prof) prof_mark(c, 2);
  }
  HIP_CHECK(hipMemcpyAsync(hst, st, sizeof(long long) * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(C_out, c.cent64.p, sizeof(double) * kd, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipMemcpyAsync(means_out, c.f64r_keep.p, sizeof(double) * kd, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipMemcpyAsync(counts_out, c.f64r_keep.as<double>() + kd, sizeof(long long) * k,
                           hipMemcpyDeviceToHost, c.stream));
  std::vector<long long> w(kd);
  HIP_CHECK(hipMemcpyAsync(w.data(), c.f64x_walk.p, sizeof(long long) * w.size(),
                           hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.f64x_walked = 0;
  for (long long v : w) c.f64x_walked += v;
  info[0] = (int32_t)hst[1];
  info[1] = max_steps == 0 ? 0 : (int32_t)hst[2];
  c.last_k = k;
  c.have_labels = max_steps > 0 || c.have_labels;
  c.last_fallback = c.n;
}

void lloyd_step_f64(Ctx& c, const double* C, int32_t k, double* sums, int64_t* counts) {
  check_k(c, k);
  if (c.mode != CDR_MODE_F64) CDR_FAIL(CDR_ERR_STATE, "lloyd_step_f64: points are not F64");
  c.run_valid = false;
  c.lab8_valid = false;
  c.zb_valid = false;
  c.big_valid = false;
  const int d = c.d;
  const int cus = lloyd_num_cus(c.device);
  upload_centroids(c, C, k);
  const bool prof = prof_step_begin(c);
  c.f64_sums.ensure(sizeof(double) * (size_t)k * d);
  c.f64_counts.ensure(sizeof(long long) * k * 2);
  long long* cnt_pre = c.f64_counts.as<long long>() + k;
  // the fused pipeline (f64sum.hip: assignment + block pass, transfers from
  // the previous step's binade predictions; CDR_F64_FUSE=0: separate passes)
  static const bool fuse_env = !exp_env("CDR_F64_FUSE") || atoi(exp_env("CDR_F64_FUSE"));
  if (fuse_env && !getenv("CDR_F64_SERIAL")) {
    snprintf(c.prof_kernel, sizeof(c.prof_kernel), "f64_assign_block<%d>", d);
    if (prof) prof_mark(c, 0);
    if (f64_step_fused(c, k, c.cent64.as<double>(), c.f64_sums.as<double>(),
                       reinterpret_cast<unsigned long long*>(c.f64_counts.as<long long>()),
                       prof)) {
      if (prof) prof_mark(c, 2);
      std::vector<long long> w((size_t)k * d);
      HIP_CHECK(hipMemcpyAsync(w.data(), c.f64x_walk.p, sizeof(long long) * w.size(),
                               hipMemcpyDeviceToHost, c.stream));
      HIP_CHECK(hipMemcpyAsync(sums, c.f64_sums.p, sizeof(double) * (size_t)k * d,
                               hipMemcpyDeviceToHost, c.stream));
      HIP_CHECK(hipMemcpyAsync(counts, c.f64_counts.p, sizeof(long long) * k,
                               hipMemcpyDeviceToHost, c.stream));
      HIP_CHECK(hipStreamSynchronize(c.stream));
      c.f64x_walked = 0;
      for (long long v : w) c.f64x_walked += v;
      c.last_k = k;
      c.have_labels = true;
      c.last_fallback = c.n;
      return;
    }
  }
  snprintf(c.prof_kernel, sizeof(c.prof_kernel),
           d <= 16 ? "assign_exact_d<double, %d>" : "assign_exact_all<double>", d);
  if (prof) prof_mark(c, 0);
  launch_assign_exact<double>(c.x64.as<double>(), c.n, c.n_pad, d, c.cent64.as<double>(), k,
                              c.labels.as<int32_t>(), cus, c.stream);
  if (prof) prof_mark(c, 1);
  HIP_CHECK(hipMemsetAsync(cnt_pre, 0, sizeof(long long) * k, c.stream));
  hipLaunchKernelGGL(count_labels, dim3(std::max(1, (int)std::min<int64_t>(ceil_div(c.n, 256), cus * 2))),
                     dim3(256), k <= kCountLds ? sizeof(unsigned) * 4 * k : 0, c.stream,
                     c.labels.as<int32_t>(), c.n, k, reinterpret_cast<unsigned long long*>(cnt_pre));
  HIP_CHECK(hipGetLastError());
  if (!getenv("CDR_F64_SERIAL") && f64_sums_parallel(c, k, c.f64_sums.as<double>())) {
    // f64sum.hip: exact row-order sums in parallel; counts from count_labels
    HIP_CHECK(hipMemcpyAsync(c.f64_counts.p, cnt_pre, sizeof(long long) * k,
                             hipMemcpyDeviceToDevice, c.stream));
    if (prof) prof_mark(c, 2);
    std::vector<long long> w((size_t)k * d);
    HIP_CHECK(hipMemcpyAsync(w.data(), c.f64x_walk.p, sizeof(long long) * w.size(),
                             hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    c.f64x_walked = 0;
    for (long long v : w) c.f64x_walked += v;
  } else {
    const int threads = k * (d + 1);
    hipLaunchKernelGGL(seq_sums_f64, dim3((threads + 63) / 64), dim3(64), 0, c.stream,
                       c.x64.as<double>(), c.n, c.n_pad, d, k, c.labels.as<int32_t>(), cnt_pre,
                       c.f64_sums.as<double>(), c.f64_counts.as<long long>());
    HIP_CHECK(hipGetLastError());
    if (prof) prof_mark(c, 2);
    c.f64x_walked = -1;
  }
  HIP_CHECK(hipMemcpyAsync(sums, c.f64_sums.p, sizeof(double) * (size_t)k * d,
                           hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(counts, c.f64_counts.p, sizeof(long long) * k,
                           hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.last_k = k;
  c.have_labels = true;
  c.last_fallback = c.n;
}

// ---------------------------------------------------------------------------
// The reference's float32 runs (X float32 keeps its dtype,
// src/kmeans_plusplus.py:6): distances are float32 norms in NumPy order with
// one rounded sqrt, np.argmin takes the first of equal float32 norms (:33-34),
// and X[mask].mean(axis=0) is a sequential float32 sum over the rows divided
// (in fp64, cast to fp32 by the caller) by the count (:41).
// ---------------------------------------------------------------------------
template <typename S, int D>
__global__ __launch_bounds__(256) void f32r_assign_kernel(const S* __restrict__ X, int64_t n,
                                                          int64_t n_pad, int d,
                                                          const float* __restrict__ C, int k,
                                                          int32_t* __restrict__ labels) {
  const int dd = D ? D : d;
  for (int64_t pt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; pt < n;
       pt += (int64_t)gridDim.x * blockDim.x) {
    float xr[D ? D : 1];
    if constexpr (D > 0) {
#pragma unroll
      for (int f = 0; f < D; ++f) xr[f] = (float)X[xidx(X, f, pt, n_pad)];
    }
    auto xv = [&](int f) { return D ? xr[D ? f : 0] : (float)X[xidx(X, f, pt, n_pad)]; };
    float Rb = INFINITY, rb = INFINITY;
    int jb = 0;
    for (int j = 0; j < k; ++j) {
      const float* cj = C + (size_t)j * dd;
      auto cv = [&](int f) { return cj[f]; };
      const float R = np_sqdist<decltype(xv), decltype(cv), float>(xv, cv, dd);
      if (R < Rb) {  // sqrt is monotone: only a smaller square can give a smaller norm
        const float r = (float)sqrt((double)R);  // the correctly rounded fp32 sqrt
        Rb = R;
        if (r < rb) {
          rb = r;
          jb = j;
        }
      }
    }
    labels[pt] = jb;
  }
}

// Serial form (k > 64 or d == 1): one thread per (cluster, feature); d == 1
// follows NumPy's contiguous reduction (8192-blocked pairwise, fp32).
template <typename S>
__global__ void f32r_seq_sums(const S* __restrict__ X, int64_t n, int64_t n_pad, int d, int k,
                              const int32_t* __restrict__ labels,
                              const long long* __restrict__ counts_in,
                              double* __restrict__ sums) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= k * d) return;
  const int j = t / d, f = t % d;
  auto col = [&](int64_t i) { return (float)X[xidx(X, f, i, n_pad)]; };
  if (d >= 2) {
    float s = 0.0f;
    bool any = false;
    for (int64_t i = 0; i < n; ++i)
      if (labels[i] == j) {
        s = any ? s + col(i) : col(i);
        any = true;
      }
    sums[(size_t)j * d + f] = (double)s;
    return;
  }
  const long long m = counts_in[j];
  int64_t cursor = 0;
  auto next = [&](int64_t) -> float {
    while (labels[cursor] != j) ++cursor;
    return col(cursor++);
  };
  float res = 0.0f;
  for (long long done = 0; done < m; done += kSeedBlock) {
    const long long blk = (m - done) < kSeedBlock ? (m - done) : kSeedBlock;
    res = res + np_pairwise<decltype(next), float>(next, blk);
  }
  sums[j] = (double)res;
}

void lloyd_step_f32r(Ctx& c, const float* C, int32_t k, double* sums, int64_t* counts) {
  check_k(c, k);
  c.run_valid = false;
  c.lab8_valid = false;
  c.zb_valid = false;
  c.big_valid = false;
  const int d = c.d;
  const int cus = lloyd_num_cus(c.device);
  c.cent32r.ensure(sizeof(float) * (size_t)k * d);
  HIP_CHECK(hipMemcpyAsync(c.cent32r.p, C, sizeof(float) * (size_t)k * d, hipMemcpyHostToDevice,
                           c.stream));
  const bool prof = prof_step_begin(c);
  snprintf(c.prof_kernel, sizeof(c.prof_kernel), "f32r_assign_kernel<%d>", d);
  if (prof) prof_mark(c, 0);
  const dim3 grid(std::max(1, (int)std::min<int64_t>(ceil_div(c.n, 256), (int64_t)cus * 8)));
  const float* dC = c.cent32r.as<float>();
  int32_t* lab = c.labels.as<int32_t>();
#define CDR_F32R_AS(S_, X_)                                                                      \
  switch (d) {                                                                                  \
    case 2: hipLaunchKernelGGL((f32r_assign_kernel<S_, 2>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dC, k, lab); break; \
    case 5: hipLaunchKernelGGL((f32r_assign_kernel<S_, 5>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dC, k, lab); break; \
    case 8: hipLaunchKernelGGL((f32r_assign_kernel<S_, 8>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dC, k, lab); break; \
    case 16: hipLaunchKernelGGL((f32r_assign_kernel<S_, 16>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dC, k, lab); break; \
    default: hipLaunchKernelGGL((f32r_assign_kernel<S_, 0>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dC, k, lab); \
  }
  if (c.mode == CDR_MODE_F32X) {
    CDR_F32R_AS(float, c.x32.as<float>())
  } else {
    CDR_F32R_AS(double, c.x64.as<double>())
  }
#undef CDR_F32R_AS
  HIP_CHECK(hipGetLastError());
  if (prof) prof_mark(c, 1);
  c.f64_sums.ensure(sizeof(double) * (size_t)k * d);
  c.f64_counts.ensure(sizeof(long long) * k * 2);
  long long* cnt_pre = c.f64_counts.as<long long>() + k;
  HIP_CHECK(hipMemsetAsync(cnt_pre, 0, sizeof(long long) * k, c.stream));
  hipLaunchKernelGGL(count_labels, dim3(std::max(1, (int)std::min<int64_t>(ceil_div(c.n, 256), cus * 2))),
                     dim3(256), k <= kCountLds ? sizeof(unsigned) * 4 * k : 0, c.stream,
                     c.labels.as<int32_t>(), c.n, k, reinterpret_cast<unsigned long long*>(cnt_pre));
  HIP_CHECK(hipGetLastError());
  if (!getenv("CDR_F64_SERIAL") && f32_sums_parallel(c, k, c.f64_sums.as<double>())) {
    c.f64x_walked = 0;
  } else {
    const int threads = k * d;
    if (c.mode == CDR_MODE_F32X)
      hipLaunchKernelGGL(f32r_seq_sums<float>, dim3((threads + 63) / 64), dim3(64), 0, c.stream,
                         c.x32.as<float>(), c.n, c.n_pad, d, k, c.labels.as<int32_t>(), cnt_pre,
                         c.f64_sums.as<double>());
    else
      hipLaunchKernelGGL(f32r_seq_sums<double>, dim3((threads + 63) / 64), dim3(64), 0, c.stream,
                         c.x64.as<double>(), c.n, c.n_pad, d, k, c.labels.as<int32_t>(), cnt_pre,
                         c.f64_sums.as<double>());
    HIP_CHECK(hipGetLastError());
    c.f64x_walked = -1;
  }
  if (prof) prof_mark(c, 2);
  HIP_CHECK(hipMemcpyAsync(sums, c.f64_sums.p, sizeof(double) * (size_t)k * d,
                           hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(counts, cnt_pre, sizeof(long long) * k, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.last_k = k;
  c.have_labels = true;
  c.last_fallback = c.n;
}

__global__ void labels_to_i64(const int32_t* __restrict__ a, int64_t n, long long* __restrict__ b) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

}  // namespace cdr

using namespace cdr;

extern "C" {

int cdr_lloyd_step(cdr_ctx* h, const double* C, int32_t k, int64_t* out,
                   int32_t out_on_device) {
  CDR_TRY
  if (!h || !C || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  lloyd_step_f32x(h->c, C, k, out, out_on_device != 0);
  CDR_CATCH
}

int cdr_lloyd_step_f64(cdr_ctx* h, const double* C, int32_t k, double* sums,
                       int64_t* counts) {
  CDR_TRY
  if (!h || !C || !sums || !counts) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  lloyd_step_f64(h->c, C, k, sums, counts);
  CDR_CATCH
}

int cdr_lloyd_f64_run(cdr_ctx* h, const double* C, int32_t k, int32_t max_steps, double tol,
                      double* C_out, double* means_out, int64_t* counts_out, int32_t* info) {
  CDR_TRY
  if (!h || !C || !C_out || !means_out || !counts_out || !info) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  lloyd_run_f64(h->c, C, k, max_steps, tol, C_out, means_out, counts_out, info);
  CDR_CATCH
}

// ---- sharded F64 sums (f64sum.hip, include/cdr.h cdr_f64s_*) ----
int cdr_f64s_begin(cdr_ctx* h, const double* C, int32_t k, int32_t nranks, int32_t rank,
                   void* tot_buf, int64_t* sizes) {
  CDR_TRY
  if (!h || !C || !tot_buf || !sizes) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  check_k(c, k);
  if (c.mode != CDR_MODE_F64) CDR_FAIL(CDR_ERR_STATE, "cdr_f64s_begin: points are not F64");
  if (nranks < 1 || rank < 0 || rank >= nranks) CDR_FAIL(CDR_ERR_ARG, "bad ranks");
  if (c.d < 2 || c.d > 16 || k > 64)
    CDR_FAIL(CDR_ERR_UNSUPPORTED, "sharded F64 sums need 2 <= d <= 16 and k <= 64");
  c.run_valid = false;
  c.lab8_valid = false;
  c.zb_valid = false;
  c.big_valid = false;
  upload_centroids(c, C, k);
  const int kd = k * c.d;
  double* slot = static_cast<double*>(tot_buf) + (size_t)rank * (kd + k);
  snprintf(c.prof_kernel, sizeof(c.prof_kernel), "f64_assign_block<%d>", c.d);
  const bool prof = prof_step_begin(c);
  if (prof) prof_mark(c, 0);
  if (!f64s_assign_totals(c, k, c.cent64.as<double>(), slot))
    CDR_FAIL(CDR_ERR_UNSUPPORTED, "sharded F64 sums: shape not covered");
  if (prof) prof_mark(c, 1);
  c.f64s_k = k;
  c.f64s_nranks = nranks;
  c.f64s_rank = rank;
  sizes[0] = (int64_t)sizeof(double) * (kd + k);
  sizes[1] = (int64_t)24 * kd * (f64s_cap() + 1);
  c.last_k = k;
  c.have_labels = true;
  CDR_CATCH
}

int cdr_f64s_build(cdr_ctx* h, const void* tot_buf, void* prog_buf) {
  CDR_TRY
  if (!h || !tot_buf || !prog_buf) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  if (c.f64s_k < 1) CDR_FAIL(CDR_ERR_STATE, "cdr_f64s_begin first");
  f64s_build(c, c.f64s_k, c.f64s_nranks, c.f64s_rank, static_cast<const double*>(tot_buf),
             prog_buf);
  CDR_CATCH
}

int cdr_f64s_finish(cdr_ctx* h, const void* tot_buf, const void* prog_buf, double* sums,
                    int64_t* counts, int32_t* status) {
  CDR_TRY
  if (!h || !tot_buf || !prog_buf || !sums || !counts || !status)
    CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  const int k = c.f64s_k, kd = k * c.d;
  if (k < 1) CDR_FAIL(CDR_ERR_STATE, "cdr_f64s_begin first");
  c.f64_sums.ensure(sizeof(double) * 2 * kd);
  c.f64_counts.ensure(sizeof(long long) * k * 2 + sizeof(int));
  int* dst = reinterpret_cast<int*>(c.f64_counts.as<long long>() + 2 * k);
  f64s_compose_all(c, k, c.f64s_nranks, static_cast<const double*>(tot_buf), prog_buf,
                   c.f64_sums.as<double>(), c.f64_counts.as<long long>(), dst);
  if (c.prof_cur >= 0) prof_mark(c, 2);  // (the step's kernels end here)
  HIP_CHECK(hipMemcpyAsync(sums, c.f64_sums.p, sizeof(double) * kd, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipMemcpyAsync(counts, c.f64_counts.p, sizeof(long long) * k, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipMemcpyAsync(status, dst, sizeof(int), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  const bool force = getenv("CDR_F64S_FORCE_CHAIN") && atoi(getenv("CDR_F64S_FORCE_CHAIN"));
  if (force) *status |= 1;  // (tests: the exact rank chain on every rank)
  CDR_CATCH
}

int cdr_f64s_chain(cdr_ctx* h, void* chain_buf) {
  CDR_TRY
  if (!h || !chain_buf) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  if (c.f64s_k < 1) CDR_FAIL(CDR_ERR_STATE, "cdr_f64s_begin first");
  f64s_chain_walk(c, c.f64s_k, static_cast<double*>(chain_buf));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  CDR_CATCH
}

int cdr_lloyd_step_f32r(cdr_ctx* h, const float* C, int32_t k, double* sums, int64_t* counts) {
  CDR_TRY
  if (!h || !C || !sums || !counts) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  lloyd_step_f32r(h->c, C, k, sums, counts);
  CDR_CATCH
}

int cdr_lloyd_labels(cdr_ctx* h, int64_t* labels) {
  CDR_TRY
  if (!h || (!labels && h->c.n > 0)) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  if (!c.have_labels) CDR_FAIL(CDR_ERR_STATE, "no Lloyd step has run");
  if (c.n == 0) return CDR_OK;
  HIP_CHECK(hipSetDevice(c.device));
  DevBuf tmp;
  tmp.ensure(sizeof(long long) * c.n);
  hipLaunchKernelGGL(labels_to_i64, dim3((int)std::min<int64_t>(ceil_div(c.n, 256), 4096)),
                     dim3(256), 0, c.stream, c.labels.as<int32_t>(), c.n, tmp.as<long long>());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(labels, tmp.p, sizeof(long long) * c.n, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  CDR_CATCH
}

int cdr_lloyd_f64_walked(cdr_ctx* h, int64_t* walked) {
  CDR_TRY
  if (!h || !walked) CDR_FAIL(CDR_ERR_ARG, "null argument");
  *walked = h->c.f64x_walked;
  CDR_CATCH
}

int cdr_lloyd_stats(cdr_ctx* h, int64_t* n_fallback) {
  CDR_TRY
  if (!h || !n_fallback) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  if (c.last_fallback < 0) {
    HIP_CHECK(hipSetDevice(c.device));
    int32_t fb = 0;
    if (c.last_screened)
      HIP_CHECK(hipMemcpyAsync(&fb, c.fb_count.as<int32_t>() + c.fb_total_slot, sizeof(int32_t),
                               hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    c.last_fallback = c.last_screened ? fb : c.n;
  }
  *n_fallback = c.last_fallback;
  CDR_CATCH
}

#ifdef CDR_EXPERIMENTS
// Timing experiments only (not in the product build or include/cdr.h): skip
// parts of the screen kernel; results are garbage while mask != 0.
int cdr_debug_screen_ablate(cdr_ctx* h, int32_t mask) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  h->c.screen_ablate = mask;
  CDR_CATCH
}
#endif

int cdr_profile_reset(cdr_ctx* h, int32_t enable) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.prof_used = 0;
  c.prof_cur = -1;
  c.prof_on = enable != 0;
  c.prof_period = enable > 1 ? enable : 1;
  c.prof_seen = 0;
  c.prof_screen_ms = c.prof_step_ms = c.prof_fb_points = 0.0;
  c.prof_launches = 0;
  c.prof_sub_ms = 0.0;
  c.prof_sub_launches = 0;
  c.fb_accum.ensure(2 * sizeof(long long));
  HIP_CHECK(hipMemsetAsync(c.fb_accum.p, 0, 2 * sizeof(long long), c.stream));
  if (c.q_acc.p) HIP_CHECK(hipMemsetAsync(c.q_acc.p, 0, c.q_acc.bytes, c.stream));
  if (c.t_acc.p) HIP_CHECK(hipMemsetAsync(c.t_acc.p, 0, c.t_acc.bytes, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  CDR_CATCH
}

int cdr_profile_read(cdr_ctx* h, double* out) {
  CDR_TRY
  if (!h || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  prof_collect(c);
  long long fb[2] = {0, 0};
  std::vector<long long> q(c.q_acc.bytes / sizeof(long long));
  std::vector<long long> tq(c.t_acc.bytes / sizeof(long long));
  if (c.fb_accum.p)
    HIP_CHECK(hipMemcpyAsync(fb, c.fb_accum.p, std::min(c.fb_accum.bytes, sizeof(fb)),
                             hipMemcpyDeviceToHost, c.stream));
  if (!q.empty())
    HIP_CHECK(hipMemcpyAsync(q.data(), c.q_acc.p, c.q_acc.bytes, hipMemcpyDeviceToHost, c.stream));
  if (!tq.empty())
    HIP_CHECK(hipMemcpyAsync(tq.data(), c.t_acc.p, c.t_acc.bytes, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  for (long long v : q) fb[1] += v;
  long long tight = 0;
  for (long long v : tq) tight += v;
  out[0] = c.prof_screen_ms;
  out[1] = (double)c.prof_launches;
  out[2] = c.prof_step_ms;
  out[3] = c.prof_fb_points + (double)fb[0];
  out[4] = (double)fb[1];
  out[5] = (double)tight;
  CDR_CATCH
}

int cdr_profile_read_sub(cdr_ctx* h, double* out) {
  CDR_TRY
  if (!h || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  prof_collect(c);
  out[0] = c.prof_sub_ms;
  out[1] = (double)c.prof_sub_launches;
  CDR_CATCH
}

int cdr_profile_kernel(cdr_ctx* h, char* buf, int32_t len) {
  CDR_TRY
  if (!h || !buf || len < 1) CDR_FAIL(CDR_ERR_ARG, "null argument");
  snprintf(buf, (size_t)len, "%s", h->c.prof_kernel);
  CDR_CATCH
}

// Test hook: screen values of every point (n_pad x ceil(k/16)*16 floats, host
// buffer) from one F32X step with centroids C.  Not part of the product path.
int cdr_debug_screen(cdr_ctx* h, const double* C, int32_t k, float* out_vals,
                     float* thr_a0a1) {
  CDR_TRY
  if (!h || !C || !out_vals) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  if (!screen_supported(c, k)) CDR_FAIL(CDR_ERR_UNSUPPORTED, "screen not used for this shape");
  const int KT = (k + 15) / 16;
  DevBuf dbg;
  dbg.ensure(sizeof(float) * (size_t)c.n_pad * KT * 16);
  HIP_CHECK(hipMemsetAsync(dbg.p, 0, sizeof(float) * (size_t)c.n_pad * KT * 16, c.stream));
  std::vector<long long> tmp((size_t)k * (c.d + 1));
  g_dbg_ptr = dbg.as<float>();
  try {
    lloyd_step_f32x(c, C, k, reinterpret_cast<int64_t*>(tmp.data()), false);
  } catch (...) {
    g_dbg_ptr = nullptr;
    throw;
  }
  g_dbg_ptr = nullptr;
  HIP_CHECK(hipMemcpy(out_vals, dbg.p, sizeof(float) * (size_t)c.n_pad * KT * 16,
                      hipMemcpyDeviceToHost));
  if (thr_a0a1) {
    if (screen32_supported(c, k)) {
      thr_a0a1[0] = g_dbg_thr[0];
      thr_a0a1[1] = g_dbg_thr[1];
    } else {
      ScreenPlan pl;
      build_screen_plan(c, C, k, pl);
      thr_a0a1[0] = pl.thrA0;
      thr_a0a1[1] = pl.thrA1;
    }
  }
  CDR_CATCH
}

}  // extern "C"
