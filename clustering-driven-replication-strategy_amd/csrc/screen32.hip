// screen32.hip — Lloyd assign + fused update for small d and k (d <= 16,
// k <= 64: BASELINE configs 2 and 3), reference src/kmeans_plusplus.py:33-41.
//
// One wave handles a group of 64 points as two 32-point tiles.  Distances come
// from v_mfma_f32_32x32x16_f16 in the ||x||^2 - 2 x.c + ||c||^2 form with the
// point norm replaced by a launch constant D (argmin is unchanged by a per-point
// shift; D keeps every screen value >= 0 so raw fp32 bits order as unsigned):
//
//   S_j = fl32( C_j + sum_f -2 chi_jf (hi_f + lo_f) - 2 clo_jf hi_f ),
//   C_j = fl32(||chat_j||^2 + D)  (the MFMA C operand, a per-lane constant)
//
// with xhat = (x - mu) 2^sigma split into fp16 hi + lo and chat likewise
// (chi + clo).  Per 32 centroids and 32 points that is three MFMAs for d = 16:
//   A1 x H  (H = [hi(q0), hi(q1)],  A1 = [-2chi(q0), -2chi(q1)])
//   A1 x L  (L = [lo(q0), lo(q1)])
//   A3 x H  (A3 = [-2clo(q0), -2clo(q1)])
// where lane half h owns the feature quads q0 = QH*h, q1 = QH*h + 1; for d <= 8
// (QH = 1) H = [hi(q0), lo(q0)], A1 = [-2chi, -2chi], A3 = [-2clo, 0] and the
// two MFMAs are A1 x H, A3 x H.  Every B operand is one 4-register tuple.
//
// Argmin: every lane keeps (best, runner-up) unsigned keys of its 32 values
// (value bits with the low 6 replaced by the row index), the two lane halves
// of a point are merged with one permlane32 swap per pair of tiles, after which
// lane l owns point base + l: one coalesced label store, one certification
// test, one fallback ballot.  A point is certified when
//     key_s > key_b * (1 + 2^-17) + T0
// (T0 = twice the rigorous screen error + the reference's rounding slack,
// derived in build_plan32 / DESIGN.md §4); uncertified points go to a per-wave
// fallback region and are re-done in exact fp64 NumPy order (fallback32).
//
// Update: certified points add their fp32 features (exact in fp64: grid data,
// see screen32_supported) into a per-workgroup LDS table sum[f][j] with
// ds_add_f64 and their count with ds_add_u32; reduce32 converts every
// workgroup's sums to exact int64 fixed point and adds them.
#include <cstdio>
#include <cmath>
#include <cstring>
#include <algorithm>
#include <vector>

#include "cdr_internal.h"
#include "exact_math.h"
#include "plan32.h"

namespace cdr {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

struct S32Args {
  const float* X;
  const float* X0;     // original points (x32): the exact fallback reads them
  const double* cent;  // k x d fp64 centroids (the exact fallback)
  int64_t n, n_pad;
  int d, k, Q;         // Q = number of stored feature quads (d4 / 4)
  const h8* frag;      // [MT][2][64]: A1, A3
  const float* cinit;  // [MT][16][64]
  const float* mu_s;   // [d] -mu_f 2^sigma
  float sig;
  float thr0, thr_rel;
  int32_t* labels;
  unsigned long long* run_sums;  // kRunSlices x (k, d+1) int64 running sums
  const long long* muf;          // PRE: int64 mu_f 2^S (null otherwise)
  double fx;                     // 2^(S - sigma) (PRE) or 2^S: table value -> fixed point
  int KP;
  int32_t* fb_list;
  int32_t* fb_count;
  int fb_cap;
  float* dbg;  // tests only: screen values (n_pad x dbg_ld) when non-null
  int dbg_ld;   // ceil(k / 16) * 16 (the cdr_debug_screen layout)
  const long long* gate;  // device loop: run only while gate[0] != 0 (null: always)
  const float* thr_dev;   // device loop: thr0 written by plan32_kernel (null: thr0)
};

__device__ __forceinline__ unsigned pack_h2(float a, float b) {
  h2 h = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(unsigned, h);
}

// hi = fp16(x) pairs (round to nearest even), lo = fp16(x - hi) pairs:
// 2 v_cvt_pk_f16_f32 + 4 v_fma_mix.
// x - hi is exact in fp32; v_fma_mix reads hi as f16 (op_sel_hi) and rounds
// x - hi once to f16 into the low / high half of the destination.
__device__ __forceinline__ void split4(const f4& x, unsigned& h01, unsigned& h23,
                                       unsigned& l01, unsigned& l23) {
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h01) : "v"(x[0]), "v"(x[1]));
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h23) : "v"(x[2]), "v"(x[3]));
  unsigned a, b;
  asm volatile(
      "v_fma_mixlo_f16 %0, %2, -1.0, %4 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %1, %3, -1.0, %6 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %2, -1.0, %5 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %1, %3, -1.0, %7 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(a), "=&v"(b)
      : "v"(h01), "v"(h23), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]));
  l01 = a;
  l23 = b;
}

__device__ __forceinline__ void merge_top2(unsigned& b, unsigned& s, unsigned b2, unsigned s2) {
  const unsigned nb = min(b, b2);
  s = min(max(b, b2), min(s, s2));
  b = nb;
}

__device__ __forceinline__ void swap32(unsigned& x, unsigned& y) {
  auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}

}  // namespace

// Exact assignment of the points the screen could not certify, run by the
// wave that found them after its last group (its region of the fallback
// list; the LDS table is still live, so no global read-modify-write and no
// extra launch).  4 lanes per point, 16 points per pass: lane c walks the
// centroids c, c + 4, c + 8, ... (fp64 rows staged in LDS with stride 17
// doubles) computing the NumPy-order fp64 squared distance and its correctly
// rounded sqrt and keeping the first minimum of its roots; the 4 candidates
// merge on (root, index) — np.argmin of np.linalg.norm, first index on ties
// (src/kmeans_plusplus.py:33-34).  The point's change goes into the table.
// Loads run ahead of the arithmetic: list entries two passes, the points'
// feature quads one pass.
template <int D>
__device__ __forceinline__ void fallback_points(const S32Args& a, const int32_t* region, int cnt,
                                                double* tsum, int* tcnt, const double* cs,
                                                int KP, bool delta, bool pre) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 2, c4 = lane & 3;
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int Q = (D + 3) / 4;
  const f4* X4 = reinterpret_cast<const f4*>(a.X0);
  __threadfence_block();  // the region was just written by this wave's lanes
  auto load_pt = [&](int e) -> int32_t { return e < cnt ? region[e] : 0; };
  auto load_x = [&](int32_t pt, f4 (&v)[Q]) {
#pragma unroll
    for (int q = 0; q < Q; ++q) v[q] = X4[(int64_t)q * a.n_pad + pt];
  };
  int32_t pt0 = load_pt(g), pt1 = load_pt(16 + g);
  f4 x0[Q];
  load_x(pt0, x0);
  for (int e0 = 0; e0 < cnt; e0 += 16) {
    const int e = e0 + g;
    const bool live = e < cnt;
    const int32_t pt = pt0;
    double x[D];
#pragma unroll
    for (int f = 0; f < D; ++f) x[f] = (double)x0[f >> 2][f & 3];
    if (e0 + 16 < cnt) {  // wave-uniform
      pt0 = pt1;
      load_x(pt0, x0);
      pt1 = load_pt(e0 + 32 + g);
    }
    double sb = INFINITY, rb = INFINITY;
    int jmin = 0x7fffffff;
    for (int j = c4; j < a.k; j += 4) {
      const double* cj = cs + j * 17;
      const double s = np_sqdist([&](int f) { return x[f]; }, [&](int f) { return cj[f]; }, D);
      // sqrt is monotone: a root can only undercut the best root when s < sb,
      // and then the roots decide (strict: first index on ties of the roots)
      if (s < sb) {
        const double r2 = sqrt(s);
        sb = s;
        if (r2 < rb) {
          rb = r2;
          jmin = j;
        }
      }
    }
#pragma unroll
    for (int o = 2; o > 0; o >>= 1) {
      const double ro = __shfl_xor(rb, o, 4);
      const int jo = __shfl_xor(jmin, o, 4);
      if (ro < rb || (ro == rb && jo < jmin)) {
        rb = ro;
        jmin = jo;
      }
    }
    if (live && c4 == 0) {
      if (jmin >= a.k) jmin = 0;  // every root NaN: np.argmin of all-NaN is 0
      const int old = delta ? a.labels[pt] : -1;  // the screen left it untouched
      if (jmin != old) {
        a.labels[pt] = jmin;
        if (pre) {  // the tables hold xt = (x - mu) 2^sigma (exact)
#pragma unroll
          for (int f = 0; f < D; ++f) x[f] = (double)fmaf((float)x[f], a.sig, a.mu_s[f]);
        }
#pragma unroll
        for (int f = 0; f < D; ++f) atomicAdd(&tsum[f * KP + jmin], x[f]);
        atomicAdd(&tcnt[jmin], 1);
        if (old >= 0) {
#pragma unroll
          for (int f = 0; f < D; ++f) atomicAdd(&tsum[f * KP + old], -x[f]);
          atomicAdd(&tcnt[old], -1);
        }
      }
    }
  }
}

__device__ __forceinline__ void fallback_tail(const S32Args& a, const int32_t* region, int cnt,
                                           double* tsum, int* tcnt, const double* cs, int KP,
                                           bool delta, bool pre) {
  switch (a.d) {
#define CDR_FBT(D_) \
  case D_: fallback_points<D_>(a, region, cnt, tsum, tcnt, cs, KP, delta, pre); break;
    CDR_FBT(1) CDR_FBT(2) CDR_FBT(3) CDR_FBT(4) CDR_FBT(5) CDR_FBT(6) CDR_FBT(7) CDR_FBT(8)
    CDR_FBT(9) CDR_FBT(10) CDR_FBT(11) CDR_FBT(12) CDR_FBT(13) CDR_FBT(14) CDR_FBT(15)
    CDR_FBT(16)
#undef CDR_FBT
    default: break;
  }
}

// QH: feature quads per lane half (1: d <= 8, 2: d <= 16); MT: 32-centroid
// tiles (1: k <= 32, 2: k <= 64).
// FULLQ: all 2*QH quads of the lane halves exist in memory (d4 == 8 QH).
// LDS table: sums [8 QH][KP] (rows of missing quads stay 0) + counts [KP].
// DELTA: `labels` holds the previous step's labels and the per-workgroup
// tables receive only the changes (+x into the new cluster, -x out of the old
// one) of points whose label changed; otherwise every certified point is added.
// ABL (timing experiments only, results are garbage): 1 no update, 2 no
// argmin (values folded into one key), 8 no HBM loads (synthetic points).
// PRE: a.X is the pre-centred copy xt = (x - mu) 2^sigma (exact, Ctx::pre_ok):
// the screen uses it as loaded and the tables sum xt (reduce32 restores x).
template <int QH, int MT, bool FULLQ, bool DELTA, bool DBG, bool PRE, int ABL = 0>
__global__ __launch_bounds__(256) void screen32(S32Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int KP = 32 * MT;
  constexpr int NF = 8 * QH;
  if (a.gate && a.gate[0] == 0) return;  // device loop stopped: uniform exit
  double* tsum = reinterpret_cast<double*>(smem);                      // [NF][KP]
  int* tcnt = reinterpret_cast<int*>(tsum + (size_t)NF * KP);          // [KP]
  double* cs = reinterpret_cast<double*>(tcnt + KP);                   // [k][17]
  for (int i = threadIdx.x; i < NF * KP; i += blockDim.x) tsum[i] = 0.0;
  for (int i = threadIdx.x; i < KP; i += blockDim.x) tcnt[i] = 0;
  for (int i = threadIdx.x; i < a.k * a.d; i += blockDim.x)
    cs[(i / a.d) * 17 + i % a.d] = a.cent[i];

  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int p = lane & 31;
  h8 A[MT][2];  // [0] = A1 (-2chi), [1] = A3 (-2clo)
  f16v Ci[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
#pragma unroll
    for (int u = 0; u < 2; ++u) A[m][u] = a.frag[(m * 2 + u) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 16; ++i) Ci[m][i] = a.cinit[(m * 16 + i) * 64 + lane];
  }
  // this lane's quads and centering constants
  int qd[QH];
  bool qok[QH];
  f4 ms[QH];
#pragma unroll
  for (int u = 0; u < QH; ++u) {
    qd[u] = QH * h + u;
    qok[u] = FULLQ || qd[u] < a.Q;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = 4 * qd[u] + i;
      ms[u][i] = f < a.d ? a.mu_s[f] : 0.0f;
    }
  }
  const float sig = a.sig, thr0 = a.thr_dev ? a.thr_dev[0] : a.thr0, thr_rel = a.thr_rel;
  const f4* Xq = reinterpret_cast<const f4*>(a.X);
  const int wpb = blockDim.x >> 6;
  const int64_t ngroups = a.n_pad >> 6;
  const int64_t gstride = (int64_t)gridDim.x * wpb;
  int64_t G = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6);
  const int wave_id = (int)G;
  int32_t* fb_region = a.fb_list + (size_t)wave_id * a.fb_cap;
  int fb_used = 0;
  __syncthreads();

  // running per-lane pointers of the next group to load (quad u; labels),
  // advanced by one grid stride per prefetch
  const int64_t gstep = (int64_t)gridDim.x * wpb * 64;
  const f4* pq[QH];
#pragma unroll
  for (int u = 0; u < QH; ++u) pq[u] = Xq + (int64_t)qd[u] * a.n_pad + (G << 6) + p;
  const int32_t* plab = a.labels + (G << 6) + lane;
  auto load = [&](f4 (&buf)[2][QH], int64_t grp) {
    if constexpr ((ABL & 8) != 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < QH; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            buf[t][u][i] = (float)((((int)grp * 7 + 13 * t + 5 * u + 3 * i + p) * 2654435761u) >> 8) *
                           0x1p-24f;
      return;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < QH; ++u) {
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (FULLQ || qok[u]) v = pq[u][32 * t];  // tile t: immediate offset 512 B
        buf[t][u] = v;
      }
  };

  // screen values of one 32-point tile -> (best, runner-up) keys of this lane
  auto tile = [&](const f4 (&xq)[QH], unsigned& bk, unsigned& sk, int64_t tbase) {
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
    u4v H, L;
#pragma unroll
    for (int u = 0; u < QH; ++u) {
      f4 xt;
      if constexpr (PRE) {
        xt = xq[u];
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) xt[i] = fmaf(xq[u][i], sig, ms[u][i]);
      }
      unsigned h01, h23, l01, l23;
      split4(xt, h01, h23, l01, l23);
      if (QH == 1) {
        H = u4v{h01, h23, l01, l23};
      } else {
        H[2 * u] = h01;
        H[2 * u + 1] = h23;
        L[2 * u] = l01;
        L[2 * u + 1] = l23;
      }
    }
    const h8 BH = __builtin_bit_cast(h8, H);
    f16v acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][0], BH, Ci[m], 0, 0, 0);
      if constexpr (QH == 2) {
        const h8 BL = __builtin_bit_cast(h8, L);
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][0], BL, acc[m], 0, 0, 0);
      }
      acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][1], BH, acc[m], 0, 0, 0);
    }
    if constexpr (DBG) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int i = 0; i < 16; ++i)
        {
          const int row = 32 * m + 8 * (i >> 2) + 4 * h + (i & 3);
          if (row < a.dbg_ld) a.dbg[(tbase + p) * a.dbg_ld + row] = acc[m][i];
        }
    }
    if constexpr ((ABL & 2) != 0) {
      unsigned z = 0;
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int i = 0; i < 16; ++i) z ^= __float_as_uint(acc[m][i]);
      bk = (z & ~63u) | (unsigned)p;
      sk = 0xFFFFFFFFu;
      return;
    }
    // keys: reg i of tile m is row 32m + 8(i/4) + 4h + (i%4); 4h is OR-ed later
    auto key = [&](int m, int i) {
      return (__float_as_uint(acc[m][i]) & ~63u) | (unsigned)(32 * m + 8 * (i >> 2) + (i & 3));
    };
    unsigned b, s;
    {
      const unsigned k0 = key(0, 0), k1 = key(0, 1);
      b = min(k0, k1);
      s = max(k0, k1);
    }
#pragma unroll
    for (int q = 2; q < 16 * MT; q += 2) {
      const unsigned x = key(q >> 4, q & 15), y = key(q >> 4, (q & 15) + 1);
      unsigned t;  // second smallest of {b, x, y}; then b = min of the three
      asm("v_med3_u32 %0, %1, %2, %3" : "=v"(t) : "v"(b), "v"(x), "v"(y));
      asm("v_min3_u32 %0, %1, %2, %3" : "=v"(b) : "v"(b), "v"(x), "v"(y));
      s = min(s, t);
    }
    bk = b | ((unsigned)h << 2);
    sk = s | ((unsigned)h << 2);
  };

  // one group of 64 points (the wave's registers xb, previous labels ob)
  auto process = [&](const f4 (&xb)[2][QH], int ob, int64_t Gp) {
    const int64_t base = Gp << 6;
    if (base >= a.n) return;  // wave-uniform: padding groups have no real points
    unsigned bA, sA, bB, sB;
    tile(xb[0], bA, sA, base);
    tile(xb[1], bB, sB, base + 32);
    // lanes < 32: tile A's point l; lanes >= 32: tile B's point l - 32
    swap32(bA, bB);
    swap32(sA, sB);
    merge_top2(bA, sA, bB, sB);
    const int64_t pt = base + lane;
    const int label = (int)(bA & 63u);
    const float vb = __uint_as_float(bA & ~63u);
    const float vs = __uint_as_float(sA & ~63u);
    const bool cert = vs > fmaf(vb, thr_rel, thr0);  // NaN: never certified
    const bool real = pt < a.n;
    const bool ok = cert && real;
    bool put = ok;
    if (DELTA) put = ok && label != ob;
    if (put) a.labels[pt] = label;
    const unsigned long long need = __ballot(real && !cert);
    if (need) {
      const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(need >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((unsigned)need, 0u));
      if (real && !cert) fb_region[fb_used + rank] = (int32_t)pt;
      fb_used += __popcll(need);
    }
    if constexpr ((ABL & 1) != 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < QH; ++u) asm volatile("" ::"v"(xb[t][u]));
      return;
    }
    // verdicts of tile A / tile B point p to both lane halves
    unsigned vA = put ? (unsigned)label : 0xFFFFFFFFu;
    unsigned vB = vA;
    swap32(vA, vB);
    unsigned oA = 0xFFFFFFFFu, oB = 0xFFFFFFFFu;
    if (DELTA) {
      oA = put ? (unsigned)ob : 0xFFFFFFFFu;
      oB = oA;
      swap32(oA, oB);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int lp = (int)(t == 0 ? vA : vB);
      if (lp >= 0) {
        double* row = tsum + 4 * QH * h * KP + lp;  // feature 4 qd[0] of label lp
#pragma unroll
        for (int u = 0; u < QH; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i) atomicAdd(&row[(4 * u + i) * KP], (double)xb[t][u][i]);
        if (DELTA) {
          const int lo = (int)(t == 0 ? oA : oB);
          double* orow = tsum + 4 * QH * h * KP + lo;
#pragma unroll
          for (int u = 0; u < QH; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i) atomicAdd(&orow[(4 * u + i) * KP], -(double)xb[t][u][i]);
        }
      }
    }
    const int lc = (int)(h == 0 ? vA : vB);
    if (lc >= 0) {
      atomicAdd(&tcnt[lc], 1);
      if (DELTA) atomicAdd(&tcnt[(int)(h == 0 ? oA : oB)], -1);
    }
  };
  auto prefetch = [&](f4 (&buf)[2][QH], int& ob, int64_t Gp) {
    if (Gp < ngroups) {
      load(buf, Gp);
      if (DELTA) ob = *plab;
    }
#pragma unroll
    for (int u = 0; u < QH; ++u) pq[u] += gstep;
    plab += gstep;
  };

#ifndef CDR_S32_DEPTH
#define CDR_S32_DEPTH 1
#endif
#if CDR_S32_DEPTH == 3
  // three register sets: loads run two groups ahead
  f4 x0[2][QH], x1[2][QH], x2[2][QH];
  int o0 = -1, o1 = -1, o2 = -1;  // DELTA: previous label of point base + lane
  prefetch(x0, o0, G);
  prefetch(x1, o1, G + gstride);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): see below
  for (; G < ngroups; G += 3 * gstride) {
    prefetch(x2, o2, G + 2 * gstride);
    process(x0, o0, G);
    if (G + gstride >= ngroups) break;
    prefetch(x0, o0, G + 3 * gstride);
    process(x1, o1, G + gstride);
    if (G + 2 * gstride >= ngroups) break;
    prefetch(x1, o1, G + 4 * gstride);
    process(x2, o2, G + 2 * gstride);
  }
#elif CDR_S32_DEPTH == 2
  // two register sets used alternately (no copies between iterations)
  f4 xa[2][QH], xb2[2][QH];
  int oa = -1, ob2 = -1;  // DELTA: previous label of point base + lane
  prefetch(xa, oa, G);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): see below
  for (; G < ngroups; G += 2 * gstride) {
    prefetch(xb2, ob2, G + gstride);
    process(xa, oa, G);
    if (G + gstride >= ngroups) break;
    prefetch(xa, oa, G + 2 * gstride);
    process(xb2, ob2, G + gstride);
  }
#else
  f4 cur[2][QH], nxt[2][QH];
  int ocur = -1, onxt = -1;  // DELTA: previous label of point base + lane
  prefetch(cur, ocur, G);
  // drain before the loop, otherwise the waitcnt pass merges these loads into
  // the loop-header state and waits for the fresh prefetch in every iteration
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  for (; G < ngroups; G += gstride) {
    prefetch(nxt, onxt, G + gstride);
    process(cur, ocur, G);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < QH; ++u) cur[t][u] = nxt[t][u];
    ocur = onxt;
  }
#endif
  if (lane == 0) {
    a.fb_count[wave_id] = fb_used;
    if (fb_used) atomicAdd(a.fb_count + gstride, fb_used);
  }
  if constexpr ((ABL & 1) == 0) {
    if (fb_used) fallback_tail(a, fb_region, fb_used, tsum, tcnt, cs, KP, DELTA, PRE);
  }
  __syncthreads();
  // This workgroup's table as exact int64 fixed point, added into slice
  // (blockIdx % kRunSlices) of the running sums: sum x 2^S = sum xt 2^(S -
  // sigma) + count mu 2^S (PRE), both exact integers.  Lanes walk the (k,
  // d+1) output contiguously; zero contributions (clusters no point of this
  // workgroup entered or left) are skipped.
  {
    const int d1 = a.d + 1, cells = a.k * d1;
    unsigned long long* out = a.run_sums + (size_t)(blockIdx.x % kRunSlices) * cells;
    for (int e = threadIdx.x; e < cells; e += blockDim.x) {
      const int j = e / d1, r = e - j * d1;
      const int cnt = tcnt[j];
      long long v;
      if (r < a.d) {
        v = __double2ll_rn(tsum[r * KP + j] * a.fx);
        if (PRE) v += (long long)cnt * a.muf[r];
      } else {
        v = cnt;
      }
      if (v) atomicAdd(&out[e], (unsigned long long)v);
    }
  }
}

// One block after the screen (the kernel boundary orders it after every
// workgroup's atomics): the sum of the kRunSlices slices of the running sums
// -> dout (device, e.g. for the all-reduce) and/or hout (mapped pinned host
// memory, with the fallback total at hout[cells]); the screen's fallback
// counter fbc[nwaves] moves to fbc[nwaves + 1] and is cleared for the next
// step.
__global__ __launch_bounds__(256) void publish32(const long long* __restrict__ out, int cells,
                                                 long long* __restrict__ dout,
                                                 long long* __restrict__ hout,
                                                 int* __restrict__ fbc, int nwaves,
                                                 long long* __restrict__ fb_acc,
                                                 const long long* __restrict__ gate) {
  // (one cell per thread over as many workgroups as needed: a single
  // workgroup looping over the cells paid one memory round trip per pass)
  if (gate && gate[0] == 0) {  // a stopped loop contributes nothing to the all-reduce
    if (dout)
      for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < cells; i += gridDim.x * blockDim.x)
        dout[i] = 0;
    return;
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < cells; i += gridDim.x * blockDim.x) {
    long long v = 0;
#pragma unroll
    for (int sl = 0; sl < kRunSlices; ++sl) v += out[(size_t)sl * cells + i];
    if (dout) dout[i] = v;
    if (hout) hout[i] = v;
  }
  if (fbc && blockIdx.x == 0) {  // (uniform)
    const int fb = block_sum_counts(fbc, nwaves);
    if (threadIdx.x == 0) {
      fbc[nwaves] = 0;
      fbc[nwaves + 1] = fb;
      if (hout) hout[cells] = fb;
      if (fb_acc) fb_acc[0] += fb;
    }
  }
}

// Zeroes n int64 (the running sums before a full, non-DELTA step) unless
// the device loop has stopped.
__global__ void zero_gated(long long* __restrict__ p, int n, const long long* __restrict__ gate) {
  if (gate && gate[0] == 0) return;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = 0;
}

// xt = (x - mu) 2^sigma = fma(x, 2^sigma, -mu 2^sigma), exact (Ctx::pre_ok).
// Padding rows and feature slots >= d stay 0.
__global__ void precenter_kernel(const float* __restrict__ x, int64_t n, int64_t n_pad, int d,
                                 const float* __restrict__ ms, float sig, float* __restrict__ xt) {
  const int d4 = d4_of(d);
  const int64_t total = (int64_t)d4 * n_pad;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = t / (4 * n_pad);  // SoA [d4/4][n_pad][4]
    const int64_t r = t - q * 4 * n_pad;
    const int64_t i = r >> 2;
    const int f = (int)(4 * q + (r & 3));
    xt[t] = (f < d && i < n) ? fmaf(x[t], sig, ms[f]) : 0.0f;
  }
}

// ---------------------------------------------------------------------------
// DELTA steps without the in-loop update: screen32d + fixup32.
//
// screen32's per-group instruction stream is ~260 VALU, and the SIMDs issue
// back to back (PMC: three waves per SIMD are active / issue-stalled 67 % of
// their cycles).  After the first step almost every point keeps its label, so
// the DELTA steps run a leaner pair:
// * screen32d reads a split screen copy (xs16: the fp16 hi / lo halves the
//   MFMA B operands consist of, split once per point set with the same
//   instructions screen32 uses: identical screen values and certification)
//   with wave-uniform base addresses, and writes only labels and two lists per
//   wave: certified points whose label changed ({pt, old | new << 16}) and
//   uncertified points;
// * fixup32 applies the changes of both lists to the running sums: it
//   gathers the moved points from x32 (1-2 % of the points), re-does the
//   uncertified ones in exact fp64 NumPy order, and adds its LDS table into
//   the int64 slices.  Integer sums, so the result equals a full recompute.
// ---------------------------------------------------------------------------

// xs16 tile of 32 points: [h = 0, 1][p = 0..31][hi(QH quads) | lo(QH quads)]
// as fp16, where lane half h owns quads QH h .. QH h + QH - 1 (screen32's
// layout; QH = 1: [hi(q), lo(q)] is the B operand itself).  Missing features
// and padding rows are 0.  HO (QH = 2 only): the hi halves alone, 16 bytes per
// (point, half) — the hi-only screen copy of screen32d<2, MT, PD, true>; with
// QH = 1 the hi quad alone, 8 bytes per (point, half).
template <int QH, bool HO = false>
__global__ void split_copy_kernel(const float* __restrict__ x, int64_t n, int64_t n_pad, int d,
                                  const float* __restrict__ ms, float sig,
                                  uint4* __restrict__ xs) {
  const int64_t total = n_pad * 2;  // (point, half) pairs
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t tile = t >> 6;
    const int h = (int)((t >> 5) & 1), p = (int)(t & 31);
    const int64_t i = tile * 32 + p;
    unsigned hw[2 * QH], lw[2 * QH];
#pragma unroll
    for (int u = 0; u < QH; ++u) {
      f4 xt;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 4 * (QH * h + u) + c;
        xt[c] = (f < d && i < n) ? fmaf(x[xidx(x, f, i, n_pad)], sig, ms[f]) : 0.0f;
      }
      split4(xt, hw[2 * u], hw[2 * u + 1], lw[2 * u], lw[2 * u + 1]);
    }
    uint4* dst = xs + (size_t)t * (HO ? 1 : QH);  // 16 QH bytes per (point, half)
    if (HO && QH == 1) {  // 8 bytes per (point, half)
      reinterpret_cast<uint2*>(xs)[t] = uint2{hw[0], hw[1]};
    } else if (HO) {
      dst[0] = uint4{hw[0], hw[1], hw[2], hw[3]};
    } else if (QH == 1) {
      dst[0] = uint4{hw[0], hw[1], lw[0], lw[1]};
    } else {
      dst[0] = uint4{hw[0], hw[1], hw[2], hw[3]};
      dst[1] = uint4{lw[0], lw[1], lw[2], lw[3]};
    }
  }
}

// labels -> their one-byte copy (k <= 64), once per run of DELTA steps
__global__ void lab8_kernel(const int32_t* __restrict__ labels, uint8_t* __restrict__ lab8,
                            int64_t n_pad) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n_pad; i += stride) {
    const int4 v = *reinterpret_cast<const int4*>(labels + i);  // n_pad: a multiple of 64
    const unsigned w = (unsigned)(v.x & 255) | (unsigned)(v.y & 255) << 8 |
                       (unsigned)(v.z & 255) << 16 | (unsigned)(v.w & 255) << 24;
    *reinterpret_cast<unsigned*>(lab8 + i) = w;
  }
}

struct S32DArgs {
  const unsigned char* XS;  // split copy (tiles of 32 points, 1024 QH bytes each)
  int64_t n, n_pad;
  const h8* frag;
  const float* cinit;
  float thr0, thr_rel;
  float Dv;                 // the plan's offset D (hi-only screen; device plan: thr_dev[1])
  const float* thr_dev;
  const long long* gate;
  int32_t* labels;
  uint8_t* lab8;      // one-byte copy of labels (Ctx::lab8): read for the old label
  int2* fb_list;      // per-wave regions of uncertified points {pt, old label}
  int32_t* fb_count;  // per-wave counts, then the step total at [nwaves]
  int2* mv_list;      // per-wave regions of moved points
  int32_t* mv_count;
  int cap;
};

// PD: groups of 64 points per wave in flight (the loads of PD - 1 groups are
// issued ahead of the one being screened).
//
// HO (hi-only, QH = 2): the screen copy holds h = fp16(xhat) alone (32 bytes
// per point at d = 16 instead of 64) and each tile takes two MFMAs, A1 x H and
// A3 x H: the screen values are those of the point h, S_j = Shat_j +- E with
// Shat_j = D + ||chat_j||^2 - 2 chat_j.h (E: the plan's bound, thr0 >= 2E + the
// reference slack).  The true decision values T_j = ||chat_j||^2 - 2 chat_j.xhat
// differ by 2 (chat_j - chat_b).delta, delta = h - xhat, |delta| <= dn =
// 2^-11 (1 + 2^-9) ||h|| + 2^-23 (fp16 round to nearest, subnormals), and
// |chat_j - chat_b| <= sqrt(G_j) + sqrt(G_b) with G_j = ||h - chat_j||^2 <=
// S_j + E - D + ||h||^2.  A point is certified when
//     v_s > v_b (1 + 2^-16) + thr0 + 2 dn (sqrt(G_s) + sqrt(G_b))
// (v: the truncated keys, S_b <= v_b (1 + 2^-17), S_j >= v_s for every j != b).
// Then sqrt(G_s) > 2 dn, so S - 2 dn sqrt(S + E - D + ||h||^2) grows with S
// above v_s and the bound holds for every j != b: T_j - T_b > slack.
//
// LR (with HO): the screen copy streams through a per-wave LDS ring of PD
// slots with global_load_lds_dwordx4 (no VGPRs hold loads in flight, so PD - 1
// groups ahead cost no occupancy); the wave waits for its own slot with an
// explicit vmcnt (loads complete in issue order) and reads it back with
// ds_read_b128 at the same lane offset.
template <int QH, int MT, int PD, bool HO = false, bool LR = false>
__global__ __launch_bounds__(256) void screen32d(S32DArgs a) {
  static_assert(!LR || (HO && QH == 2 && PD <= 4), "LDS ring: hi-only d > 8, at most 4 slots");
  // H1: hi-only with d <= 8.  Lane half h holds hi(q_h) (8 bytes); the B
  // operand is [hi, hi] against A = [-2 chi, -2 clo]: one MFMA per tile
  constexpr bool H1 = HO && QH == 1;
  if (a.gate && a.gate[0] == 0) return;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int p = lane & 31;
  h8 A[MT][2];
  f16v Ci[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
#pragma unroll
    for (int u = 0; u < 2; ++u) A[m][u] = a.frag[(m * 2 + u) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 16; ++i) Ci[m][i] = a.cinit[(m * 16 + i) * 64 + lane];
    if constexpr (H1)  // plan (QH = 1): A1 = [-2chi, -2chi], A3 = [-2clo, 0]
#pragma unroll
      for (int i = 0; i < 4; ++i) A[m][0][4 + i] = A[m][1][i];
  }
  const float thr0 = a.thr_dev ? a.thr_dev[0] : a.thr0, thr_rel = a.thr_rel;
  const float Dlo = (a.thr_dev ? a.thr_dev[1] : a.Dv) * (1.0f - 0x1p-19f);  // < D
  const int wpb = blockDim.x >> 6;
  const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  const int nwaves = gridDim.x * wpb;
  const int64_t ngroups = a.n_pad >> 6;
  int2* fb_region = a.fb_list + (size_t)wave * a.cap;
  int2* mv_region = a.mv_list + (size_t)wave * a.cap;
  int fb_used = 0, mv_used = 0;
  // per group: two tiles of 1024 QH bytes; lane (h, p) reads 16 QH bytes at
  // (h * 32 + p) * 16 QH of each tile
  constexpr int NL = HO ? 1 : QH;  // 16-byte loads per tile and lane (H1: one 8-byte load)
  constexpr int kTile = H1 ? 512 : 1024 * NL;
  const unsigned loff = (unsigned)((h * 32 + p) * (H1 ? 8 : 16 * NL));
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  struct Buf {
    u4v v[2][NL];  // [tile][0] = H (QH = 2: hi of both quads; QH = 1: hi | lo), [tile][1] = L
    int ob;
  };
  auto load = [&](Buf& b, int64_t G) {
    if (G < ngroups) {
      const unsigned char* base = a.XS + (size_t)G * (2 * kTile);  // wave-uniform
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < NL; ++u) {
          if constexpr (H1) {
            const uint2 w = *reinterpret_cast<const uint2*>(base + loff + t * kTile);
            b.v[t][u] = u4v{w.x, w.y, w.x, w.y};
          } else {
            b.v[t][u] = *reinterpret_cast<const u4v*>(base + loff + t * kTile + 16 * u);
          }
        }
      b.ob = a.lab8[G * 64 + lane];
    }
  };
  // (best, runner-up) keys of one 32-point tile, as screen32's tile()
  auto tile = [&](const u4v (&v)[NL], unsigned& bk, unsigned& sk, float& hp) {
    const h8 BH = __builtin_bit_cast(h8, v[0]);
    f16v acc[MT];
    if constexpr (HO) {  // this lane's part of ||h||^2 (fp16 products are exact in fp32)
      hp = 0.0f;
#pragma unroll
      for (int i = 0; i < (H1 ? 4 : 8); i += 2)
        hp = __builtin_amdgcn_fdot2(h2{BH[i], BH[i + 1]}, h2{BH[i], BH[i + 1]}, hp, false);
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][0], BH, Ci[m], 0, 0, 0);
      if constexpr (QH == 2 && !HO) {
        const h8 BL = __builtin_bit_cast(h8, v[1]);
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][0], BL, acc[m], 0, 0, 0);
      }
      if constexpr (!H1) acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][1], BH, acc[m], 0, 0, 0);
    }
    auto key = [&](int m, int i) {
      return (__float_as_uint(acc[m][i]) & ~63u) | (unsigned)(32 * m + 8 * (i >> 2) + (i & 3));
    };
    unsigned b, s;
    {
      const unsigned k0 = key(0, 0), k1 = key(0, 1);
      b = min(k0, k1);
      s = max(k0, k1);
    }
#pragma unroll
    for (int q = 2; q < 16 * MT; q += 2) {
      const unsigned x = key(q >> 4, q & 15), y = key(q >> 4, (q & 15) + 1);
      unsigned t;
      asm("v_med3_u32 %0, %1, %2, %3" : "=v"(t) : "v"(b), "v"(x), "v"(y));
      asm("v_min3_u32 %0, %1, %2, %3" : "=v"(b) : "v"(b), "v"(x), "v"(y));
      s = min(s, t);
    }
    bk = b | ((unsigned)h << 2);
    sk = s | ((unsigned)h << 2);
  };
  auto process = [&](const Buf& b, int64_t G) {
    const int64_t base = G << 6;
    if (base >= a.n) return;  // wave-uniform: padding groups have no real points
    unsigned bA, sA, bB, sB;
    float hA, hB;
    tile(b.v[0], bA, sA, hA);
    tile(b.v[1], bB, sB, hB);
    swap32(bA, bB);
    swap32(sA, sB);
    merge_top2(bA, sA, bB, sB);
    const int64_t pt = base + lane;
    const int label = (int)(bA & 63u);
    const float vb = __uint_as_float(bA & ~63u);
    const float vs = __uint_as_float(sA & ~63u);
    float thr = fmaf(vb, thr_rel, thr0);
    if constexpr (HO) {  // the hi-only certificate (above the kernel)
      unsigned ua = __float_as_uint(hA), ub = __float_as_uint(hB);
      swap32(ua, ub);
      // ||h||^2 from below by at most 9 roundings (and flushed fp16 subnormals)
      const float hh = fmaf(__uint_as_float(ua) + __uint_as_float(ub), 1.0f + 0x1p-18f, 0x1p-20f);
      // v_sqrt_f32 (1 ulp; its arguments kept normal)
      const float dn = fmaf(0x1p-11f * (1.0f + 0x1p-9f), __builtin_amdgcn_sqrtf(hh), 0x1p-23f);
      const float K = thr0 + hh - Dlo;  // G = S + E - D + ||h||^2 from above (16 ulp(D) spare)
      const float Gs = fmaxf(vs + K, 0x1p-100f), Gb = fmaxf(fmaf(vb, thr_rel, K), 0x1p-100f);
      thr += 2.0f * (1.0f + 0x1p-19f) * dn *
             (__builtin_amdgcn_sqrtf(Gs) + __builtin_amdgcn_sqrtf(Gb));
    }
    const bool cert = vs > thr;  // NaN: never certified
    const bool real = pt < a.n;
    const bool moved = cert && real && label != b.ob;
    if (moved) {
      a.labels[pt] = label;
      a.lab8[pt] = (uint8_t)label;
    }
    const unsigned long long mv = __ballot(moved);
    if (mv) {
      const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(mv >> 32),
                                              __builtin_amdgcn_mbcnt_lo((unsigned)mv, 0u));
      if (moved) mv_region[mv_used + r] = int2{(int)pt, b.ob | (label << 16)};
      mv_used += __popcll(mv);
    }
    const unsigned long long need = __ballot(real && !cert);
    if (need) {
      const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(need >> 32),
                                              __builtin_amdgcn_mbcnt_lo((unsigned)need, 0u));
      if (real && !cert) fb_region[fb_used + r] = int2{(int)pt, b.ob};
      fb_used += __popcll(need);
    }
  };
  const int64_t gs = nwaves;
  if constexpr (LR) {
    constexpr int kSlot = 2048 + 64;  // two hi tiles of 1024 bytes, 64 one-byte labels
    __shared__ __attribute__((aligned(16))) unsigned char ring[4 * PD * kSlot];
    // this wave's slots (a scalar base: M0 without per-load readfirstlane)
    unsigned char* wring = ring + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * PD * kSlot;
    // 3 vector-memory operations per group, all LDS DMA (nothing lands in
    // VGPRs, so the compiler adds no vmcnt wait of its own): two tile loads
    // and the labels (16 lanes x 4 bytes)
    auto issue = [&](int slot, int64_t G) {
      if (G < ngroups) {
        const unsigned char* gx = a.XS + (size_t)G * 2048;  // scalar base + lane offset
        const unsigned char* gl = a.lab8 + G * 64;
        unsigned char* dst = wring + slot * kSlot;  // wave-uniform (M0)
        __builtin_amdgcn_global_load_lds(gx + (unsigned)(lane * 16), dst, 16, 0, 0);
        __builtin_amdgcn_global_load_lds(gx + (unsigned)(1024 + lane * 16), dst + 1024, 16, 0, 0);
        if (lane < 16) __builtin_amdgcn_global_load_lds(gl + (unsigned)(lane * 4), dst + 2048, 4, 0, 0);
      }
    };
#pragma unroll
    for (int i = 0; i < PD - 1; ++i) issue(i, wave + i * gs);
    for (int64_t G = wave; G < ngroups; G += PD * gs) {
#pragma unroll
      for (int i = 0; i < PD; ++i) {
        const int64_t Gi = G + i * gs;
        if (Gi >= ngroups) break;
        issue((i + PD - 1) % PD, Gi + (PD - 1) * gs);
        // groups issued after Gi (wave-uniform): wait until 3 x that many remain
        int later = 0;
#pragma unroll
        for (int j = 1; j < PD; ++j) later += Gi + j * gs < ngroups ? 1 : 0;
        if (later >= 3) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        else if (later == 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else if (later == 1) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        Buf b;
        const unsigned char* src = wring + i * kSlot + lane * 16;
        b.v[0][0] = *reinterpret_cast<const u4v*>(src);
        b.v[1][0] = *reinterpret_cast<const u4v*>(src + 1024);
        b.ob = wring[i * kSlot + 2048 + lane];
        process(b, Gi);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {  // (the step's total: fixup32)
      a.fb_count[wave] = fb_used;
      a.mv_count[wave] = mv_used;
    }
    return;
  }
  Buf buf[PD];
#pragma unroll
  for (int i = 0; i < PD - 1; ++i) load(buf[i], wave + i * gs);
  for (int64_t G = wave; G < ngroups; G += PD * gs) {
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      const int64_t Gi = G + i * gs;
      if (Gi >= ngroups) break;
      load(buf[(i + PD - 1) % PD], Gi + (PD - 1) * gs);
      process(buf[i], Gi);
    }
  }
  if (lane == 0) {  // (the step's total: fixup32)
    a.fb_count[wave] = fb_used;
    a.mv_count[wave] = mv_used;
  }
}

constexpr int kFixMaxR = 16;  // screen waves per fixup32 workgroup at most

struct FixArgs {
  const float* XA;     // the points row-major, d4 floats per point (one line each)
  int64_t n_pad;
  const double* cent;  // k x d fp64 centroids of the step
  int k, d;
  int32_t* labels;
  uint8_t* lab8;  // kept equal to labels (screen32d reads it)
  const int2* fb_list;  // {pt, old label}
  const int32_t* fb_count;
  const int2* mv_list;
  const int32_t* mv_count;
  int cap;
  int regions;  // screen32d waves
  int fr;       // screen waves (list regions) per workgroup, <= kFixMaxR
  double fx;    // 2^S
  unsigned long long* run_sums;  // kRunSlices x (k, d+1)
  const long long* gate;
  int abl;  // timing experiments only (0 in the product build): 1 no moves, 2 no fallback,
           // 4 no flush, 8 first candidate only, 16 no point gather, 32 no label / table change
  // the step's screen (the uncertified points are screened again)
  const unsigned char* XS;
  const h8* frag;
  const float* cinit;
  float thr0, thr_rel;
  const float* thr_dev;
  // hi-only screen copy (screen32h): the re-screen splits the points itself
  // from XA, as split_copy_kernel<2> does (the same hi / lo bits)
  int ho;
  const float* ms;  // -mu_f 2^sigma
  float sig;
  // screen32b's per-point bound words (null otherwise): a label change here
  // leaves the point's word "no bound" with its new label
  uint32_t* zb;
};

// screen32b's bound word of a point whose bound is unknown (a quiet NaN: the
// bound test fails) — the low 6 bits carry the label
constexpr unsigned kZbStale = 0x7FC00000u;

// Workgroup b applies the lists of screen32d waves FR b .. FR b + FR - 1 (a region
// spread over the whole workgroup) to an LDS table (rows padded to 65: the
// lanes of one point hit different banks).
// * Moves, 4 lanes per point (lane q: feature quad q): +x into the new
//   cluster, -x out of the old one.
// * Uncertified points, 64 per wave: the screen of screen32d is recomputed
//   for them (the same plan, so the same values), and every centroid whose
//   key is within the certification threshold of the best key is a candidate
//   (|S_j - T_j| <= E for all j: the reference's argmin is among them; a point
//   is certified exactly when the best is the only one).  The lane owning the
//   point evaluates its candidates in index order in exact fp64 NumPy order
//   with a correctly rounded sqrt: np.argmin of np.linalg.norm, first index on
//   ties (src/kmeans_plusplus.py:33-34).
template <int Q>
struct FixDims {
  static constexpr int QH = Q <= 2 ? 1 : 2;  // quads per lane half of the split screen
  static constexpr int DM = 4 * Q;           // features a point row holds (d <= DM)
};
constexpr int kFixTS = 65;  // table row stride
// LDS of one fixup workgroup: tsum [16][kFixTS] | cs [64][17] (fp64) | tcnt [64] |
// s_mv, s_fb [kFixMaxR + 1]
constexpr size_t kFixLdsBytes =
    sizeof(double) * (16 * kFixTS + 64 * 17) + sizeof(int) * (64 + 2 * (kFixMaxR + 1));
struct FixLds {
  double* tsum;
  double* cs;
  int* tcnt;
  int* s_mv;
  int* s_fb;
  __device__ explicit FixLds(unsigned char* base) {
    tsum = reinterpret_cast<double*>(base);
    cs = tsum + 16 * kFixTS;
    tcnt = reinterpret_cast<int*>(cs + 64 * 17);
    s_mv = tcnt + 64;
    s_fb = s_mv + kFixMaxR + 1;
  }
};

// The lists of screen waves r0 .. r0 + FR - 1 applied by one workgroup to an
// LDS table (rows padded to 65: the lanes of one point hit different banks),
// then to slice `slice` of the running sums.  The caller has put the regions'
// counts in s_mv[1 .. FR] / s_fb[1 .. FR]; every thread calls it.  Q: feature
// quads of a point row (d <= 4 Q; d itself is a runtime value).
// * Moves, 4 lanes per point (lane q: feature quad q): +x into the new
//   cluster, -x out of the old one.
// * Uncertified points, 64 per wave: the split screen of screen32d is
//   computed for them (the same plan, so the same values), and every centroid
//   whose key is within the certification threshold of the best key is a
//   candidate (|S_j - T_j| <= E for all j: the reference's argmin is among
//   them; a point is certified exactly when the best is the only one).  The
//   lane owning the point evaluates its candidates in index order in exact fp64
//   NumPy order with a correctly rounded sqrt: np.argmin of np.linalg.norm,
//   first index on ties (src/kmeans_plusplus.py:33-34).
// np_sqdist (exact_math.h: NumPy's pairwise order of sum((x - c)^2)) for a
// runtime d <= 16 with every index a constant, so that x stays in registers:
// d < 8 sequential from 0.0; else 8 accumulators over the first 8 (d & ~7)
// features, the fixed tree, then the tail in order.
__device__ __forceinline__ double np_sqdist16(const float (&x)[16], const double* c, int d) {
  auto sq = [&](int f) {
    const double u = (double)x[f] - c[f];
    return u * u;
  };
  if (d < 8) {
    double res = 0.0;
#pragma unroll
    for (int f = 0; f < 8; ++f)
      if (f < d) res = res + sq(f);
    return res;
  }
  double r[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = sq(i);
  if (d >= 16) {
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = r[i] + sq(8 + i);
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  const int dd = d - (d & 7);
#pragma unroll
  for (int f = 8; f < 16; ++f)
    if (f >= dd && f < d) res = res + sq(f);
  return res;
}

// Plan operands of the re-screen: from global memory (fixup32) or from the
// screen's LDS copies (screen32p: sA [MT][2][64] h8, sC [MT][4][2][4] f32).
struct FixPlan {
  const h8* sA;
  const float* sC;
};
template <int Q, int MT>
__device__ __forceinline__ void fixup_regions(const FixArgs& a, int r0, int FR, int slice,
                                              const FixLds& L, FixPlan P = FixPlan{nullptr, nullptr}) {
  constexpr int CS = 17;
  constexpr int TS = kFixTS;
  constexpr int QH = FixDims<Q>::QH;
  constexpr int DM = FixDims<Q>::DM;
  double* tsum = L.tsum;
  double* cs = L.cs;
  int* tcnt = L.tcnt;
  int* s_mv = L.s_mv;
  int* s_fb = L.s_fb;
  const int k = a.k, d = a.d;
  // the step's centroids (fp64), loaded by every thread at once
#pragma unroll 4
  for (int i = threadIdx.x; i < k * d; i += blockDim.x) {
    const double v = a.cent[i];
    cs[(i / d) * CS + i % d] = v;
  }
  for (int i = threadIdx.x; i < DM * TS; i += blockDim.x) tsum[i] = 0.0;
  for (int i = threadIdx.x; i < 64; i += blockDim.x) tcnt[i] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    s_mv[0] = s_fb[0] = 0;
    for (int r = 1; r <= FR; ++r) {
      s_mv[r] += s_mv[r - 1];
      s_fb[r] += s_fb[r - 1];
    }
  }
  __syncthreads();
  const int nmv = s_mv[FR], nfb = s_fb[FR];
  if (nmv == 0 && nfb == 0) return;  // uniform: nothing changes here
  const f4* XA4 = reinterpret_cast<const f4*>(a.XA);  // point i: XA4[i * Q + q]
  auto region_of = [&](const int* pre, int e, int& r, int& i) {
    r = 0;
    while (r < FR - 1 && e >= pre[r + 1]) ++r;
    i = e - pre[r];
  };
  const int g = threadIdx.x >> 2, q4 = threadIdx.x & 3;
  // moved points: 64 per pass, lane q4 adds feature quad q4
  for (int e0 = 0; e0 < ((a.abl & 1) ? 0 : nmv); e0 += 64) {
    const int e = e0 + g;
    if (e < nmv && q4 < Q) {
      int r, i;
      region_of(s_mv, e, r, i);
      const int2 rec = a.mv_list[(size_t)(r0 + r) * a.cap + i];
      const f4 xq = XA4[(int64_t)rec.x * Q + q4];
      const int to = rec.y >> 16, from = rec.y & 0xFFFF;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 4 * q4 + c;
        if (f < d) {
          atomicAdd(&tsum[f * TS + to], (double)xq[c]);
          atomicAdd(&tsum[f * TS + from], -(double)xq[c]);
        }
      }
      if (q4 == 0) {
        atomicAdd(&tcnt[to], 1);
        atomicAdd(&tcnt[from], -1);
      }
    }
  }
  if (nfb && !(a.abl & 2)) {
    constexpr int kTile = 1024 * QH;
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int h = lane >> 5, p = lane & 31;
    // centroid tile m's screen values of B (one tile's accumulator live at a
    // time: this body also runs in screen32p's tail, beside its registers)
    auto screen_m = [&](int m, const u4v (&vt)[QH]) -> f16v {
      const h8 A0 = P.sA ? P.sA[(m * 2 + 0) * 64 + lane] : a.frag[(m * 2 + 0) * 64 + lane];
      const h8 A1 = P.sA ? P.sA[(m * 2 + 1) * 64 + lane] : a.frag[(m * 2 + 1) * 64 + lane];
      f16v acc;
      if (P.sC) {
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) {
          const f4 c4v = *reinterpret_cast<const f4*>(P.sC + ((m * 4 + i4) * 2 + h) * 4);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[4 * i4 + i] = c4v[i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = a.cinit[(m * 16 + i) * 64 + lane];
      }
      const h8 BH = __builtin_bit_cast(h8, vt[0]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, BH, acc, 0, 0, 0);
      if constexpr (QH == 2) {
        const h8 BL = __builtin_bit_cast(h8, vt[QH - 1]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, BL, acc, 0, 0, 0);
      }
      return __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, BH, acc, 0, 0, 0);
    };
    const float thr0 = a.thr_dev ? a.thr_dev[0] : a.thr0, thr_rel = a.thr_rel;
    auto rec_of = [&](int e) -> int2 {
      int r, i;
      region_of(s_fb, e, r, i);
      return a.fb_list[(size_t)(r0 + r) * a.cap + i];
    };
    for (int e0 = wv * 64; e0 < nfb; e0 += blockDim.x) {
      // tile t holds list entries e0 + 32 t .. + 31; lane (h, p) the B
      // operand of entry e0 + 32 t + p (its half h), as screen32d loads it
      int32_t ptt[2], oldt[2];
      u4v v[2][QH];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int e = e0 + 32 * t + p;
        const int2 rec = e < nfb ? rec_of(e) : int2{-1, 0};
        ptt[t] = rec.x;
        oldt[t] = rec.y;
        const int32_t q = ptt[t] < 0 ? 0 : ptt[t];
        if (a.ho) {  // QH quads of half h, split as split_copy_kernel<QH> does
          unsigned hw[4], lw[4];
#pragma unroll
          for (int u = 0; u < QH; ++u) {
            const int qq = QH * h + u;
            const f4 xr = qq < Q ? XA4[(int64_t)q * Q + qq] : f4{0.f, 0.f, 0.f, 0.f};
            f4 xt;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const int f = 4 * qq + c;
              xt[c] = f < d ? fmaf(xr[c], a.sig, a.ms[f]) : 0.0f;
            }
            split4(xt, hw[2 * u], hw[2 * u + 1], lw[2 * u], lw[2 * u + 1]);
          }
          if constexpr (QH == 1) {
            v[t][0] = u4v{hw[0], hw[1], lw[0], lw[1]};
          } else {
            v[t][0] = u4v{hw[0], hw[1], hw[2], hw[3]};
            v[t][QH - 1] = u4v{lw[0], lw[1], lw[2], lw[3]};
          }
        } else {
          const unsigned char* src =
              a.XS + (size_t)(q >> 5) * kTile + (h * 32 + (q & 31)) * 16 * QH;
#pragma unroll
          for (int u = 0; u < QH; ++u) v[t][u] = *reinterpret_cast<const u4v*>(src + 16 * u);
        }
      }
      // this lane's point after the half swap: entry e0 + lane (tile lane >> 5)
      const int own = h ? ptt[1] : ptt[0];  // lane (h, p) owns entry e0 + 32 h + p
      const int old = h ? oldt[1] : oldt[0];   // (selects: no indexed private arrays)
      const int e_own = e0 + lane;
      const bool live = e_own < nfb;
      f4 xq[Q];
      if (live) {
#pragma unroll
        for (int q = 0; q < Q; ++q)
          xq[q] = (a.abl & 16) ? f4{0.f, 0.f, 0.f, 0.f} : XA4[(int64_t)own * Q + q];
      }
      // screen values and candidate masks per tile: bit 16 m + i of a lane's
      // mask = value i of centroid tile m in its half (row 32 m + 8 (i / 4) +
      // 4 h + i % 4); immediates only, so nothing is hoisted into registers
      unsigned mine[2], other[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        // best key of the point over both halves (as screen32d forms keys)
        unsigned bk = 0xFFFFFFFFu;
#pragma nounroll
        for (int m = 0; m < MT; ++m) {
          const f16v acc = screen_m(m, v[t]);
          const unsigned rb = 32u * (unsigned)m;
#pragma unroll
          for (int i = 0; i < 16; ++i)
            bk = min(bk, (__float_as_uint(acc[i]) & ~63u) | (rb + (unsigned)(8 * (i >> 2) + (i & 3))));
        }
        bk |= (unsigned)h << 2;
        bk = min(bk, (unsigned)__shfl_xor((int)bk, 32));
        const float tau = fmaf(__uint_as_float(bk & ~63u), thr_rel, thr0);
        unsigned cm = 0;
#pragma nounroll
        for (int m = 0; m < MT; ++m) {  // the same values again (recomputed, bit-identical)
          const f16v acc = screen_m(m, v[t]);
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            // not excluded: key value <= tau (NaN: a candidate)
            const float kv = __uint_as_float(__float_as_uint(acc[i]) & ~63u);
            if (!(kv > tau)) cm |= 1u << (16 * m + i);
          }
        }
        mine[t] = cm;
        other[t] = (unsigned)__shfl_xor((int)cm, 32);
      }
      // lane (h, p) owns tile h's point p: its rows of half h are in mine[h],
      // those of half 1 - h in other[h]; as a 64-bit row mask
      unsigned long long cand = 0;
      {
        const unsigned mh0 = h == 0 ? mine[0] : other[1], mh1 = h == 0 ? other[0] : mine[1];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          unsigned mm = hh ? mh1 : mh0;  // rows of half hh of tile h
          while (mm) {
            const int bb = __builtin_ctz(mm);
            mm &= mm - 1;
            const int m = bb >> 4, i = bb & 15;
            cand |= 1ull << (32 * m + 8 * (i >> 2) + 4 * hh + (i & 3));
          }
        }
        if (k < 64) cand &= (1ull << k) - 1;
      }
      if (live) {
        float x[16];  // (fp32 data: converted exactly where used)
#pragma unroll
        for (int f = 0; f < 16; ++f) x[f] = f < DM ? xq[f >> 2][f & 3] : 0.0f;
        double sb = INFINITY, rb = INFINITY;
        int jmin = 0x7fffffff;
        unsigned long long cmk = (a.abl & 8) ? (cand & (~cand + 1)) : cand;
        while (cmk) {  // increasing j
          const int j = __builtin_ctzll(cmk);
          cmk &= cmk - 1;
          const double sq = np_sqdist16(x, cs + j * CS, d);
          if (sq < sb) {  // sqrt is monotone: only a smaller square can give a smaller root
            const double rt = sqrt(sq);
            sb = sq;
            if (rt < rb) {
              rb = rt;
              jmin = j;
            }
          }
        }
        if (jmin >= k) jmin = 0;  // every root NaN: np.argmin of all-NaN is 0
        if (jmin != old && !(a.abl & 32)) {
          a.labels[own] = jmin;
          a.lab8[own] = (uint8_t)jmin;
          if (a.zb) a.zb[own] = kZbStale | (unsigned)jmin;  // (screen32b: bound unknown)
#pragma unroll
          for (int f = 0; f < DM; ++f) {
            if (f < d) {
              atomicAdd(&tsum[f * TS + jmin], (double)x[f]);
              atomicAdd(&tsum[f * TS + old], -(double)x[f]);
            }
          }
          atomicAdd(&tcnt[jmin], 1);
          atomicAdd(&tcnt[old], -1);
        }
      }
    }
  }
  __syncthreads();
  if (a.abl & 4) return;
  const int d1 = d + 1, cells = k * d1;
  unsigned long long* out = a.run_sums + (size_t)slice * cells;
  for (int e = threadIdx.x; e < cells; e += blockDim.x) {
    const int j = e / d1, r = e - j * d1;
    const long long v = r < d ? __double2ll_rn(tsum[r * TS + j] * a.fx) : (long long)tcnt[j];
    if (v) atomicAdd(&out[e], (unsigned long long)v);
  }
}

// One workgroup per FR screen waves (a.fr), after the screen (screen32d).
template <int Q, int MT>
__global__ __launch_bounds__(256, 3) void fixup32(FixArgs a) {
  if (a.gate && a.gate[0] == 0) return;
  __shared__ __attribute__((aligned(16))) unsigned char lds[kFixLdsBytes];
  const FixLds L(lds);
  const int FR = a.fr;
  const int r0 = blockIdx.x * FR;
  if (threadIdx.x < FR) {
    const int r = r0 + threadIdx.x;
    L.s_mv[threadIdx.x + 1] = r < a.regions ? a.mv_count[r] : 0;
    L.s_fb[threadIdx.x + 1] = r < a.regions ? a.fb_count[r] : 0;
  }
  fixup_regions<Q, MT>(a, r0, FR, blockIdx.x % kRunSlices, L);
}
// Pruned DELTA screen: screen32p (d <= 16, k <= 64; configs 2 and 3).
//
// screen32h spends ~213 VALU per 64 points on the k-way screen (64 MFMA values
// and a keyed top-2 per point) and is VALU-issue bound.  After the first step
// almost every point stays with its label a deep inside its cluster, where one
// distance decides it.  screen32p gives each lane ONE point and first tries
// the triangle inequality in distance space (t_j = ||xhat - chat_j|| =
// 2^sigma ||x - C_j||, the reference's distance up to a power of two):
//   t_j >= ||chat_a - chat_j|| - t_a >= h_a - t_a   for every j != a,
// h_a = min_j ||chat_a - chat_j||, so a is the argmin when 2 t_a < h_a (with
// margins).  t_a comes from the hi-only screen copy h = fp16(xhat) in fp32
// (16 v_fma_mix differences and packed fp32 squares against c32_a) and is
// bounded rigorously:
//   | ||h - c32_a|| - sqrt(q_a) | <= 2^-19 sqrt(q_a)   (q_a: 2 roundings + 9
//       along any summation path, every term >= 0; v_sqrt_f32 1 ulp),
//   ||h - xhat|| <= dn  (the fp16 rounding of the point, screen32_prune_dn),
//   ||c32_a - chat_a|| <= ec_a  (the fp32 rounding of the centroid),
// so ub_a = sqrt(q_a)(1 + 2^-18) + E_a with E_a >= (dn + ec_a)(1 + 2^-20)
// bounds t_a from above, and the point keeps a when
//   h_a (1 - 2^-22) - ub_a > ub_a (1 + 2^-20):
// every other exact distance then exceeds t_a by more than 2^-21 relative,
// far above the reference's own fp64 rounding (< 2^-45), so np.argmin of the
// reference's norms is a (src/kmeans_plusplus.py:33-34).
//
// The points this test cannot decide (near a second centroid, or of a
// centroid far from its points) are appended — their 32 (d <= 8: 16) bytes
// and {pt, a} — to a per-wave LDS queue laid out as the MFMA B operands.
// Whenever 64 are queued the wave runs screen32h's k-way screen and hi-only
// certificate on them (the same plan, keys and bounds), so the MFMA work
// shrinks to the queued fraction; its moved points go to the move region,
// its uncertified ones to the fallback region, exactly as in screen32d, and
// fixup32 finishes the step.  Every point is still read and decided every
// step.
//
// c32, E and h come with the step's plan (the prune block, plan32.h: built by
// plan32_build on the device right after the centroids move, or by the host's
// build_plan32), so a workgroup only stages 5.6 KB of it into LDS.
// ---------------------------------------------------------------------------
struct S32PArgs {
  const unsigned char* XS;  // hi-only screen copy (screen32h / screen32h1 layout)
  int64_t n, n_pad;
  int k, d;
  const float* prune;  // the plan's prune block (plan32.h: c32 | E | h)
  // the k-way screen of the queued points: screen32h's plan
  const h8* frag;
  const float* cinit;
  float thr0, thr_rel, Dv;
  const float* thr_dev;
  const long long* gate;
  int32_t* labels;
  uint8_t* lab8;
  int2* fb_list;  // per-wave regions {pt, old label}
  int32_t* fb_count;
  int2* mv_list;  // per-wave regions {pt, old | new << 16}
  int32_t* mv_count;
  int cap;
  long long* q_acc;  // profiling: points queued for the k-way screen, per wave (null: off)
  FixArgs fx;        // the fused fixup (fixup32's arguments, fr = 4)
  int fuse;
  int abl;  // timing experiments only (0 in the product build): 1 no drains,
            // 2 no per-point work (loads and the label byte only)
};

// fp32 (lo / hi fp16 half of w) - c, one rounding (v_fma_mix_f32)
__device__ __forceinline__ float mix_sub_lo(unsigned w, float c) {
  float r;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(w), "v"(c));
  return r;
}
__device__ __forceinline__ float mix_sub_hi(unsigned w, float c) {
  float r;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r)
      : "v"(w), "v"(c));
  return r;
}

// QH: 2 for d = 9..16 (16 bytes per point half), 1 for d <= 8 (8 bytes);
// MT: 32-centroid tiles of the k-way screen; PD: groups in flight per wave.
template <int Q, int MT, int PD>
__global__ __launch_bounds__(256, 5) void screen32p(S32PArgs a) {
  constexpr int QH = FixDims<Q>::QH;
  if (a.gate && a.gate[0] == 0) return;
  constexpr bool H1 = QH == 1;
  constexpr int kTile = H1 ? 512 : 1024;  // bytes per 32-point tile
  constexpr int kHalf = kTile / 2;
  constexpr int kPB = H1 ? 8 : 16;        // bytes per (point, half)
  constexpr int NWH = kPB / 4;            // dwords per point half
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) float c32s[64 * kPrStr + 128];
  float* const eb = c32s + 64 * kPrStr;  // E_j
  float* const hc = eb + 64;             // h_j
  // per wave: a ring of 2 blocks x 64 queued points (2 tiles each, B layout)
  // per wave: a ring of 2 blocks x 64 queued points (2 tiles each, B layout)
  // and their {pt, old label}; after the last drain the same LDS holds the
  // fused fixup's table (FixLds)
  constexpr size_t kQBytes = 4 * 2 * 2 * kTile + 4 * 128 * sizeof(int2);
  __shared__ __attribute__((aligned(16))) unsigned char qlds[kQBytes > kFixLdsBytes ? kQBytes : kFixLdsBytes];
  typedef unsigned char QRow[2][2 * kTile];
  QRow* qd = reinterpret_cast<QRow*>(qlds);
  int2 (*qm)[128] = reinterpret_cast<int2 (*)[128]>(qlds + 4 * 2 * 2 * kTile);
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const int h = lane >> 5;
  const int p = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wv);
  const int nwaves = gridDim.x * 4;
  const int64_t ngroups = a.n_pad >> 6;
  typedef unsigned u2v __attribute__((ext_vector_type(2)));
  struct Buf {
    u4v q0, q1;           // the loaded halves (QH = 2)
    u2v h0, h1;           // (QH = 1)
    unsigned w[2 * NWH];  // the lane's point: half 0 then half 1 (packed fp16 pairs)
    int ob;
  };
  // lane l: point 64 G + l = tile 2 G + (l >> 5), column l & 31
  unsigned loff = (unsigned)(h * kTile + p * kPB);
  unsigned lane4 = (unsigned)lane;
  // The group loads are issued from inline asm (SGPR base + lane offset) and
  // waited for with an explicit vmcnt: the compiler neither sees them nor
  // inserts waits of its own (its waits for conditional loads were vmcnt(0),
  // which drained the prefetch every few groups).  Vector-memory operations
  // complete in issue order, so before group i the wave waits until at most
  // 3 (PD - 1) of them are outstanding: the later groups' loads (and any
  // stores issued after them) may stay in flight.  A group past the end
  // reloads the last one (every iteration issues exactly 3 loads).
  auto load = [&](Buf& b, int64_t G) __attribute__((always_inline)) {
    const int64_t Gc = G < ngroups ? G : ngroups - 1;
    const unsigned char* base = a.XS + (size_t)Gc * (2 * kTile);  // wave-uniform
    const uint8_t* lbase = a.lab8 + Gc * 64;
    if constexpr (H1) {
      asm volatile("global_load_dwordx2 %0, %1, %2\n\t"
                   "global_load_dwordx2 %3, %1, %2 offset:256"
                   : "=&v"(b.h0), "+v"(loff), "+s"(base), "=&v"(b.h1));
    } else {
      asm volatile("global_load_dwordx4 %0, %1, %2\n\t"
                   "global_load_dwordx4 %3, %1, %2 offset:512"
                   : "=&v"(b.q0), "+v"(loff), "+s"(base), "=&v"(b.q1));
    }
    asm volatile("global_load_ubyte %0, %1, %2" : "=&v"(b.ob), "+v"(lane4), "+s"(lbase));
  };
  // wait for buffer b, `later` groups having been issued after it
  auto wait = [&](Buf& b, int later) __attribute__((always_inline)) {
    if constexpr (H1) {
      if (later >= 2) asm volatile("s_waitcnt vmcnt(6)" : "+v"(b.h0), "+v"(b.h1), "+v"(b.ob));
      else if (later == 1) asm volatile("s_waitcnt vmcnt(3)" : "+v"(b.h0), "+v"(b.h1), "+v"(b.ob));
      else asm volatile("s_waitcnt vmcnt(0)" : "+v"(b.h0), "+v"(b.h1), "+v"(b.ob));
      b.w[0] = b.h0.x; b.w[1] = b.h0.y; b.w[2] = b.h1.x; b.w[3] = b.h1.y;
    } else {
      if (later >= 2) asm volatile("s_waitcnt vmcnt(6)" : "+v"(b.q0), "+v"(b.q1), "+v"(b.ob));
      else if (later == 1) asm volatile("s_waitcnt vmcnt(3)" : "+v"(b.q0), "+v"(b.q1), "+v"(b.ob));
      else asm volatile("s_waitcnt vmcnt(0)" : "+v"(b.q0), "+v"(b.q1), "+v"(b.ob));
      b.w[0] = b.q0.x; b.w[1] = b.q0.y; b.w[2] = b.q0.z; b.w[3] = b.q0.w;
      b.w[4] = b.q1.x; b.w[5] = b.q1.y; b.w[6] = b.q1.z; b.w[7] = b.q1.w;
    }
  };
  const int64_t gs = nwaves;
  Buf buf[PD];
  // the first groups' loads overlap the prologue
#pragma unroll
  for (int i = 0; i < PD - 1; ++i) load(buf[i], wave + i * gs);

  // ---- k-way screen plan (screen32d<QH, MT, PD, HO = true>), staged in LDS
  // and read by a wave only when it drains its queue (no VGPRs held):
  // fragments [MT][2][64] h8, C operand as [MT][4][2 halves][4] per 16 values
  __shared__ h8 sA[MT * 2 * 64];
  __shared__ __attribute__((aligned(16))) float sC[MT * 4 * 2 * 4];
  // Every global load of the staging is issued before the first LDS store
  // (one round trip for the whole prologue, not one per loop iteration).
  // cinit[(m * 16 + ii) * 64 + ln] belongs to row 32 m + 8 (ii >> 2) + 4 (ln >> 5)
  // + (ii & 3): one value per (m, ii, ln >> 5), kept as sC[m][ii >> 2][ln >> 5][ii & 3].
  constexpr int kPr4 = (64 * kPrStr + 128) / 4;  // prune block in float4
  static_assert(kPr4 <= 512 && MT * 2 * 64 <= 256, "prologue: two float4 per thread");
  const f4* prune4 = reinterpret_cast<const f4*>(a.prune);
  const f4 pv0 = prune4[t];
  const f4 pv1 = t + 256 < kPr4 ? prune4[t + 256] : f4{0.f, 0.f, 0.f, 0.f};
  h8 av = {};
  if (t < MT * 2 * 64) av = a.frag[t];
  float cv = 0.0f;
  const int cm = t >> 5, ci4 = (t >> 3) & 3, chh = (t >> 2) & 1, cc = t & 3;
  if (t < MT * 32) cv = a.cinit[(cm * 16 + ci4 * 4 + cc) * 64 + chh * 32];
  const float thr0 = a.thr_dev ? a.thr_dev[0] : a.thr0, thr_rel = a.thr_rel;
  const float Dlo = (a.thr_dev ? a.thr_dev[1] : a.Dv) * (1.0f - 0x1p-19f);  // < D
  // the plan's fp32 centroids c32, their bounds E and nearest-centroid distances h
  // (contiguous in the plan and here: c32s | eb | hc)
  reinterpret_cast<f4*>(c32s)[t] = pv0;
  if (t + 256 < kPr4) reinterpret_cast<f4*>(c32s)[t + 256] = pv1;
  if (t < MT * 2 * 64) sA[t] = av;
  if (t < MT * 32) sC[t] = cv;
  __syncthreads();

  int2* fb_region = a.fb_list + (size_t)wave * a.cap;
  int2* mv_region = a.mv_list + (size_t)wave * a.cap;
  int fb_used = 0, mv_used = 0;
  // q = ||h - c32_j||^2: one fma_mix difference per feature, packed fp32 squares
  auto dist2 = [&](const Buf& b, int j) __attribute__((always_inline)) -> float {
    const f4* c4 = reinterpret_cast<const f4*>(c32s + j * kPrStr);  // 16-byte rows
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 acc = {0.0f, 0.0f};
    // dword i of the lane's point holds features 2i, 2i + 1 (half 0 then half 1)
#pragma unroll
    for (int q = 0; q < NWH; ++q) {
      const f4 cq = c4[q];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = 2 * q + u;
        const f2 df = {mix_sub_lo(b.w[i], cq[2 * u]), mix_sub_hi(b.w[i], cq[2 * u + 1])};
        acc = __builtin_elementwise_fma(df, df, acc);
      }
    }
    return acc.x + acc.y;
  };
  // (best, runner-up) keys of one 32-point tile of queued points, screen32d's tile()
  // The centroid tiles m are screened one after another (a loop that is not
  // unrolled, fragments and C operand read from LDS inside it), so only one
  // tile's accumulators are ever live: 4 waves per SIMD instead of 3.
  auto tile = [&](const u4v& v, unsigned& bk, unsigned& sk, float& hp) __attribute__((always_inline)) {
    const h8 BH = __builtin_bit_cast(h8, v);
    hp = 0.0f;  // this lane's part of ||h||^2 (fp16 products are exact in fp32)
#pragma unroll
    for (int i = 0; i < (H1 ? 4 : 8); i += 2)
      hp = __builtin_amdgcn_fdot2(h2{BH[i], BH[i + 1]}, h2{BH[i], BH[i + 1]}, hp, false);
    unsigned b = 0xFFFFFFFFu, s = 0xFFFFFFFFu;
#pragma nounroll
    for (int m = 0; m < MT; ++m) {
      h8 A0 = sA[(m * 2 + 0) * 64 + lane];
      const h8 A1 = sA[(m * 2 + 1) * 64 + lane];
      if constexpr (H1)  // plan (QH = 1): A1 = [-2chi, -2chi], A3 = [-2clo, 0]
#pragma unroll
        for (int i = 0; i < 4; ++i) A0[4 + i] = A1[i];
      f16v acc;
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const f4 c4v = *reinterpret_cast<const f4*>(sC + ((m * 4 + i4) * 2 + h) * 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[4 * i4 + i] = c4v[i];
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, BH, acc, 0, 0, 0);
      if constexpr (!H1) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, BH, acc, 0, 0, 0);
      const unsigned rb = 32u * (unsigned)m;
      auto key = [&](int i) {
        return (__float_as_uint(acc[i]) & ~63u) | (rb + (unsigned)(8 * (i >> 2) + (i & 3)));
      };
#pragma unroll
      for (int q = 0; q < 16; q += 2) {
        const unsigned x = key(q), y = key(q + 1);
        unsigned tq;
        asm("v_med3_u32 %0, %1, %2, %3" : "=v"(tq) : "v"(b), "v"(x), "v"(y));
        asm("v_min3_u32 %0, %1, %2, %3" : "=v"(b) : "v"(b), "v"(x), "v"(y));
        s = min(s, tq);
      }
    }
    bk = b | ((unsigned)h << 2);
    sk = s | ((unsigned)h << 2);
  };
  // the k-way screen of queue block qb (nvalid entries), then its lists
  auto drain = [&](int qb, int nvalid) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's queue writes
    const unsigned char* src = qd[wv][qb];
    u4v v[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      if constexpr (H1) {
        const uint2 x = *reinterpret_cast<const uint2*>(src + tt * kTile + lane * kPB);
        v[tt] = u4v{x.x, x.y, x.x, x.y};
      } else {
        v[tt] = *reinterpret_cast<const u4v*>(src + tt * kTile + lane * kPB);
      }
    }
    const int2 meta = qm[wv][qb * 64 + lane];  // lane l owns entry l after the swap
    unsigned bA = 0, sA = 0, bB = 0, sB = 0;
    float hA = 0.0f, hB = 0.0f;
    // one point tile at a time (a loop that is not unrolled)
#pragma nounroll
    for (int tt = 0; tt < 2; ++tt) {
      unsigned bk, sk;
      float hp;
      tile(tt == 0 ? v[0] : v[1], bk, sk, hp);
      if (tt == 0) {
        bA = bk;
        sA = sk;
        hA = hp;
      } else {
        bB = bk;
        sB = sk;
        hB = hp;
      }
    }
    swap32(bA, bB);
    swap32(sA, sB);
    merge_top2(bA, sA, bB, sB);
    const int label = (int)(bA & 63u);
    const float vb = __uint_as_float(bA & ~63u);
    const float vs = __uint_as_float(sA & ~63u);
    float thr = fmaf(vb, thr_rel, thr0);
    {  // the hi-only certificate (screen32d)
      unsigned ua = __float_as_uint(hA), ub = __float_as_uint(hB);
      swap32(ua, ub);
      const float hh = fmaf(__uint_as_float(ua) + __uint_as_float(ub), 1.0f + 0x1p-18f, 0x1p-20f);
      const float dn = fmaf(0x1p-11f * (1.0f + 0x1p-9f), __builtin_amdgcn_sqrtf(hh), 0x1p-23f);
      const float K = thr0 + hh - Dlo;
      const float Gs = fmaxf(vs + K, 0x1p-100f), Gb = fmaxf(fmaf(vb, thr_rel, K), 0x1p-100f);
      thr += 2.0f * (1.0f + 0x1p-19f) * dn * (__builtin_amdgcn_sqrtf(Gs) + __builtin_amdgcn_sqrtf(Gb));
    }
    const bool valid = lane < nvalid;
    const bool cert = vs > thr;  // NaN: never certified
    const int pt = meta.x, ob = meta.y;
    const bool moved = valid && cert && label != ob;
    if (moved) {
      a.labels[pt] = label;
      a.lab8[pt] = (uint8_t)label;
    }
    // both lists in straight-line code (two identical guarded blocks were
    // merged by the optimiser into one updating fb_used / mv_used through a
    // pointer, which put both counters in scratch memory)
    const bool unc = valid && !cert;
    const unsigned long long mv = __ballot(moved);
    const unsigned long long need = __ballot(unc);
    const int rm = __builtin_amdgcn_mbcnt_hi((unsigned)(mv >> 32),
                                             __builtin_amdgcn_mbcnt_lo((unsigned)mv, 0u));
    const int rn = __builtin_amdgcn_mbcnt_hi((unsigned)(need >> 32),
                                             __builtin_amdgcn_mbcnt_lo((unsigned)need, 0u));
    if (moved) mv_region[mv_used + rm] = int2{pt, ob | (label << 16)};
    if (unc) fb_region[fb_used + rn] = int2{pt, ob};
    mv_used += __popcll(mv);
    fb_used += __popcll(need);
  };
  int qh = 0, qn = 0;  // queue head (next slot, mod 128) and length: wave-uniform
  int qtot = 0;        // points this wave queued (profiling)
  auto process = [&](const Buf& b, int64_t G) __attribute__((always_inline)) {
    const int64_t base = G << 6;
    if (base >= a.n) return;  // wave-uniform: padding groups have no real points
    const int64_t pt = base + lane;
    const bool real = pt < a.n;
    const int ao = b.ob;
    if (a.abl & 2) {  // timing experiments: streaming only
      if (b.w[0] == 0x7fffffffu && b.w[2 * NWH - 1] == 0x7fffffffu) fb_used += ao;
      return;
    }
    const float qa = dist2(b, ao);
    const float uba = fmaf(__builtin_amdgcn_sqrtf(qa), 1.0f + 0x1p-18f, eb[ao]);
    const bool keep = fmaf(hc[ao], 1.0f - 0x1p-22f, -uba) > uba * (1.0f + 0x1p-20f);
    const bool q = real && !keep;
    const unsigned long long m = __ballot(q);
    if (m) {
      if (q) {
        const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        const int slot = (qh + r) & 127;
        const int e = slot & 63;
        unsigned char* dst = qd[wv][slot >> 6] + (e >> 5) * kTile + (e & 31) * kPB;
        if constexpr (H1) {
          *reinterpret_cast<uint2*>(dst) = uint2{b.w[0], b.w[1]};
          *reinterpret_cast<uint2*>(dst + kHalf) = uint2{b.w[2], b.w[3]};
        } else {
          *reinterpret_cast<uint4*>(dst) = uint4{b.w[0], b.w[1], b.w[2], b.w[3]};
          *reinterpret_cast<uint4*>(dst + kHalf) = uint4{b.w[4], b.w[5], b.w[6], b.w[7]};
        }
        qm[wv][slot] = int2{(int)pt, ao};
      }
      const int c = __popcll(m);
      qh = (qh + c) & 127;
      qn += c;
      qtot += c;
      if (qn >= 64) {
        if (!(a.abl & 1)) drain(((qh - qn) & 127) >> 6, 64);
        qn -= 64;
      }
    }
  };
  for (int64_t G = wave; G < ngroups; G += PD * gs) {
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      const int64_t Gi = G + i * gs;
      if (Gi >= ngroups) break;
      load(buf[(i + PD - 1) % PD], Gi + (PD - 1) * gs);
      wait(buf[i], PD - 1);
      process(buf[i], Gi);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the reloads past the end
  if (qn > 0) {  // the partial block (queue tail at a block start: 64 | qh - qn)
    drain(((qh - qn) & 127) >> 6, qn);
  }
  // per-wave counts only (their sum is the step's fallback total, formed by
  // the finalize): thousands of same-address atomics at the end of this
  // kernel serialised in L2 for tens of microseconds
  if (lane == 0) {
    a.fb_count[wave] = fb_used;
    a.mv_count[wave] = mv_used;
    if (a.q_acc) a.q_acc[wave] += qtot;  // (profiling) this wave's own slot
  }
  if (!a.fuse) return;
  // ---- fixup32's work for this workgroup's four waves, fused: no extra
  // launch, and the tail of one workgroup overlaps the others' streaming ----
  __syncthreads();  // every queue drained (its LDS becomes the table); lists written
  const FixLds L(qlds);
  if (lane == 0) {
    L.s_mv[wv + 1] = mv_used;
    L.s_fb[wv + 1] = fb_used;
  }
  fixup_regions<Q, MT>(a.fx, blockIdx.x * 4, 4, blockIdx.x % kRunSlices, L, FixPlan{sA, sC});
}

// ---------------------------------------------------------------------------
// Bounded DELTA screen: screen32b (device loop; d <= 16, k <= 64: configs 2, 3).
//
// screen32p still reads every point's 32-byte hi copy every step.  After the
// first steps almost every point keeps its label by a wide margin and the
// centroids move little, so a point's distances can be bounded across steps
// instead of recomputed (Hamerly's bounds, SURVEY.md §7 hard parts (c): exact,
// the same labels, less work).  With t_j(s) = ||xhat - chat_j(s)|| (the
// reference's distance up to 2^sigma) and the centroid drifts
// delta_j(s) >= ||chat_j(s) - chat_j(s - 1)||, M(s) = max_j delta_j(s):
//   t_a(t) <= t_a(t0) + sum_{t0 < s <= t} delta_a(s),
//   min_{j != a} t_j(t) >= min_{j != a} t_j(t0) - sum_{t0 < s <= t} M(s).
// ll_finalize32 keeps the cumulative W_j(t) = sum_{s <= t} (M(s) + delta_j(s))
// as exact int64 multiples of 2^-40 (every increment rounded up) and hands
// this step W_j rounded up and down to fp32 (wup / wdn).  A point whose label
// a was decided at step t0 with rigorous bounds u0 >= t_a(t0) and
// l0 <= min_{j != a} t_j(t0) stores ONE word
//   Z = l0 (1 - 2^-20) - u0 + wdn_a(t0)     (rounded down; low 6 bits: a)
// and keeps a at step t when Z > wup_a(t): then
//   min_{j != a} t_j(t) > t_a(t) + 2^-20 l0 > t_a(t) (1 + 2^-22),
// far above the reference's fp64 rounding (< 2^-45), so np.argmin of the
// reference's norms is a (src/kmeans_plusplus.py:33-34) and the point's
// coordinates are not read at all.
//
// Per wave: phase 1 streams the bound words (4 per lane, 1 KiB per load, four
// chunks in flight) and lists the points that fail in LDS; phase 2 gathers
// those points' hi rows (AoS copy XH, one line per point) 64 at a time, one
// batch ahead, and decides them exactly as screen32p does (triangle test
// against c32_a, else screen32h's k-way screen and hi-only certificate, else
// the exact fallback of the fused fixup), writing the point's new word:
//   triangle kept:  u0 = ub_a, l0 = h_a (1 - 2^-22) - ub_a;
//   k-way certified (label b, keys vb <= vs):
//     u0 = sqrt(vb (1 + 2^-16) + thr0 + ||h||^2_up - D_lo) (1 + 2^-19) + dn,
//     l0 = sqrt(vs - thr0 - D_hi + ||h||^2_lo) (1 - 2^-19) - dn
//     (|S_j - exact| <= E < thr0 / 2: thr0 also covers the fp32 rounding of
//     these sums; every other key is >= vs);
//   uncertified: "no bound" (kZbStale | old label; the fixup rewrites the
//     label if the exact decision moves the point).
// Moves and fallbacks go to the same per-wave lists as screen32p's, and the
// fused fixup finishes the step, so labels and int64 running sums are those
// of the full screen.
// ---------------------------------------------------------------------------
#ifndef CDR_S32BS_DEPTH
#define CDR_S32BS_DEPTH 2  // gathered batches in flight in screen32bs's phase 2 (experiments: 3)
#endif
#ifndef CDR_S32BS_LAZY
#define CDR_S32BS_LAZY 1  // screen32bs: phase 2 interleaved with the stream (0: in bursts)
#endif
constexpr int kBChunk = 256;  // points per wave-chunk of the bound stream (4 per lane)
constexpr int kBList = 512;   // per-wave LDS list of the points whose bound failed
constexpr int kBPD = 4;       // chunks in flight per wave (phase 1)

struct S32BArgs {
  S32PArgs p;                // the pruned screen's plan, lists and fused fixup
  const unsigned char* XH;   // AoS hi-only copy: 2 x 16 B (d <= 8: 2 x 8 B) per point
  uint32_t* zb;              // per point: Z bits | label (n_pad words)
  const float* wup;          // [64] W_j of this step's centroids, rounded up
  const float* wdn;          // [64] rounded down
  int64_t nchunks;           // n_pad / kBChunk
  long long* t_acc;          // profiling: points whose bound failed, per wave (null: off)
  int dbg;                   // tests only (CDR_BOUNDS_DBG): 1 = every bound fails
  unsigned long long* tprof; // experiments build only: per-wave timestamps (null: off)
  // screen32bs: chunk shares per CU slot (the workgroups blockIdx / slot_wg
  // = s share chunks [R_s, R_s+1) in proportion wsl[s]); slot_wg 0: one
  // strided split over all waves
  int slot_wg;
  int wsl[4];
  // split form (screen32bz streams the words, screen32bs<Q, MT, true> decides):
  // per-wave lists of the failed points in screen32bz's entry format, their
  // lengths, and the entries each list has room for
  uint32_t* zl;
  int32_t* zn;
  int64_t zcap;
  // the fused screen32bs: 2-byte words and their tables in
  // Ctx::bnd (plan32.h kBnd*)
  uint16_t* zh;
  const unsigned char* bt;
  // the 2-byte screen's dynamic tail (slot_wg > 0; null: off): each
  // generation region streams its first dyn_pct % statically (strided over
  // its waves) and hands the rest out kBPD chunks at a time from a counter
  // (dyn[((par * 4 + region) * 8 + xcd) * 32]: per XCD, a 128-byte line
  // each; the launch zeroes the other parity's counters for the next one)
  unsigned* dyn;
  int dyn_par, dyn_pct;
};
constexpr int kZ16Chunk = 512;  // points per wave-chunk of the 2-byte word stream (8 per lane)
// the dynamic tail's static percent (100: off; 90: 3-5 us less per config-3
// step than 100, profiles/r05_dynamic_tail_ab.txt)
constexpr int kS32DynPct = 90;
// ... from this many chunks per wave: a wave's last claim (the one that finds
// the pool empty) is an exposed atomic round trip, and with a few chunks per
// wave the tail costs more than it balances (12.5M x 16: 0.050 ms per step
// without, 0.055 with; 10M x 8: 0.036 / 0.040)
constexpr int kS32DynMinChunks = 24;

// The chunks wave `wv` of this workgroup streams: wbase + i * wstride below
// wend.  With slot_wg > 0 the workgroups of one CU slot (launch generation)
// share a region in proportion to its weight: the later generations on a CU
// get fewer issue slots (oldest-first) and otherwise finish last.
__device__ __forceinline__ void bs_range(const S32BArgs& B, int wv, int64_t& wbase, int& wstride,
                                         int64_t& wend, int64_t* rr0 = nullptr,
                                         int* rsl = nullptr) {
  const int64_t nchunks = B.nchunks;
  wbase = (int64_t)blockIdx.x * 4 + wv;
  wend = nchunks;
  wstride = (int)gridDim.x * 4;
  if (B.slot_wg < 0) {
    // contiguous ranges: wave w streams chunks [w cpw, (w + 1) cpw), so the
    // rows its failed points gather lie in one ~cpw * 16 KiB stretch of the
    // row-major copy (a few pages: the gathers stay TLB-resident) instead of
    // spread over the whole copy
    const int64_t nw = (int64_t)gridDim.x * 4, cpw = (nchunks + nw - 1) / nw;
    wbase = wbase * cpw;
    wend = wbase + cpw < nchunks ? wbase + cpw : nchunks;
    wstride = 1;
  } else if (B.slot_wg > 0) {
    const int ns = (int)gridDim.x / B.slot_wg;
    const int sl = (int)blockIdx.x / B.slot_wg;
    int wsum = 0, wpre = 0;
    for (int q = 0; q < ns; ++q) {
      wsum += B.wsl[q];
      if (q < sl) wpre += B.wsl[q];
    }
    const int64_t R0 = nchunks * wpre / wsum, R1 = nchunks * (wpre + B.wsl[sl]) / wsum;
    wstride = B.slot_wg * 4;
    wbase = R0 + (int64_t)((int)blockIdx.x - sl * B.slot_wg) * 4 + wv;
    wend = R1;
    if (rr0) *rr0 = R0;
    if (rsl) *rsl = sl;
  }
  wbase = __builtin_amdgcn_readfirstlane((int)wbase);
}

// Host mirror of bs_range: the most chunks any wave of the grid streams.
// the largest generation region (chunks; slot_wg > 0)
static int64_t bs_max_region(const S32BArgs& B, int nwg) {
  const int ns = nwg / B.slot_wg;
  int wsum = 0;
  for (int q = 0; q < ns; ++q) wsum += B.wsl[q];
  int64_t mx = 0, wpre = 0;
  for (int q = 0; q < ns; ++q) {
    mx = std::max<int64_t>(mx, B.nchunks * (wpre + B.wsl[q]) / wsum - B.nchunks * wpre / wsum);
    wpre += B.wsl[q];
  }
  return mx;
}

static int64_t bs_max_chunks(const S32BArgs& B, int nwg) {
  const int64_t nchunks = B.nchunks;
  if (B.slot_wg <= 0) return ceil_div(nchunks, (int64_t)nwg * 4);  // (strided or contiguous)
  const int ns = nwg / B.slot_wg;
  int wsum = 0;
  for (int q = 0; q < ns; ++q) wsum += B.wsl[q];
  int64_t mx = 0, wpre = 0;
  for (int q = 0; q < ns; ++q) {
    const int64_t R0 = nchunks * wpre / wsum, R1 = nchunks * (wpre + B.wsl[q]) / wsum;
    mx = std::max<int64_t>(mx, ceil_div(R1 - R0, (int64_t)B.slot_wg * 4));
    wpre += B.wsl[q];
  }
  return mx;
}

// The stored word of bounds (l0, u0) and W_a rounded down (see above):
// Z = l0 (1 - 2^-20) - u0 + w minus 2^-21 (|l0| + u0 + w), which covers the
// three fp32 roundings of the sum; no usable bound -> -1 (the test fails).
__device__ __forceinline__ unsigned zb_pack(float l0, float u0, float w, unsigned label) {
  if (!(l0 > 0.0f) || !(u0 >= 0.0f) || !(w >= 0.0f)) return 0xBF800000u | label;
  l0 = fminf(l0, 0x1p60f) * (1.0f - 0x1p-20f);
  const float s = (l0 - u0) + w;
  const float m = 0x1p-21f * ((l0 + u0) + w);
  const float z = s - m;
  return (z > 0.0f ? (__float_as_uint(z) & ~63u) : 0xBF800000u) | label;
}

// The 2-byte word of a decided point: zb_pack's Z relative to the point's
// base (w = W_a - G_a rounded down), truncated to its code (plan32.h); no
// bound (code 0) when Z <= G_a + 2^E0.
__device__ __forceinline__ unsigned short zb16_pack(float l0, float u0, float w, int e0,
                                                    unsigned label) {
  if (!(l0 > 0.0f) || !(u0 >= 0.0f) || !(w >= 0.0f)) return (unsigned short)label;
  l0 = fminf(l0, 0x1p60f) * (1.0f - 0x1p-20f);
  const float s = (l0 - u0) + w;
  const float m = 0x1p-21f * ((l0 + u0) + w);
  int c = zb16_code(s - m, e0);
  c = c < 0 ? 0 : (c > 1022 ? 1022 : c);
  return (unsigned short)((unsigned)c << 6 | label);
}
// A kept word carried to a new base (G_a grows by dg >= the exact step) and
// exponent: dec(code) - dg rounded down, then truncated; codes 0 and 1023 stay
__device__ __forceinline__ unsigned zb16_rebase(unsigned w, float dg, int e0o, int e0n) {
  const unsigned c = w >> 6;
  if (c == 0u || c == 1023u) return w;
  const float t = zb16_dec((int)c, e0o) - dg;  // |error| <= 2^-24 |t|
  int cn = t > 0.0f ? zb16_code(t * (1.0f - 0x1p-22f), e0n) : -1;
  cn = cn < 0 ? 0 : (cn > 1022 ? 1022 : cn);
  return (unsigned)cn << 6 | (w & 63u);
}

template <int Q, int MT>
__global__ __launch_bounds__(256, 4) void screen32b(S32BArgs B) {
  const S32PArgs& a = B.p;
  constexpr int QH = FixDims<Q>::QH;
  if (a.gate && a.gate[0] == 0) return;
  constexpr bool H1 = QH == 1;
  constexpr int kTile = H1 ? 512 : 1024;  // bytes per 32-point tile of the queue
  constexpr int kHalf = kTile / 2;
  constexpr int kPB = H1 ? 8 : 16;        // bytes per (point, half)
  constexpr int NWH = kPB / 4;            // dwords per point half
  constexpr int kRow = 2 * kPB;           // bytes per point in XH
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) float c32s[64 * kPrStr + 128];
  float* const eb = c32s + 64 * kPrStr;  // E_j
  float* const hc = eb + 64;             // h_j
  // per wave: the k-way queue (screen32p's ring) and, after the last drain,
  // the fused fixup's table (FixLds)
  constexpr size_t kQBytes = 4 * 2 * 2 * kTile + 4 * 128 * sizeof(int2);
  __shared__ __attribute__((aligned(16))) unsigned char qlds[kQBytes > kFixLdsBytes ? kQBytes : kFixLdsBytes];
  typedef unsigned char QRow[2][2 * kTile];
  QRow* qd = reinterpret_cast<QRow*>(qlds);
  int2 (*qm)[128] = reinterpret_cast<int2 (*)[128]>(qlds + 4 * 2 * 2 * kTile);
  // per wave: points whose bound failed, (chunk iteration << 14 | offset << 6 | label)
  __shared__ unsigned flist[4][kBList];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wv);
  const int nwaves = gridDim.x * 4;
  const int64_t nchunks = B.nchunks;

  // ---- phase 1 loads: the first chunks overlap the prologue ----
  // Ordinary loads (the compiler's s_waitcnt counts them): every iteration
  // issues exactly one, a chunk past the end reloads the last one, so the
  // counts are the same on every path and kBPD - 1 chunks stay in flight.
  auto zload = [&](u4v& z, int64_t ci) __attribute__((always_inline)) {
    const int64_t cc = ci < nchunks ? ci : nchunks - 1;  // past the end: reload the last
    z = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(B.zb + cc * kBChunk) + lane);
  };
  u4v zc[kBPD];
#pragma unroll
  for (int i = 0; i < kBPD - 1; ++i) zload(zc[i], wave + (int64_t)i * nwaves);

  // ---- the plan (screen32p's staging, one round trip) ----
  __shared__ h8 sA[MT * 2 * 64];
  __shared__ __attribute__((aligned(16))) float sC[MT * 4 * 2 * 4];
  constexpr int kPr4 = (64 * kPrStr + 128) / 4;
  static_assert(kPr4 <= 512 && MT * 2 * 64 <= 256, "prologue: two float4 per thread");
  const f4* prune4 = reinterpret_cast<const f4*>(a.prune);
  const f4 pv0 = prune4[t];
  const f4 pv1 = t + 256 < kPr4 ? prune4[t + 256] : f4{0.f, 0.f, 0.f, 0.f};
  h8 av = {};
  if (t < MT * 2 * 64) av = a.frag[t];
  float cv = 0.0f;
  const int cm = t >> 5, ci4 = (t >> 3) & 3, chh = (t >> 2) & 1, cc = t & 3;
  if (t < MT * 32) cv = a.cinit[(cm * 16 + ci4 * 4 + cc) * 64 + chh * 32];
  const float wup_l = B.wup[lane], wdn_l = B.wdn[lane];  // lane j: W_j (k <= 64)
  const float thr0 = a.thr_dev ? a.thr_dev[0] : a.thr0, thr_rel = a.thr_rel;
  const float Dv = a.thr_dev ? a.thr_dev[1] : a.Dv;
  const float Dlo = Dv * (1.0f - 0x1p-19f), Dhi = Dv * (1.0f + 0x1p-19f);  // D_lo < D < D_hi
  reinterpret_cast<f4*>(c32s)[t] = pv0;
  if (t + 256 < kPr4) reinterpret_cast<f4*>(c32s)[t + 256] = pv1;
  if (t < MT * 2 * 64) sA[t] = av;
  if (t < MT * 32) sC[t] = cv;
  __syncthreads();

  int2* fb_region = a.fb_list + (size_t)wave * a.cap;
  int2* mv_region = a.mv_list + (size_t)wave * a.cap;
  int fb_used = 0, mv_used = 0;
  struct Row {
    unsigned w[2 * NWH];  // the point's hi row: half 0 then half 1 (packed fp16 pairs)
  };
  // q = ||h - c32_j||^2 (screen32p's dist2)
  auto dist2 = [&](const Row& b, int j) __attribute__((always_inline)) -> float {
    const f4* c4 = reinterpret_cast<const f4*>(c32s + j * kPrStr);
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 acc = {0.0f, 0.0f};
#pragma unroll
    for (int q = 0; q < NWH; ++q) {
      const f4 cq = c4[q];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = 2 * q + u;
        const f2 df = {mix_sub_lo(b.w[i], cq[2 * u]), mix_sub_hi(b.w[i], cq[2 * u + 1])};
        acc = __builtin_elementwise_fma(df, df, acc);
      }
    }
    return acc.x + acc.y;
  };
  // (best, runner-up) keys of one 32-point tile of queued points (screen32p's tile)
  auto tile = [&](const u4v& v, unsigned& bk, unsigned& sk, float& hp) __attribute__((always_inline)) {
    const h8 BH = __builtin_bit_cast(h8, v);
    hp = 0.0f;
#pragma unroll
    for (int i = 0; i < (H1 ? 4 : 8); i += 2)
      hp = __builtin_amdgcn_fdot2(h2{BH[i], BH[i + 1]}, h2{BH[i], BH[i + 1]}, hp, false);
    unsigned b = 0xFFFFFFFFu, s = 0xFFFFFFFFu;
#pragma nounroll
    for (int m = 0; m < MT; ++m) {
      h8 A0 = sA[(m * 2 + 0) * 64 + lane];
      const h8 A1 = sA[(m * 2 + 1) * 64 + lane];
      if constexpr (H1)
#pragma unroll
        for (int i = 0; i < 4; ++i) A0[4 + i] = A1[i];
      f16v acc;
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const f4 c4v = *reinterpret_cast<const f4*>(sC + ((m * 4 + i4) * 2 + (lane >> 5)) * 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[4 * i4 + i] = c4v[i];
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, BH, acc, 0, 0, 0);
      if constexpr (!H1) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, BH, acc, 0, 0, 0);
      const unsigned rb = 32u * (unsigned)m;
      auto key = [&](int i) {
        return (__float_as_uint(acc[i]) & ~63u) | (rb + (unsigned)(8 * (i >> 2) + (i & 3)));
      };
#pragma unroll
      for (int q = 0; q < 16; q += 2) {
        const unsigned x = key(q), y = key(q + 1);
        unsigned tq;
        asm("v_med3_u32 %0, %1, %2, %3" : "=v"(tq) : "v"(b), "v"(x), "v"(y));
        asm("v_min3_u32 %0, %1, %2, %3" : "=v"(b) : "v"(b), "v"(x), "v"(y));
        s = min(s, tq);
      }
    }
    bk = b | ((unsigned)(lane >> 5) << 2);
    sk = s | ((unsigned)(lane >> 5) << 2);
  };
  // the k-way screen of queue block qb (nvalid entries), its lists and bound words
  auto drain = [&](int qb, int nvalid) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's queue writes
    const unsigned char* src = qd[wv][qb];
    u4v v[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      if constexpr (H1) {
        const uint2 x = *reinterpret_cast<const uint2*>(src + tt * kTile + lane * kPB);
        v[tt] = u4v{x.x, x.y, x.x, x.y};
      } else {
        v[tt] = *reinterpret_cast<const u4v*>(src + tt * kTile + lane * kPB);
      }
    }
    const int2 meta = qm[wv][qb * 64 + lane];  // lane l owns entry l after the swap
    unsigned bA = 0, sA_ = 0, bB = 0, sB = 0;
    float hA = 0.0f, hB = 0.0f;
#pragma nounroll
    for (int tt = 0; tt < 2; ++tt) {
      unsigned bk, sk;
      float hp;
      tile(tt == 0 ? v[0] : v[1], bk, sk, hp);
      if (tt == 0) {
        bA = bk;
        sA_ = sk;
        hA = hp;
      } else {
        bB = bk;
        sB = sk;
        hB = hp;
      }
    }
    swap32(bA, bB);
    swap32(sA_, sB);
    merge_top2(bA, sA_, bB, sB);
    const int label = (int)(bA & 63u);
    const float vb = __uint_as_float(bA & ~63u);
    const float vs = __uint_as_float(sA_ & ~63u);
    float thr = fmaf(vb, thr_rel, thr0);
    unsigned ua = __float_as_uint(hA), ub = __float_as_uint(hB);
    swap32(ua, ub);
    const float hsum = __uint_as_float(ua) + __uint_as_float(ub);
    const float hh = fmaf(hsum, 1.0f + 0x1p-18f, 0x1p-20f);  // >= ||h||^2
    const float hl = hsum * (1.0f - 0x1p-18f);               // <= ||h||^2
    const float dn = fmaf(0x1p-11f * (1.0f + 0x1p-9f), __builtin_amdgcn_sqrtf(hh), 0x1p-23f);
    {  // the hi-only certificate (screen32d)
      const float K = thr0 + hh - Dlo;
      const float Gs = fmaxf(vs + K, 0x1p-100f), Gb = fmaxf(fmaf(vb, thr_rel, K), 0x1p-100f);
      thr += 2.0f * (1.0f + 0x1p-19f) * dn * (__builtin_amdgcn_sqrtf(Gs) + __builtin_amdgcn_sqrtf(Gb));
    }
    const bool valid = lane < nvalid;
    const bool cert = vs > thr;  // NaN: never certified
    const int pt = meta.x, ob = meta.y;
    const bool moved = valid && cert && label != ob;
    if (moved) {
      a.labels[pt] = label;
      a.lab8[pt] = (uint8_t)label;
    }
    // the point's bound word: from its best and runner-up keys, or "no bound"
    const float gb = fmaf(vb, thr_rel, thr0 + hh - Dlo);
    const float gs = vs - ((thr0 + Dhi) - hl);
    const float u0 = fmaf(__builtin_amdgcn_sqrtf(fmaxf(gb, 0.0f)), 1.0f + 0x1p-19f, dn);
    const float l0 = fmaf(__builtin_amdgcn_sqrtf(fmaxf(gs, 0.0f)), 1.0f - 0x1p-19f, -dn);
    const float wl = __shfl(wdn_l, label);
    if (valid) B.zb[pt] = cert ? zb_pack(l0, u0, wl, (unsigned)label) : (kZbStale | (unsigned)ob);
    const bool unc = valid && !cert;
    const unsigned long long mv = __ballot(moved);
    const unsigned long long need = __ballot(unc);
    const int rm = __builtin_amdgcn_mbcnt_hi((unsigned)(mv >> 32),
                                             __builtin_amdgcn_mbcnt_lo((unsigned)mv, 0u));
    const int rn = __builtin_amdgcn_mbcnt_hi((unsigned)(need >> 32),
                                             __builtin_amdgcn_mbcnt_lo((unsigned)need, 0u));
    if (moved) mv_region[mv_used + rm] = int2{pt, ob | (label << 16)};
    if (unc) fb_region[fb_used + rn] = int2{pt, ob};
    mv_used += __popcll(mv);
    fb_used += __popcll(need);
  };
  int qh = 0, qn = 0;  // k-way queue head (next slot, mod 128) and length: wave-uniform
  int qtot = 0, ttot = 0;
  // one gathered point per lane: the triangle test, else the k-way queue
  auto process = [&](const Row& b, bool valid, int pt, int ao) __attribute__((always_inline)) {
    const float qa = dist2(b, ao);
    const float uba = fmaf(__builtin_amdgcn_sqrtf(qa), 1.0f + 0x1p-18f, eb[ao]);
    const float l0 = fmaf(hc[ao], 1.0f - 0x1p-22f, -uba);
    const bool keep = l0 > uba * (1.0f + 0x1p-20f);
    if (valid && keep) B.zb[pt] = zb_pack(l0, uba, __shfl(wdn_l, ao), (unsigned)ao);
#ifdef CDR_EXPERIMENTS
    const bool q = valid && !keep && !(B.dbg & 8);  // (timing: no k-way screen)
#else
    const bool q = valid && !keep;
#endif
    const unsigned long long m = __ballot(q);
    if (m) {
      if (q) {
        const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        const int slot = (qh + r) & 127;
        const int e = slot & 63;
        unsigned char* dst = qd[wv][slot >> 6] + (e >> 5) * kTile + (e & 31) * kPB;
        if constexpr (H1) {
          *reinterpret_cast<uint2*>(dst) = uint2{b.w[0], b.w[1]};
          *reinterpret_cast<uint2*>(dst + kHalf) = uint2{b.w[2], b.w[3]};
        } else {
          *reinterpret_cast<uint4*>(dst) = uint4{b.w[0], b.w[1], b.w[2], b.w[3]};
          *reinterpret_cast<uint4*>(dst + kHalf) = uint4{b.w[4], b.w[5], b.w[6], b.w[7]};
        }
        qm[wv][slot] = int2{pt, ao};
      }
      const int c = __popcll(m);
      qh = (qh + c) & 127;
      qn += c;
      qtot += c;
      if (qn >= 64) {
        drain(((qh - qn) & 127) >> 6, 64);
        qn -= 64;
      }
    }
  };
  // ---- phase 2: the listed points, 64 per batch, the next batch's rows in flight ----
  // The gathers are ordinary loads too: a load issued from inline asm leaves
  // a register the allocator may copy (at a join, around a call-sized block)
  // before the data lands, which the compiler's own counts never do.
  unsigned* const fl = flist[wv];
  struct GB {
    Row r;
    int pt, ao;
    bool valid;
  };
  auto gload = [&](GB& g, int b, int cnt) __attribute__((always_inline)) {
    const int e = 64 * b + lane;
    g.valid = e < cnt;
    const unsigned ent = fl[g.valid ? e : 64 * b];  // (entry 64 b exists)
    const int64_t ci = wave + (int64_t)(ent >> 14) * nwaves;
    const int64_t pt = ci * kBChunk + ((ent >> 6) & 255);
    g.pt = (int)pt;
    g.ao = (int)(ent & 63);
    const u4v* src = reinterpret_cast<const u4v*>(B.XH + pt * kRow);
    const u4v q0 = __builtin_nontemporal_load(src);
    g.r.w[0] = q0.x; g.r.w[1] = q0.y; g.r.w[2] = q0.z; g.r.w[3] = q0.w;
    if constexpr (!H1) {
      const u4v q1 = __builtin_nontemporal_load(src + 1);
      g.r.w[4] = q1.x; g.r.w[5] = q1.y; g.r.w[6] = q1.z; g.r.w[7] = q1.w;
    }
  };
  // every full batch of the list (all of it when `last`); a partial batch
  // stays at the front for the next call
  auto phase2 = [&](int& cnt, bool last) __attribute__((always_inline)) {
    const int nb = last ? (cnt + 63) >> 6 : cnt >> 6;
    if (nb == 0) return;
    ttot += last ? cnt : nb * 64;
#ifdef CDR_EXPERIMENTS
    if (B.dbg & 4) {  // timing experiments only: the listed points are not decided
      cnt = 0;
      return;
    }
#endif
    // three batches in flight: every slot is reloaded unconditionally (past
    // the end: the last batch again, not processed), so the compiler's
    // counts let the two later batches stay in flight while one is decided
    GB g[3];
    gload(g[0], 0, cnt);
    gload(g[1], nb > 1 ? 1 : 0, cnt);
    for (int b = 0; b < nb; b += 3) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int nx = b + i + 2;
        gload(g[(i + 2) % 3], nx < nb ? nx : nb - 1, cnt);
        if (b + i < nb) process(g[i].r, g[i].valid, g[i].pt, g[i].ao);
      }
    }
    const int done = nb * 64;
    const int rem = last ? 0 : cnt - done;
    if (rem > 0) {
      const unsigned v = lane < rem ? fl[done + lane] : 0u;
      __builtin_amdgcn_wave_barrier();
      if (lane < rem) fl[lane] = v;
    }
    cnt = rem;
  };

  // ---- phase 1: the bound words, 4 points per lane per chunk ----
  int cnt = 0;  // listed points (wave-uniform)
  int64_t it = 0;
  for (int64_t C0 = wave; C0 < nchunks; C0 += (int64_t)kBPD * nwaves) {
#pragma unroll
    for (int i = 0; i < kBPD; ++i, ++it) {
      const int64_t Ci = C0 + (int64_t)i * nwaves;
      if (Ci >= nchunks) break;
      zload(zc[(i + kBPD - 1) % kBPD], Ci + (int64_t)(kBPD - 1) * nwaves);
      const u4v z = zc[i];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const unsigned w = z[u];
        const unsigned lab = w & 63u;
#ifdef CDR_EXPERIMENTS
        const bool fail = (!(__uint_as_float(w & ~63u) > __shfl(wup_l, (int)lab)) || (B.dbg & 1)) &&
                          !(B.dbg & 16);  // (timing: the stream alone)
#else
        const bool fail = !(__uint_as_float(w & ~63u) > __shfl(wup_l, (int)lab)) || (B.dbg & 1);
#endif
        const unsigned long long m = __ballot(fail);
        if (m) {
          if (fail) {
            const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            fl[cnt + r] = (unsigned)it << 14 | (unsigned)(4 * lane + u) << 6 | lab;
          }
          cnt += __popcll(m);
        }
      }
      if (cnt > kBList - kBChunk) phase2(cnt, false);
    }
  }
  phase2(cnt, true);
  if (qn > 0) drain(((qh - qn) & 127) >> 6, qn);  // the partial queue block
  if (lane == 0) {
    a.fb_count[wave] = fb_used;
    a.mv_count[wave] = mv_used;
    if (a.q_acc) a.q_acc[wave] += qtot;
    if (B.t_acc) B.t_acc[wave] += ttot;
  }
#ifdef CDR_EXPERIMENTS
  if (B.dbg & 2) return;  // (timing: no fused fixup)
#endif
  if (!a.fuse) return;
  __syncthreads();  // every queue drained (its LDS becomes the table); lists written
  const FixLds L(qlds);
  if (lane == 0) {
    L.s_mv[wv + 1] = mv_used;
    L.s_fb[wv + 1] = fb_used;
  }
  fixup_regions<Q, MT>(a.fx, blockIdx.x * 4, 4, blockIdx.x % kRunSlices, L, FixPlan{sA, sC});
}

// ---------------------------------------------------------------------------
// screen32bz: phase 1 of the bounded screen as its own launch (the split form,
// CDR_S32BS_SPLIT=1; the fused kernel is the default).  Streams every
// point's bound word (4 per lane per 1 KiB chunk, KPD chunks in flight per
// wave) and lists the points whose bound fails in the
// wave's region of B.zl, in screen32bs's entry format (chunk iteration << 14 |
// offset << 6 | label); screen32bs<Q, MT, true> then decides the lists with
// every wave of the chip on the gathers and the MFMA screen.  In the fused
// form a wave stops streaming while it decides a batch, so the stream and the
// decisions add up; split, the stream is a plain HBM-bound pass (no plan, no
// LDS beyond the list staging, low register count) and the decisions run at
// full occupancy.  Entries are staged in LDS and written 64 at a time (one
// 256-byte store), so stores rarely sit between a chunk load and its use.
// ---------------------------------------------------------------------------
template <int KPD>
__global__ __launch_bounds__(256) void screen32bz(S32BArgs B) {
  const S32PArgs& a = B.p;
  if (a.gate && a.gate[0] == 0) return;
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  constexpr int kZList = KPD * kBChunk + 64;
  __shared__ unsigned flist[4][kZList];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wv);
  const int64_t nchunks = B.nchunks;
  int64_t wbase, wend;
  int wstride;
  bs_range(B, wv, wbase, wstride, wend);
  auto zload = [&](u4v& z, int64_t ci) __attribute__((always_inline)) {
    const int64_t cc = ci < nchunks ? ci : nchunks - 1;
    z = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(B.zb + cc * kBChunk) + lane);
  };
  u4v zc[KPD];
#pragma unroll
  for (int i = 0; i < KPD - 1; ++i) zload(zc[i], wbase + (int64_t)i * wstride);
  const float wup_l = B.wup[lane];  // lane j: W_j rounded up (k <= 64)
  unsigned* const fl = flist[wv];
  uint32_t* const out = B.zl + (size_t)wave * B.zcap;
  int cnt = 0, total = 0;
  int it = 0;
  for (int64_t C0 = wbase; C0 < wend; C0 += (int64_t)KPD * wstride) {
#pragma unroll
    for (int i = 0; i < KPD; ++i, ++it) {
      const int64_t Ci = C0 + (int64_t)i * wstride;
      if (Ci >= wend) break;
      zload(zc[(i + KPD - 1) % KPD], Ci + (int64_t)(KPD - 1) * wstride);
      const u4v z = zc[i];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const unsigned w = z[u];
        const unsigned lab = w & 63u;
        const bool fail = !(__uint_as_float(w & ~63u) > __shfl(wup_l, (int)lab)) || (B.dbg & 1);
        const unsigned long long m = __ballot(fail);
        if (m) {
          if (fail) {
            const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            fl[cnt + r] = (unsigned)it << 14 | (unsigned)(4 * lane + u) << 6 | lab;
          }
          cnt += __popcll(m);
        }
      }
    }
    if (cnt >= 64) {  // whole 64-entry rows out, the rest to the front
      const int full = cnt & ~63;
      __builtin_amdgcn_wave_barrier();
      for (int o = 0; o < full; o += 64) out[total + o + lane] = fl[o + lane];
      const int rem = cnt - full;
      const unsigned v = lane < rem ? fl[full + lane] : 0u;
      __builtin_amdgcn_wave_barrier();
      if (lane < rem) fl[lane] = v;
      total += full;
      cnt = rem;
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (lane < cnt) out[total + lane] = fl[lane];
  if (lane == 0) B.zn[wave] = total + cnt;
}

// ---------------------------------------------------------------------------
// screen32bs: the bounded screen deciding in registers (device loop; d <= 16,
// k <= 64).  Phase 1 is screen32b's.  Phase 2 gathers the listed points' fp32
// rows (XA: one 64-byte line per point at d = 16, the same memory
// transactions as screen32b's 32-byte hi row) and decides each batch of 64
// without a queue, a list or a fixup pass:
//   * xhat32 = fma(x, 2^sigma, -mu 2^sigma) (split_copy_kernel's values) and
//     the triangle test against c32_a with q = ||xhat32 - c32_a||^2 (the same
//     rounding count as screen32p's; E_a >= dn + ec covers ||xhat32 - xhat||
//     + ||c32_a - chat_a||, as it covers the fp16 row);
//   * when any lane of the batch fails it, the SPLIT screen of the whole batch
//     (screen32d's 2-3 MFMA per centroid tile on the hi / lo halves of
//     xhat32, formed in registers: one permlane32 swap per operand dword turns
//     the lanes' own rows into both 32-point B operands) and screen32d's
//     certificate vs > vb thr_rel + thr0, the K-case bounds from (vb, vs)
//     relative to xhat32 (|S_j - (D + ||chat_j||^2 - 2 chat_j . xhat32)| <= E
//     <= thr0 / 2), then the rounding of xhat32 (dn32 <= 2^-24 ||xhat32||);
//   * when any lane is not certified (near ties), fixup_regions' candidate set
//     (every key within the threshold of the best) evaluated in exact fp64
//     NumPy order: np.argmin of the reference's norms
//     (src/kmeans_plusplus.py:33-34); such a point keeps "no bound".
// Moves go into a per-workgroup int64 table in LDS ([k][d + 1], run_sums'
// layout) flushed into one run_sums slice at the end when the workgroup moved
// anything.  The split screen is ~2^8 tighter than the hi-only one, so almost
// no point needs the exact fp64 pass.
// SPLIT: phase 1 ran in screen32bz (same grid, so wave w decides the list of
// screen32bz's wave w and decodes its entries with the same chunk range); the
// batches come from that list, entries two batches ahead and rows one batch
// ahead of the decision.
// ---------------------------------------------------------------------------
template <int Q, int MT, bool SPLIT = false>
__global__ __launch_bounds__(256, 4) void screen32bs(S32BArgs B) {
  const S32PArgs& a = B.p;
  const FixArgs& F = a.fx;
#ifdef CDR_EXPERIMENTS
  unsigned long long tp[8] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0, 0, 0, 0};
#define CDR_TP(i) tp[i] = __builtin_amdgcn_s_memrealtime()
#else
#define CDR_TP(i)
#endif
  constexpr int QH = FixDims<Q>::QH;
  constexpr int DM = FixDims<Q>::DM;
  // near ties: the fused kernel lists them and resolves them after its last
  // batch (inlined in the streaming loop, the resolver costs registers and
  // code the stream needs); the split decide kernel resolves them at once
#ifndef CDR_S32BS_DEFER
#define CDR_S32BS_DEFER 1
#endif
  constexpr bool DEFER = !SPLIT && CDR_S32BS_DEFER;
  // the dynamic tail's counters for the next launch (the other parity; before
  // the gate, so a skipped launch leaves them zeroed too)
  if (!SPLIT && B.dyn && blockIdx.x == 0 && threadIdx.x < 32)
    B.dyn[((B.dyn_par ^ 1) * 32 + threadIdx.x) * 32] = 0u;
  if (a.gate && a.gate[0] == 0) return;
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  __shared__ __attribute__((aligned(16))) float c32s[64 * kPrStr + 128];
  float* const eb = c32s + 64 * kPrStr;  // E_j
  float* const hc = eb + 64;             // h_j
  // per wave: points whose bound failed (screen32b's entries); room for the
  // kBPD chunks streamed between two phase-2 passes, so phase 2 has one call
  // site (code size: the decision is inlined once)
  constexpr int kSList = kBPD * kBChunk + 256;
  __shared__ __attribute__((aligned(16))) unsigned flist[4][SPLIT ? 1 : kSList];
  __shared__ unsigned long long mtab[64 * 17];  // this workgroup's moves, [k][d + 1]
  __shared__ float msl[16];                     // -mu_f 2^sigma
  __shared__ unsigned tls[64];                  // 2-byte words: this step's code thresholds
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const int h = lane >> 5, p = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wv);
  const int64_t nchunks = B.nchunks;
  const int k = a.k, d = a.d, d1 = d + 1;

  // ---- phase 1 loads: 2-byte words, 8 per lane per 1 KiB chunk (the split
  // form: screen32bz streamed 4-byte words) ----
  // points per chunk and the entry format's chunk-iteration shift
  constexpr int CH = SPLIT ? kBChunk : kZ16Chunk;
  constexpr int SH = SPLIT ? 14 : 15;
  auto zload = [&](u4v& z, int64_t ci) __attribute__((always_inline)) {
    const int64_t cc = ci < nchunks ? ci : nchunks - 1;
    z = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(B.zh + cc * kZ16Chunk) + lane);
  };
  // this wave's chunks: wbase + i wstride below wend
  int64_t wbase, wend;
  int wstride;
  int64_t rR0 = 0;
  int rsl = 0;
  bs_range(B, wv, wbase, wstride, wend, &rR0, &rsl);
  // the dynamic tail (B.dyn): this wave's static chunks end at swend, the
  // region's pool [P0, wend) goes out kBPD chunks at a time from dctr
  // (chunk indices: int, below 2^31 - the host's n_pad)
  const bool dyn = !SPLIT && B.dyn != nullptr && B.slot_wg > 0;
  // The pool is split over the 8 XCDs (workgroup b runs on XCD b % 8), one
  // counter each in its own 128-byte line: claims on one address serialise
  // (~10 ns apart, measured), so one counter per region holds the waves up
  int swend = (int)wend, P0 = (int)wend, P1 = (int)wend;
  if (dyn) {
    const int spw = (int)((wend - rR0) * B.dyn_pct / 100 / wstride);  // static chunks per wave
    swend = (int)rR0 + spw * wstride;
    const int xcd = blockIdx.x & 7;
    P0 = swend + (int)((wend - swend) * xcd / 8);
    P1 = swend + (int)((wend - swend) * (xcd + 1) / 8);
  }
  // the entries' chunk field: region-relative chunk (dynamic tail) or the
  // chunk ordinal in this wave's range
  const int ebase = dyn ? (int)rR0 : (int)wbase;
  const int estride = dyn ? 1 : wstride;
  u4v zc[kBPD];

  // ---- the plan ----
  __shared__ h8 sA[MT * 2 * 64];
  __shared__ __attribute__((aligned(16))) float sC[MT * 4 * 2 * 4];
  constexpr int kPr4 = (64 * kPrStr + 128) / 4;
  static_assert(kPr4 <= 512 && MT * 2 * 64 <= 256, "prologue: two float4 per thread");
  const f4* prune4 = reinterpret_cast<const f4*>(a.prune);
  const f4 pv0 = prune4[t];
  const f4 pv1 = t + 256 < kPr4 ? prune4[t + 256] : f4{0.f, 0.f, 0.f, 0.f};
  h8 av = {};
  if (t < MT * 2 * 64) av = a.frag[t];
  float cv = 0.0f;
  const int cm = t >> 5, ci4 = (t >> 3) & 3, chh = (t >> 2) & 1, cc = t & 3;
  if (t < MT * 32) cv = a.cinit[(cm * 16 + ci4 * 4 + cc) * 64 + chh * 32];
  // lane j: W_j (4-byte words: wup for the test, wdn for new words); 2-byte
  // words: W_j - G_j for new words (the thresholds T_j: LDS, below) and the
  // codes' exponent
  float wup_l = 0.0f, wnew_l;
  int e0n = 0;
  if constexpr (SPLIT) {
    wup_l = B.wup[lane];
    wnew_l = B.wdn[lane];
  } else {
    wnew_l = reinterpret_cast<const float*>(B.bt + kBndWdg)[lane];
    e0n = reinterpret_cast<const int*>(B.bt + kBndHdr)[2];
  }
  // a decided point's word (ok: bounds (l0, u0); w = __shfl(wnew_l, lab),
  // taken by every lane) or "no bound"
  auto zput = [&](int pt, bool ok, float l0, float u0, float w, unsigned lab) __attribute__((always_inline)) {
    if constexpr (SPLIT) B.zb[pt] = ok ? zb_pack(l0, u0, w, lab) : (kZbStale | lab);
    else B.zh[pt] = ok ? zb16_pack(l0, u0, w, e0n, lab) : (unsigned short)lab;
  };
  const float msv = lane < d ? F.ms[lane] : 0.0f;        // lane f: -mu_f 2^sigma
  const float thr0 = a.thr_dev ? a.thr_dev[0] : a.thr0, thr_rel = a.thr_rel;
  const float Dv = a.thr_dev ? a.thr_dev[1] : a.Dv;
  const float Dlo = Dv * (1.0f - 0x1p-19f), Dhi = Dv * (1.0f + 0x1p-19f);
  const float sig = F.sig;
  reinterpret_cast<f4*>(c32s)[t] = pv0;
  if (t + 256 < kPr4) reinterpret_cast<f4*>(c32s)[t + 256] = pv1;
  if (t < MT * 2 * 64) sA[t] = av;
  if (t < MT * 32) sC[t] = cv;
  for (int e = t; e < 64 * 17; e += 256) mtab[e] = 0ull;
  if (t < 16) msl[t] = msv;
  if constexpr (!SPLIT) {
    // (CDR_BOUNDS_DBG=1, tests: every real point's bound fails)
    if (t < 64) tls[t] = (B.dbg & 1) ? 1022u : reinterpret_cast<const unsigned*>(B.bt + kBndT)[t];
  }
  __syncthreads();
  CDR_TP(1);

  int fb_used = 0, mv_used = 0, qtot = 0, ttot = 0;
  const f4* XA4 = reinterpret_cast<const f4*>(F.XA);  // point i: XA4[i * Q + q]

  // (best, runner-up) keys of one 32-point tile of the split screen
  auto screen_m = [&](int m, const u4v (&v)[QH]) __attribute__((always_inline)) -> f16v {
    asm volatile("" ::: "memory");  // the plan is read here, not held in registers
    const h8 A0 = sA[(m * 2 + 0) * 64 + lane];
    const h8 A1 = sA[(m * 2 + 1) * 64 + lane];
    f16v acc;
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4) {
      const f4 c4v = *reinterpret_cast<const f4*>(sC + ((m * 4 + i4) * 2 + h) * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[4 * i4 + i] = c4v[i];
    }
    const h8 BH = __builtin_bit_cast(h8, v[0]);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, BH, acc, 0, 0, 0);
    if constexpr (QH == 2) {
      const h8 BL = __builtin_bit_cast(h8, v[QH - 1]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, BL, acc, 0, 0, 0);
    }
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, BH, acc, 0, 0, 0);
  };
  auto tile = [&](const u4v (&v)[QH], unsigned& bk, unsigned& sk) __attribute__((always_inline)) {
    unsigned b = 0xFFFFFFFFu, s = 0xFFFFFFFFu;
#pragma nounroll
    for (int m = 0; m < MT; ++m) {
      const f16v acc = screen_m(m, v);
      const unsigned rb = 32u * (unsigned)m;
      auto key = [&](int i) {
        return (__float_as_uint(acc[i]) & ~63u) | (rb + (unsigned)(8 * (i >> 2) + (i & 3)));
      };
#pragma unroll
      for (int q = 0; q < 16; q += 2) {
        const unsigned x = key(q), y = key(q + 1);
        unsigned tq;
        asm("v_med3_u32 %0, %1, %2, %3" : "=v"(tq) : "v"(b), "v"(x), "v"(y));
        asm("v_min3_u32 %0, %1, %2, %3" : "=v"(b) : "v"(b), "v"(x), "v"(y));
        s = min(s, tq);
      }
    }
    bk = b | ((unsigned)h << 2);
    sk = s | ((unsigned)h << 2);
  };
  // candidate rows of tile v for the point of this lane's column (threshold
  // tau of that point): bit 16 m + i = value i of centroid tile m in half h
  auto cmask = [&](const u4v (&v)[QH], float tau) __attribute__((always_inline)) -> unsigned {
    unsigned r = 0;
#pragma nounroll
    for (int m = 0; m < MT; ++m) {
      const f16v acc = screen_m(m, v);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float kv = __uint_as_float(__float_as_uint(acc[i]) & ~63u);
        if (!(kv > tau)) r |= 1u << (16 * m + i);  // (NaN: a candidate)
      }
    }
    return r;
  };
  // q = ||xhat32 - c32_j||^2 in fp32: one rounding per difference, two fma
  // chains of <= 8 and one add, every term >= 0, so |q - exact| <= 2^-20 q
  // and |sqrt(q) - ||xhat32 - c32_j||| <= 2^-19 sqrt(q) (v_sqrt_f32: 1 ulp)
  auto q32 = [&](const float (&xh)[DM], int j) __attribute__((always_inline)) -> float {
    const f4* c4 = reinterpret_cast<const f4*>(c32s + j * kPrStr);
    f2 acc = {0.0f, 0.0f};
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const f4 cq = c4[q];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const f2 df = {xh[4 * q + 2 * u] - cq[2 * u], xh[4 * q + 2 * u + 1] - cq[2 * u + 1]};
        acc = __builtin_elementwise_fma(df, df, acc);
      }
    }
    return acc.x + acc.y;
  };
  struct GB {
    f4 x[Q];  // the point's fp32 row
    int pt, ao;
    bool valid;
  };
  // the split screen operands of the wave's 64 rows (lane l: point l): the
  // hi / lo halves of xhat32; lanes 0-31 keep their own half 0 for tile 0 and
  // receive lane 32 + p's half 0 for tile 1, lanes 32-63 receive lane p's
  // half 1 for tile 0 and keep their own half 1 for tile 1
  auto split_tiles = [&](const float (&xh)[DM], u4v (&T0)[QH], u4v (&T1)[QH]) __attribute__((always_inline)) {
    unsigned hw[4 * QH], lw[4 * QH];
#pragma unroll
    for (int qq = 0; qq < 2 * QH; ++qq) {
      f4 xt = {0.f, 0.f, 0.f, 0.f};
      if (qq < Q) xt = f4{xh[4 * qq], xh[4 * qq + 1], xh[4 * qq + 2], xh[4 * qq + 3]};
      split4(xt, hw[2 * qq], hw[2 * qq + 1], lw[2 * qq], lw[2 * qq + 1]);
    }
    unsigned ad[4 * QH], bd[4 * QH];  // quads 0 .. QH-1 | quads QH .. 2QH-1
    if constexpr (QH == 1) {  // [hi(q), lo(q)]
      ad[0] = hw[0]; ad[1] = hw[1]; ad[2] = lw[0]; ad[3] = lw[1];
      bd[0] = hw[2]; bd[1] = hw[3]; bd[2] = lw[2]; bd[3] = lw[3];
    } else {  // [hi(q0), hi(q1)], [lo(q0), lo(q1)]
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ad[i] = hw[i];
        ad[4 + i] = lw[i];
        bd[i] = hw[4 + i];
        bd[4 + i] = lw[4 + i];
      }
    }
#pragma unroll
    for (int i = 0; i < 4 * QH; ++i) swap32(ad[i], bd[i]);
#pragma unroll
    for (int u = 0; u < QH; ++u) {
      T0[u] = u4v{ad[4 * u], ad[4 * u + 1], ad[4 * u + 2], ad[4 * u + 3]};
      T1[u] = u4v{bd[4 * u], bd[4 * u + 1], bd[4 * u + 2], bd[4 * u + 3]};
    }
  };
  // (best, runner-up) keys of this lane's point over both tiles and halves
  auto keys = [&](const u4v (&T0)[QH], const u4v (&T1)[QH], unsigned& b, unsigned& s) __attribute__((always_inline)) {
    unsigned bB, sB;
    tile(T0, b, s);
    tile(T1, bB, sB);
    swap32(b, bB);
    swap32(s, sB);
    merge_top2(b, s, bB, sB);
  };
  auto rowhat = [&](const f4 (&x)[Q], float (&xh)[DM]) __attribute__((always_inline)) {
#pragma unroll
    for (int f = 0; f < DM; ++f) xh[f] = f < d ? fmaf(x[f >> 2][f & 3], sig, msl[f]) : 0.0f;
  };
  // a point leaving cluster ao for lab: labels and this workgroup's table
  // (row: the point's row when the caller holds it, else read again)
  auto move = [&](bool live, int pt, int ao, int lab, const f4* row) __attribute__((always_inline)) {
    const bool moved = live && lab != ao;
    const unsigned long long mm = __ballot(moved);
    if (!mm) return;
    if (moved) {
      a.labels[pt] = lab;
      a.lab8[pt] = (uint8_t)lab;
      f4 xr[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) xr[q] = row ? row[q] : XA4[(int64_t)pt * Q + q];
#pragma unroll
      for (int f = 0; f < DM; ++f) {
        if (f < d) {
          const long long v = __double2ll_rn((double)xr[f >> 2][f & 3] * F.fx);
          atomicAdd(&mtab[lab * d1 + f], (unsigned long long)v);
          atomicAdd(&mtab[ao * d1 + f], (unsigned long long)-v);
        }
      }
      atomicAdd(&mtab[lab * d1 + d], 1ull);
      atomicAdd(&mtab[ao * d1 + d], ~0ull);
    }
    mv_used += __popcll(mm);
  };
  int2* fb_region = a.fb_list + (size_t)wave * a.cap;
  // A point the split screen could not certify (a near tie; best key bkey):
  // every centroid whose key is within the threshold of the best is a
  // candidate (|S_j - T_j| <= E: the reference's argmin is among them); the
  // candidates' direct fp32 distances from the LDS c32 copy decide with
  // rigorous intervals, and only an interval overlap falls to the exact fp64
  // NumPy-order evaluation (np.argmin of the reference's norms,
  // src/kmeans_plusplus.py:33-34).  Every lane of the wave calls it (the
  // screen values come from MFMAs over the wave's 64 points); lanes with
  // live = false return ao.  c2: decided by the direct distances, with the
  // bounds (u0, l0) of its new bound word; otherwise the point keeps "no
  // bound".
  auto near_tie = [&](bool live, int ao, unsigned bkey, const float (&xh)[DM],
                      const u4v (&T0)[QH], const u4v (&T1)[QH], const f4 (&xr)[Q], float xx,
                      bool& c2, float& u0, float& l0) __attribute__((always_inline)) -> int {
    const double* cs = F.cent;
    const float tau = fmaf(__uint_as_float(bkey & ~63u), thr_rel, thr0);
    // tile tt's column p is the point of lane 32 tt + p, which holds its tau
    unsigned mine[2], other[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const float tau_t = __shfl(tau, 32 * tt + p);
      const unsigned r = cmask(tt == 0 ? T0 : T1, tau_t);
      mine[tt] = r;
      other[tt] = (unsigned)__shfl_xor((int)r, 32);
    }
    int lab = ao;
    c2 = false;
    u0 = l0 = 0.0f;
    if (live) {
      unsigned long long cand = 0;
      const unsigned mh0 = h == 0 ? mine[0] : other[1], mh1 = h == 0 ? other[0] : mine[1];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        unsigned mmk = hh ? mh1 : mh0;  // rows of half hh of this lane's tile
        while (mmk) {
          const int bb = __builtin_ctz(mmk);
          mmk &= mmk - 1;
          const int m = bb >> 4, i = bb & 15;
          cand |= 1ull << (32 * m + 8 * (i >> 2) + 4 * hh + (i & 3));
        }
      }
      if (k < 64) cand &= (1ull << k) - 1;
      // the candidates' direct fp32 distances (c32 in LDS): t_j = ||xhat -
      // chat_j|| lies within sqrt(q_j) (1 -+ 2^-19) -+ (dn32 + ec_j), where
      // dn32 >= ||xhat32 - xhat|| and ec_j >= ||c32_j - chat_j||: c32 is
      // the fp32 rounding of chat_j in fp64, so ec_j <= (2^-24 + 2^-51)
      // ||chat_j|| <= 2^-24 (1 + 2^-18) ||c32_j||
      const float xu = fmaf(xx, 1.0f + 0x1p-19f, 0x1p-120f);
      const float xl = xx * (1.0f - 0x1p-19f);
      const float dn32 = fmaf(0x1p-24f * (1.0f + 0x1p-20f), __builtin_amdgcn_sqrtf(xu), 0x1p-120f);
      float ub = INFINITY, lo_other = INFINITY, lb_best = INFINITY, rbest = INFINITY;
      int jb = 0;
      bool bad = false;  // a NaN distance: the exact pass decides
      unsigned long long cm2 = cand;
      while (cm2) {  // increasing j
        const int j = __builtin_ctzll(cm2);
        cm2 &= cm2 - 1;
        float nc;
        {
          const float zr[DM] = {};
          nc = q32(zr, j);  // ||c32_j||^2 (the same rounding bound)
        }
        const float ec = fmaf(0x1p-24f * (1.0f + 0x1p-18f),
                              __builtin_amdgcn_sqrtf(nc * (1.0f + 0x1p-19f)), 0x1p-120f);
        const float e2 = (dn32 + ec) * (1.0f + 0x1p-20f);
        const float r = __builtin_amdgcn_sqrtf(q32(xh, j));
        const float U = fmaf(r, 1.0f + 0x1p-19f, e2), L = fmaf(r, 1.0f - 0x1p-19f, -e2);
        bad = bad || !(U == U) || !(L == L);
        if (r < rbest) {
          lo_other = fminf(lo_other, lb_best);
          rbest = r;
          ub = U;
          lb_best = L;
          jb = j;
        } else {
          lo_other = fminf(lo_other, L);
        }
      }
      // every other centroid's key is above tau: its distance is at least
      const float gs = tau - ((thr0 + Dhi) - xl);
      const float lnc = fmaf(__builtin_amdgcn_sqrtf(fmaxf(gs, 0.0f)), 1.0f - 0x1p-19f, -dn32);
      c2 = !bad && rbest < INFINITY && lo_other > ub * (1.0f + 0x1p-20f);
      if (c2) {
        lab = jb;
        u0 = ub;
        l0 = fminf(lo_other, lnc);
      } else {
        float x[16];  // fp32 data, converted exactly where used
#pragma unroll
        for (int f = 0; f < 16; ++f) x[f] = f < DM ? xr[f >> 2][f & 3] : 0.0f;
        double sb = INFINITY, rb = INFINITY;
        int jmin = 0x7fffffff;
        while (cand) {  // increasing j
          const int j = __builtin_ctzll(cand);
          cand &= cand - 1;
          const double sq = np_sqdist16(x, cs + j * d, d);
          if (sq < sb) {  // sqrt is monotone: only a smaller square gives a smaller root
            const double rt = sqrt(sq);
            sb = sq;
            if (rt < rb) {
              rb = rt;
              jmin = j;
            }
          }
        }
        lab = jmin >= k ? 0 : jmin;  // every root NaN: np.argmin of all-NaN is 0
      }
    }
    return lab;
  };
  // one gathered batch: lane l decides point l
  auto decide = [&](const GB& g) __attribute__((always_inline)) {
    const bool valid = g.valid;
    const int pt = g.pt, ao = g.ao;
    float xh[DM];
    rowhat(g.x, xh);
    // triangle test: q = ||xhat32 - c32_a||^2
    const float qa = q32(xh, ao);
    const float uba = fmaf(__builtin_amdgcn_sqrtf(qa), 1.0f + 0x1p-18f, eb[ao]);
    const float l0P = fmaf(hc[ao], 1.0f - 0x1p-22f, -uba);
    const bool keep = l0P > uba * (1.0f + 0x1p-20f);
    const float w_ao = __shfl(wnew_l, ao);
    if (valid && keep) zput(pt, true, l0P, uba, w_ao, (unsigned)ao);
    const bool need = valid && !keep;
    const unsigned long long nm = __ballot(need);
    if (!nm) return;
    qtot += __popcll(nm);
#ifdef CDR_EXPERIMENTS
    if (B.dbg & 8) return;  // (timing: no k-way screen)
#endif
    // ||xhat32||^2 (fp32, 16 roundings at most: relative 2^-19 covers them)
    float xx;
    {
      f2 acc = {0.0f, 0.0f};
#pragma unroll
      for (int f = 0; f < DM; f += 2) {
        const f2 v = {xh[f], xh[f + 1]};
        acc = __builtin_elementwise_fma(v, v, acc);
      }
      xx = acc.x + acc.y;
    }
    unsigned bA, sA_;
    u4v T0[QH], T1[QH];
    split_tiles(xh, T0, T1);
    keys(T0, T1, bA, sA_);
    const int label = (int)(bA & 63u);
    const float vb = __uint_as_float(bA & ~63u);
    const float vs = __uint_as_float(sA_ & ~63u);
    const bool cert = vs > fmaf(vb, thr_rel, thr0);  // NaN: never certified
    const bool unc = need && !cert;
    const float w_lab = __shfl(wnew_l, label);
    // K-case: the point's bound word from its split keys
    if (need && cert) {
      const float xu = fmaf(xx, 1.0f + 0x1p-19f, 0x1p-120f);  // >= ||xhat32||^2
      const float xl = xx * (1.0f - 0x1p-19f);               // <= ||xhat32||^2
      const float dn32 = fmaf(0x1p-24f * (1.0f + 0x1p-20f), __builtin_amdgcn_sqrtf(xu), 0x1p-120f);
      const float gb = fmaf(vb, thr_rel, thr0 + xu - Dlo);
      const float gs = vs - ((thr0 + Dhi) - xl);
      const float u0 = fmaf(__builtin_amdgcn_sqrtf(fmaxf(gb, 0.0f)), 1.0f + 0x1p-19f, dn32);
      const float l0 = fmaf(__builtin_amdgcn_sqrtf(fmaxf(gs, 0.0f)), 1.0f - 0x1p-19f, -dn32);
      zput(pt, true, l0, u0, w_lab, (unsigned)label);
    }
    const unsigned long long um = __ballot(unc);
    if constexpr (DEFER) {
    // uncertified (near ties): the wave's list {point, best key}, resolved
    // after the workgroup's last batch
    if (um) {
      if (unc) {
        const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(um >> 32),
                                                __builtin_amdgcn_mbcnt_lo((unsigned)um, 0u));
        // (the best key's label bits carry the old label: near_tie reads
        // the key's value only, and the tail needs no lab8 load)
        fb_region[fb_used + r] = int2{pt, (int)((bA & ~63u) | (unsigned)ao)};
      }
      fb_used += __popcll(um);
    }
    move(need && cert, pt, ao, label, nullptr);
    } else {
    // uncertified (near ties, ~1 in 5 re-read points at config 3) resolved
    // now, while the row, the split operands and the best key are in
    // registers: no list, no dependent re-gather of the row and label
    int labf = label;
    if (um) {
#ifdef CDR_EXPERIMENTS
      if (!(B.dbg & 2)) {  // (timing: no near-tie pass)
#endif
      bool c2;
      float u0, l0;
      const int lab = near_tie(unc, ao, bA, xh, T0, T1, g.x, xx, c2, u0, l0);
      const float wl = __shfl(wnew_l, lab);
      if (unc) {
        labf = lab;
        zput(pt, c2, l0, u0, wl, (unsigned)lab);
      }
#ifdef CDR_EXPERIMENTS
      } else if (unc) {
        labf = ao;
      }
#endif
      fb_used += __popcll(um);
    }
    move(need, pt, ao, labf, g.x);
    }
  };

  // ---- phase 2: the listed points, 64 per batch, two batches in flight ----
  unsigned* const fl = flist[wv];
  auto gload = [&](GB& g, int b, int cnt) __attribute__((always_inline)) {
    const int e = 64 * b + lane;
    g.valid = e < cnt;
    const unsigned ent = fl[g.valid ? e : 64 * b];  // (entry 64 b exists)
    const int64_t ci = ebase + (int64_t)(ent >> SH) * estride;
    const int64_t pt = ci * CH + ((ent >> 6) & (CH - 1));
    g.pt = (int)pt;
    g.ao = (int)(ent & 63);
#pragma unroll
    for (int q = 0; q < Q; ++q) g.x[q] = __builtin_nontemporal_load(XA4 + pt * Q + q);
  };
  auto phase2 = [&](int& cnt, bool last) __attribute__((always_inline)) {
    const int nb = last ? (cnt + 63) >> 6 : cnt >> 6;
    if (nb == 0) return;
    ttot += last ? cnt : nb * 64;
#ifdef CDR_EXPERIMENTS
    if (B.dbg & 4) {  // (timing: the listed points are not decided)
      cnt = 0;
      return;
    }
#endif
    // the next batch's rows load while one is decided (past the end: the
    // last batch again, not decided); the copy waits for them after it
#if CDR_S32BS_DEPTH >= 3
    GB cur, nxt, nx2;
    gload(cur, 0, cnt);
    gload(nxt, nb > 1 ? 1 : 0, cnt);
#pragma nounroll
    for (int b = 0; b < nb; ++b) {
      gload(nx2, b + 2 < nb ? b + 2 : nb - 1, cnt);
      decide(cur);
      cur = nxt;
      nxt = nx2;
    }
#else
    GB cur, nxt;
    gload(cur, 0, cnt);
#pragma nounroll
    for (int b = 0; b < nb; ++b) {
      gload(nxt, b + 1 < nb ? b + 1 : nb - 1, cnt);
      decide(cur);
      cur = nxt;
    }
#endif
    const int done = nb * 64;
    const int rem = last ? 0 : cnt - done;
    if (rem > 0) {
      const unsigned v = lane < rem ? fl[done + lane] : 0u;
      __builtin_amdgcn_wave_barrier();
      if (lane < rem) fl[lane] = v;
    }
    cnt = rem;
  };

  if constexpr (SPLIT) {
    // ---- the list screen32bz's wave `wave` wrote: 64 entries per batch ----
    const uint32_t* const L = B.zl + (size_t)wave * B.zcap;
    const int total = B.zn[wave];
    const int nb = (total + 63) >> 6;
    ttot = total;
    if (nb > 0) {
      auto eload = [&](int b) __attribute__((always_inline)) -> unsigned {
        const int e = 64 * b + lane;
        return L[e < total ? e : 64 * b];  // (entry 64 b exists: b < nb)
      };
      auto fill = [&](GB& g, unsigned ent, int b) __attribute__((always_inline)) {
        g.valid = 64 * b + lane < total;
        const int64_t ci = wbase + (int64_t)(ent >> 14) * wstride;
        const int64_t pt = ci * kBChunk + ((ent >> 6) & 255);
        g.pt = (int)pt;
        g.ao = (int)(ent & 63);
#pragma unroll
        for (int q = 0; q < Q; ++q) g.x[q] = __builtin_nontemporal_load(XA4 + pt * Q + q);
      };
      GB cur, nxt;
      unsigned en = eload(0);
      fill(cur, en, 0);
      en = eload(nb > 1 ? 1 : 0);
#pragma nounroll
      for (int b = 0; b < nb; ++b) {
        // the next batch's rows and the one after's entries load while this
        // batch is decided (past the end: the last batch again, not decided)
        const int b1 = b + 1 < nb ? b + 1 : nb - 1;
        fill(nxt, en, b1);
        en = eload(b + 2 < nb ? b + 2 : nb - 1);
#ifdef CDR_EXPERIMENTS
        if (!(B.dbg & 4))  // (timing: the listed points are gathered, not decided)
#endif
        decide(cur);
        cur = nxt;
      }
    }
  } else {
#if CDR_S32BS_LAZY
  // Phase 2 interleaved with the stream: after every kBPD chunks the batch
  // whose rows were gathered one group of chunks earlier is decided and the
  // next 64 listed points' rows are gathered, so a batch's gather latency
  // hides behind the stream instead of stalling the wave.  Only when the
  // list would overflow (steps where most bounds fail) are batches decided
  // back to back.
  GB cur;
  bool pend = false;
  int head = 0;  // listed entries before head are gathered (wave-uniform)
  // (returns with room for one more chunk's entries: the stream breaks its
  // group early when a chunk would not fit, which only dense failures do)
  auto step2 = [&](int& cnt, bool last) __attribute__((always_inline)) {
    constexpr int kRoom = CH;
    for (;;) {
      if (pend) {
#ifdef CDR_EXPERIMENTS
        const unsigned long long td0 = __builtin_amdgcn_s_memrealtime();
        if (!SPLIT) __builtin_amdgcn_s_waitcnt(0x0F70);  // (timing: the gathered rows' arrival)
        const unsigned long long td1 = __builtin_amdgcn_s_memrealtime();
#endif
        decide(cur);
        pend = false;
#ifdef CDR_EXPERIMENTS
        const unsigned long long td2 = __builtin_amdgcn_s_memrealtime();
        tp[5] += td2 - td1;  // decide
        tp[6] += 1;          // batches
        tp[7] += td1 - td0;  // waiting for the rows (and the stream's loads)
#endif
      }
      const int avail = cnt - head;
      if (avail >= 64 || (last && avail > 0)) {
        const int e = head + lane;
        cur.valid = e < cnt;
        const unsigned ent = fl[cur.valid ? e : head];
        const int64_t ci = ebase + (int64_t)(ent >> SH) * estride;
        const int64_t pt = ci * CH + ((ent >> 6) & (CH - 1));
        cur.pt = (int)pt;
        cur.ao = (int)(ent & 63);
#pragma unroll
        for (int q = 0; q < Q; ++q) cur.x[q] = __builtin_nontemporal_load(XA4 + pt * Q + q);
        const int take = avail < 64 ? avail : 64;
        head = __builtin_amdgcn_readfirstlane(head + take);
        ttot += take;
        pend = true;
      }
      if (head > 0 && !last && cnt + kRoom > kSList) {  // compact [head, cnt) to the front
        const int m = cnt - head;
        for (int o = 0; o < m; o += 64) {  // (writes stay below the reads still to come)
          const int e2 = o + lane;
          const unsigned v = e2 < m ? fl[head + e2] : 0u;
          __builtin_amdgcn_wave_barrier();
          if (e2 < m) fl[e2] = v;
          __builtin_amdgcn_wave_barrier();
        }
        cnt = m;
        head = 0;
      }
      const bool again = last ? (pend || cnt > head) : (cnt - head + kRoom > kSList);
      if (!again) break;
    }
  };
#else
  constexpr int head = 0;  // (phase 2 in bursts compacts the list itself)
#endif

  // ---- phase 1: the bound words, 8 points per lane per chunk ----
  // Groups of kBPD chunks issued together, phase 2 between groups.  The waits
  // must stay exact: vmcnt counts stores too and is in order, so a store or a
  // reload between a chunk's load and its use made the compiler wait for
  // every load in flight (a rebase is zh_rebase_kernel's).  A chunk whose
  // entries would not fit the list (dense failures: the first bounded step)
  // hands the rest of the wave's range to a plain loop, one chunk at a time,
  // phase 2 draining the list whenever it must.
  int cnt = 0;
  int it = 0;  // chunk ordinal within this wave's range (the entries' high bits)
  auto insert = [&](const u4v& z, int ci) __attribute__((always_inline)) {
    const unsigned enc = dyn ? (unsigned)(ci - ebase) : (unsigned)it;
    // the 8 thresholds from LDS (independent reads, one wait), then the
    // tests; entries only from chunks with a failed point
    unsigned fm = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const unsigned w = (z[u >> 1] >> (16 * (u & 1))) & 0xFFFFu;
      fm |= (unsigned)((w >> 6) <= tls[w & 63u]) << u;
    }
#ifdef CDR_EXPERIMENTS
    if (B.dbg & 16) fm = 0;  // (timing: the stream alone)
#endif
    if (__ballot(fm != 0u)) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool fail = (fm >> u) & 1u;
        const unsigned long long m = __ballot(fail);
        if (m) {
          if (fail) {
            const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            fl[cnt + r] = enc << 15 | (unsigned)(8 * lane + u) << 6 |
                          ((z[u >> 1] >> (16 * (u & 1))) & 63u);
          }
          // (readfirstlane: uniform to the compiler, so the loops branch on
          // scalars and the waits stay exact)
          cnt = __builtin_amdgcn_readfirstlane(cnt + __popcll(m));
        }
      }
    }
    ++it;
  };
  // the group walk: chunks gC + i gS below gEnd (static: this wave's range;
  // then, with the dynamic tail, groups claimed from the region's pool)
  int gC = (int)wbase, gEnd = swend;
  bool dynph = false;
#define gS (dynph ? 1 : wstride)
  int ncl = -1;  // a claim made ahead: its pool offset (-1: none)
  // a wave claims while its near-tie region (a.cap points) holds the chunks
  // it may yet stream: the one in hand and the one claimed (the host sizes
  // the regions so the waves' budgets cover the pool)
#define budget (a.cap / CH - 2 * kBPD)
  auto claim = [&]() __attribute__((always_inline)) -> unsigned {
    unsigned v = 0;
    if (lane == 0)
      v = atomicAdd(B.dyn + ((B.dyn_par * 4 + rsl) * 8 + (blockIdx.x & 7)) * 32, (unsigned)kBPD);
    return v;
  };
  // the next group when the current phase is spent (uniform)
  auto next_group = [&]() __attribute__((always_inline)) -> bool {
    if (gC < gEnd) return true;
    if (!dyn) return false;
    dynph = true;
    if (ncl < 0) {
      if (it > budget) return false;
      ncl = (int)__builtin_amdgcn_readfirstlane(claim());
    }
    gC = P0 + ncl;
    ncl = -1;
    gEnd = gC + kBPD < P1 ? gC + kBPD : P1;
    return gC < gEnd;
  };
  int C0 = gC;
  bool dense = false;  // (wave-uniform) the plain loop takes over at chunk C0
  for (bool first = true;; first = false) {
    const bool more = next_group();  // (wave-uniform)
    // phase 2 first: the rows it gathers load under this group's stream, and
    // this group's loads are the youngest, so each chunk waits for itself
    // only (vmcnt(kBPD - 1 - i)) whatever phase 2 issued
#if CDR_S32BS_LAZY
    if (!first) step2(cnt, !more);
#else
    if (!first && (!more || cnt - head + CH > kSList - (kBPD - 1) * CH)) phase2(cnt, !more);
#endif
    if (!more) break;
#pragma unroll
    for (int i = 0; i < kBPD; ++i) {
      zload(zc[i], gC + i * gS);
      __builtin_amdgcn_sched_barrier(0);  // (issued in chunk order)
    }
    // the next dynamic group's claim, ahead of its use (returned under this
    // group's tests)
    const bool ahead = dyn && it <= budget && (dynph || gC + kBPD * gS >= gEnd);
    unsigned clv = 0;
    if (ahead) clv = claim();
#pragma unroll
    for (int i = 0; i < kBPD; ++i) {
      const int Ci = gC + i * gS;
      if (Ci >= gEnd) break;
      if (cnt - head + CH > kSList) {  // (dense failures only)
        dense = true;
        C0 = Ci;
        break;
      }
      insert(zc[i], Ci);
    }
    if (ahead) ncl = (int)__builtin_amdgcn_readfirstlane(clv);
    if (dense) break;
    gC = dynph ? gEnd : gC + kBPD * gS;
  }
  if (dense) {
    // the rest of the current group / phase one chunk at a time, then (the
    // dynamic tail) further claimed groups
    gC = C0;
    for (;;) {
      const bool more = next_group();
#if CDR_S32BS_LAZY
      if (!more || cnt - head + CH > kSList) step2(cnt, !more);  // (returns with room)
#else
      if (!more || cnt - head + CH > kSList) phase2(cnt, !more);
#endif
      if (!more) break;
      u4v z;
      zload(z, gC);
      insert(z, gC);
      gC += gS;
    }
  }
#undef gS
#undef budget
  }  // (!SPLIT)
  // ---- the uncertified points: the same split screen again (the same values),
  // every centroid whose key is within the threshold of the best is a
  // candidate (|S_j - T_j| <= E: the reference's argmin is among them), and
  // the candidates in exact fp64 NumPy order (fixup_regions' decision) from
  // an LDS copy of the step's centroids (the lists' LDS, free now) ----
  CDR_TP(2);
#ifdef CDR_EXPERIMENTS
  if (B.dbg & 2) fb_used = 0;  // (timing: no exact pass)
#endif
  if constexpr (DEFER) {
  // the next batch's records and rows load while one is decided
  // (Q = 4: the records only - the rows ahead too spill registers)
  constexpr int QA = Q < 4 ? Q : 0;
  auto tload = [&](int e0, int2& rec, f4 (&xr)[Q]) __attribute__((always_inline)) {
    const int e = e0 + lane;
    rec = fb_region[e < fb_used ? e : e0];
#pragma unroll
    for (int q = 0; q < QA; ++q) xr[q] = XA4[(int64_t)rec.x * Q + q];
  };
  int2 rec_n = {0, 0};
  f4 xr_n[Q];
  if (fb_used > 0) tload(0, rec_n, xr_n);
  for (int e0 = 0; e0 < fb_used; e0 += 64) {
    const int e = e0 + lane;
    const bool live = e < fb_used;
    const int2 rec = rec_n;
    f4 xr[Q];
#pragma unroll
    for (int q = 0; q < QA; ++q) xr[q] = xr_n[q];
#pragma unroll
    for (int q = QA; q < Q; ++q) xr[q] = XA4[(int64_t)rec.x * Q + q];
    if (e0 + 64 < fb_used) tload(e0 + 64, rec_n, xr_n);
    const int pt = rec.x;
    const int ao = rec.y & 63;  // (the record's: unchanged until this pass decides the point)
    float xh[DM];
    rowhat(xr, xh);
    u4v T0[QH], T1[QH];
    split_tiles(xh, T0, T1);
    float xx;
    {
      f2 acc = {0.0f, 0.0f};
#pragma unroll
      for (int f = 0; f < DM; f += 2) {
        const f2 v = {xh[f], xh[f + 1]};
        acc = __builtin_elementwise_fma(v, v, acc);
      }
      xx = acc.x + acc.y;
    }
    bool c2;
    float u0, l0;
    const int lab = near_tie(live, ao, (unsigned)rec.y, xh, T0, T1, xr, xx, c2, u0, l0);
    const float w_lab = __shfl(wnew_l, lab);
    if (live) zput(pt, c2, l0, u0, w_lab, (unsigned)lab);  // the direct bounds, or none
    move(live, pt, ao, lab, xr);
  }
  }  // DEFER
  CDR_TP(3);
  if (lane == 0) {
    a.fb_count[wave] = fb_used;
    a.mv_count[wave] = mv_used;
    if (a.q_acc) a.q_acc[wave] += qtot;
    if (B.t_acc) B.t_acc[wave] += ttot;
  }
  // this workgroup's moves into one run_sums slice (nothing to do: no atomics)
  if (__syncthreads_or(mv_used)) {
    const int cells = k * d1;
    unsigned long long* out = F.run_sums + (size_t)(blockIdx.x % kRunSlices) * cells;
    for (int e = t; e < cells; e += 256) {
      const unsigned long long v = mtab[e];
      if (v) atomicAdd(&out[e], v);
    }
  }
#ifdef CDR_EXPERIMENTS
  CDR_TP(4);
  if (B.tprof && lane == 0)
    for (int q = 0; q < 8; ++q) B.tprof[(size_t)wave * 8 + q] = tp[q];
#endif
#undef CDR_TP
}

// Bound words before the first bounded step of a run of them: every real
// point "no bound" with its current label (lab8), padding rows "always keep".
__global__ void zb_reset_kernel(const uint8_t* __restrict__ lab8, uint32_t* __restrict__ zb,
                                int64_t n, int64_t n_pad, const long long* __restrict__ gate) {
  if (gate && gate[0] == 0) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad;
       i += (int64_t)gridDim.x * blockDim.x)
    zb[i] = i < n ? (kZbStale | lab8[i]) : 0x7F000000u;  // (2^127: above any W)
}

// 2-byte words before the first bounded step: every real point "no bound"
// (code 0) with its current label, padding rows "always keep" (code 1023).
__global__ void zh_reset_kernel(const uint8_t* __restrict__ lab8, uint16_t* __restrict__ zh,
                                int64_t n, int64_t n_pad, const long long* __restrict__ gate) {
  if (gate && gate[0] == 0) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad;
       i += (int64_t)gridDim.x * blockDim.x)
    zh[i] = i < n ? (uint16_t)lab8[i] : (uint16_t)kZ16Pad;
}

// A rebase of the 2-byte words (plan32.h; decided by ll_finalize32, run
// before the next screen at the steps the host allows, gated on the device):
// every kept word to the new base and exponent, 8 words per thread
// (dec(code) - dG rounded down, truncated; codes 0 and 1023 stay).
__global__ __launch_bounds__(256) void zh_rebase_kernel(uint16_t* __restrict__ zh, int64_t n_pad,
                                                        const unsigned char* __restrict__ bt,
                                                        const long long* __restrict__ gate) {
  if (gate && gate[0] == 0) return;
  const int* hd = reinterpret_cast<const int*>(bt + kBndHdr);
  if (hd[3] == 0) return;
  __shared__ float dgs[64];
  if (threadIdx.x < 64) dgs[threadIdx.x] = reinterpret_cast<const float*>(bt + kBndDG)[threadIdx.x];
  __syncthreads();
  const int e0o = hd[1], e0n = hd[2];
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  u4v* z4 = reinterpret_cast<u4v*>(zh);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad / 8;
       i += (int64_t)gridDim.x * blockDim.x) {
    u4v z = __builtin_nontemporal_load(z4 + i);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned lo = z[q] & 0xFFFFu, hi = z[q] >> 16;
      z[q] = zb16_rebase(lo, dgs[lo & 63u], e0o, e0n) | zb16_rebase(hi, dgs[hi & 63u], e0o, e0n) << 16;
    }
    __builtin_nontemporal_store(z, z4 + i);
  }
}

void zh_rebase(Ctx& c, const long long* gate) {
  if (!c.zb_valid || c.zb_fmt != 16 || !c.bnd_ok) return;  // (no words to carry)
  hipLaunchKernelGGL(zh_rebase_kernel, dim3(2048), dim3(256), 0, c.stream, c.zb.as<uint16_t>(),
                     c.n_pad, reinterpret_cast<const unsigned char*>(c.bnd.p), gate);
  HIP_CHECK(hipGetLastError());
}

// The hi-only screen copy row by row (XH: screen32b's gathers read one line
// per point), from the tiled copy: tile of 32 points [2 halves][32][kPB].
template <int kPB>
__global__ void aos_hi_kernel(const unsigned char* __restrict__ xs, int64_t n_pad,
                              unsigned char* __restrict__ xh) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_pad * 2;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pt = t >> 1;
    const int hh = (int)(t & 1);
    const unsigned char* s = xs + (pt >> 5) * (64 * kPB) + hh * (32 * kPB) + (pt & 31) * kPB;
    unsigned char* d = xh + pt * (2 * kPB) + hh * kPB;
    if constexpr (kPB == 16) *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
    else *reinterpret_cast<uint2*>(d) = *reinterpret_cast<const uint2*>(s);
  }
}
// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct Plan32 {
  int QH, MT;
  float thr0, thr_rel;
  float Dv = 0.0f;  // the offset D (device plan: in the plan buffer)
  std::vector<h8> frag;      // [MT][2][64]
  std::vector<float> cinit;  // [MT][16][64]
  std::vector<float> prune;  // the prune block (plan32.h: c32 | E | h)
};

extern int lloyd_num_cus(int device);

// dst[i] = src[i] for 16-byte words; src is mapped pinned host memory.
__global__ __launch_bounds__(256) void pull_host_kernel(const uint4* __restrict__ src,
                                                        uint4* __restrict__ dst, int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) dst[i] = src[i];
}

// Shapes and data this kernel covers: F32X points, d <= 16, k <= 64, and every
// per-workgroup fp64 sum exact: |x| 2^S < 2^30 (F32X) and a workgroup sees at
// most ceil(groups / nwg) * 64 points, so its sums stay below 2^53 grid units
// when that count is < 2^23.  nwg >= #CUs (screen32_step).
bool screen32_supported(const Ctx& c, int k) {
  if (c.mode != CDR_MODE_F32X || c.d > 16 || k > 64 || k < 1) return false;
  if (exp_env("CDR_NO_SCREEN32")) return false;
  const int64_t groups = c.n_pad / 64;
  const int64_t per_wg = ceil_div(groups, lloyd_num_cus(c.device)) * 64;
  return per_wg < (int64_t(1) << 23);
}

// Point side of the bound: |xhat_f| <= max(fmax - mu, mu - fmin) 2^sigma.
void plan32_point_side(const Ctx& c, double& xxmax, double& l1x) {
  const double sc = std::ldexp(1.0, c.sigma);
  xxmax = 0.0;
  l1x = 0.0;
  for (int f = 0; f < c.d; ++f) {
    // (also bounds |fp16(xhat_f)|: the hi-only screen treats h as the point)
    const double dev =
        std::fmax(c.fmax[f] - (double)c.mu[f], (double)c.mu[f] - c.fmin[f]) * sc *
            (1.0 + std::ldexp(1.0, -11)) + std::ldexp(1.0, -25);
    xxmax += dev * dev;
    l1x += dev;
  }
  xxmax *= 1.0 + 1e-6;
}

// Fragments, C operand and certification constants.
static bool build_plan32(const Ctx& c, const double* C, int k, Plan32& pl) {
  const int d = c.d;
  const int Q = d4_of(d) / 4;
  pl.QH = Q <= 2 ? 1 : 2;
  pl.MT = k <= 32 ? 1 : 2;
  const double sc = std::ldexp(1.0, c.sigma);
  std::vector<double> ch((size_t)k * d), cc(k, 0.0);
  double ccmax = 0.0, l1c = 0.0, cabs = 0.0;
  for (int j = 0; j < k; ++j) {
    double s = 0.0, l1 = 0.0;
    for (int f = 0; f < d; ++f) {
      const double v = (C[(size_t)j * d + f] - (double)c.mu[f]) * sc;
      ch[(size_t)j * d + f] = v;
      s += v * v;
      l1 += std::fabs(v);
      cabs = std::fmax(cabs, std::fabs(v));
    }
    cc[j] = s;
    ccmax = std::fmax(ccmax, s);
    l1c = std::fmax(l1c, l1);
  }
  if (!(cabs <= 1024.0)) return false;  // fp16 split range (and NaN) guard
  double xxmax, l1x, D;
  plan32_point_side(c, xxmax, l1x);
  plan32_bounds(ccmax, l1c, xxmax, l1x, pl.QH, D, pl.thr0);
  pl.Dv = (float)D;
  pl.thr_rel = 1.0f + std::ldexp(1.0f, -16);  // the 64-ulp key truncation (2^-18 rel.)
  const int MT = pl.MT;
  pl.frag.assign((size_t)MT * 2 * 64, h8{});
  pl.cinit.assign((size_t)MT * 16 * 64, 0.0f);
  for (int m = 0; m < MT; ++m)
    for (int lane = 0; lane < 64; ++lane) {
      float cin[16];
      plan32_lane(ch.data(), cc.data(), D, k, d, pl.QH, m, lane, pl.frag[(m * 2 + 0) * 64 + lane],
                  pl.frag[(m * 2 + 1) * 64 + lane], cin);
      for (int i = 0; i < 16; ++i) pl.cinit[(m * 16 + i) * 64 + lane] = cin[i];
    }
  // prune block (screen32p), the quantities plan32_build computes on the device
  pl.prune.assign(kPrBytes / sizeof(float), 0.0f);
  float* pc = pl.prune.data();
  float* pE = pc + 64 * kPrStr;
  float* ph = pE + 64;
  std::vector<double> ec(64, 0.0);
  double ecmax = 0.0;
  const double dn = plan32_prune_dn(xxmax);
  for (int j = 0; j < 64; ++j) {
    double e2 = 0.0, n2 = 0.0;
    for (int f = 0; f < d && j < k; ++f) {
      const double v = (C[(size_t)j * d + f] - (double)c.mu[f]) * sc;
      const float cf = (float)v;
      pc[j * kPrStr + f] = cf;
      const double r = (double)cf - v;
      e2 += r * r;
      n2 += v * v;
    }
    ec[j] = plan32_prune_ec(e2, n2);
    pE[j] = plan32_prune_E(dn, ec[j]);
    if (j < k) ecmax = std::fmax(ecmax, ec[j]);
  }
  for (int r = 0; r < 64; ++r) {
    double sm = INFINITY;
    for (int j = 0; j < k && r < k; ++j) {
      if (j == r) continue;
      double s2 = 0.0;
      for (int f = 0; f < 16; ++f) {
        const double df = (double)pc[r * kPrStr + f] - (double)pc[j * kPrStr + f];
        s2 += df * df;
      }
      sm = std::fmin(sm, s2);
    }
    ph[r] = r < k ? plan32_prune_h(sm, ec[r], ecmax) : INFINITY;
  }
  return true;
}

// Device plan of the loop's centroids (c.ll_C) at begin / resume; later
// steps are planned by ll_finalize right after it moves the centroids.
__global__ __launch_bounds__(256) void plan32_kernel(const double* __restrict__ C, int k, int d,
                                                     int QH, int MT,
                                                     const double* __restrict__ mu, double sc,
                                                     double xxmax, double l1x,
                                                     long long* __restrict__ state,
                                                     unsigned char* __restrict__ plan) {
  if (state[0] == 0) return;
  plan32_build(C, k, d, QH, MT, mu, sc, xxmax, l1x, state, plan);
}

static int s32_blocks_per_cu(int QH, int MT, size_t lds) {
  int nb = 0;
  hipError_t e = hipErrorInvalidValue;
  if (QH == 1 && MT == 1) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, screen32<1, 1, true, false, false, true>, 256, lds);
  if (QH == 1 && MT == 2) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, screen32<1, 2, true, false, false, true>, 256, lds);
  if (QH == 2 && MT == 1) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, screen32<2, 1, true, false, false, true>, 256, lds);
  if (QH == 2 && MT == 2) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, screen32<2, 2, true, false, false, true>, 256, lds);
  if (e != hipSuccess || nb < 1) nb = 2;
  return nb > 8 ? 8 : nb;
}

// Device plan of the loop's current centroids (c.ll_C; mu as fp64 after the
// d reference values in c.ll_ref) into c.frag.
void plan32_launch(Ctx& c, int k, int QH, int MT) {
  hipLaunchKernelGGL(plan32_kernel, dim3(1), dim3(256), 0, c.stream, c.ll_C.as<double>(), k, c.d,
                     QH, MT, c.ll_ref.as<double>() + c.d, std::ldexp(1.0, c.sigma), c.ll_xxmax,
                     c.ll_l1x, c.ll_state.as<long long>(), static_cast<unsigned char*>(c.frag.p));
  HIP_CHECK(hipGetLastError());
}

// Build the exact pre-centred copy xt = (x - mu) 2^sigma once per point set
// (Ctx::pre_ok) and the int64 mu 2^S that restores x sums from xt sums.
void ensure_precentered(Ctx& c) {
  if (!c.pre_ok || c.xt_valid) return;
  const int d = c.d;
  c.xt32.ensure(sizeof(float) * (size_t)d4_of(d) * c.n_pad);
  hipLaunchKernelGGL(precenter_kernel, dim3(4096), dim3(256), 0, c.stream, c.x32.as<float>(),
                     c.n, c.n_pad, d, c.mu_s.as<float>(), (float)std::ldexp(1.0, c.sigma),
                     c.xt32.as<float>());
  HIP_CHECK(hipGetLastError());
  std::vector<long long> muf(d);
  for (int f = 0; f < d; ++f) muf[f] = std::llrint(std::ldexp((double)c.mu[f], c.scale_bits));
  c.muf.ensure(sizeof(long long) * d);
  HIP_CHECK(hipMemcpyAsync(c.muf.p, muf.data(), sizeof(long long) * d, hipMemcpyHostToDevice,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));  // muf is a stack vector
  c.xt_valid = true;
}

// One F32X Lloyd step through screen32; returns false (nothing launched) when
// the centroids are out of the fp16 split range.
// Row-major copy of the points (d4 floats per point): fixup32's gathers touch
// one line (and one page) per point instead of one per feature quad.
__global__ void aos_copy_kernel(const float4* __restrict__ x, int64_t n_pad, int Q,
                                float4* __restrict__ xa) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_pad * Q;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / Q;
    const int q = (int)(t - i * Q);
    xa[t] = x[(int64_t)q * n_pad + i];
  }
}

// Split screen copy and row-major copy (screen32d / fixup32), built once per
// point set.
// The row-major copy alone (also the large-k path's gathers, screen_big.hip).
void ensure_rowmajor(Ctx& c) {
  if (c.xa_valid) return;
  const int Q = d4_of(c.d) / 4;
  c.xa32.ensure(sizeof(float) * (size_t)c.n_pad * 4 * Q);
  hipLaunchKernelGGL(aos_copy_kernel, dim3(4096), dim3(256), 0, c.stream, c.x32.as<float4>(),
                     c.n_pad, Q, c.xa32.as<float4>());
  HIP_CHECK(hipGetLastError());
  c.xa_valid = true;
}

// QH = 1, 2: the hi / lo split copy; 3: the hi-only copy of d > 8, 4: of d <= 8 (HO)
static void ensure_split(Ctx& c, int QH) {
  if (c.xs_valid && c.xs_qh == QH) return;
  ensure_rowmajor(c);
  c.xs16.ensure((size_t)c.n_pad * (QH == 4 ? 16 : QH == 3 ? 32 : 32 * QH));
  const float sig = (float)std::ldexp(1.0, c.sigma);
  if (QH == 4)
    hipLaunchKernelGGL((split_copy_kernel<1, true>), dim3(4096), dim3(256), 0, c.stream,
                       c.x32.as<float>(), c.n, c.n_pad, c.d, c.mu_s.as<float>(), sig,
                       c.xs16.as<uint4>());
  else if (QH == 3)
    hipLaunchKernelGGL((split_copy_kernel<2, true>), dim3(4096), dim3(256), 0, c.stream,
                       c.x32.as<float>(), c.n, c.n_pad, c.d, c.mu_s.as<float>(), sig,
                       c.xs16.as<uint4>());
  else if (QH == 1)
    hipLaunchKernelGGL(split_copy_kernel<1>, dim3(4096), dim3(256), 0, c.stream, c.x32.as<float>(),
                       c.n, c.n_pad, c.d, c.mu_s.as<float>(), sig, c.xs16.as<uint4>());
  else
    hipLaunchKernelGGL(split_copy_kernel<2>, dim3(4096), dim3(256), 0, c.stream, c.x32.as<float>(),
                       c.n, c.n_pad, c.d, c.mu_s.as<float>(), sig, c.xs16.as<uint4>());
  HIP_CHECK(hipGetLastError());
  c.xs_valid = true;
  c.xs_qh = QH;
}

template <int QH, int MT, int PD, bool HO = false, bool LR = false>
static int s32d_blocks_per_cu() {
  static int nb = 0;
  if (!nb) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, screen32d<QH, MT, PD, HO, LR>, 256, 0) != hipSuccess ||
        nb < 1)
      nb = 2;
    if (nb > 8) nb = 8;
  }
  return nb;
}

#define CDR_S32P_ALL(X) X(1, 1, 3) X(1, 2, 3) X(2, 1, 3) X(2, 2, 3) \
                        X(3, 1, 3) X(3, 2, 3) X(4, 1, 3) X(4, 2, 3)

// (Q: feature quads; PD: 3 groups in flight)
static int screen32p_blocks_per_cu(int Q, int MT, int PD) {
  static int cache[4][2] = {};
  int& nb = cache[Q - 1][MT - 1];
  if (!nb) {
    hipError_t e = hipErrorInvalidValue;
#define CDR_S32P_OCC(Q_, M_, P_) \
    if (Q == Q_ && MT == M_ && PD == P_) \
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, screen32p<Q_, M_, P_>, 256, 0);
    CDR_S32P_ALL(CDR_S32P_OCC)
#undef CDR_S32P_OCC
    if (e != hipSuccess || nb < 1) nb = 2;
    if (nb > 8) nb = 8;
  }
  return nb;
}

static void screen32p_launch(int Q, int MT, int PD, dim3 grid, hipStream_t s,
                             const S32PArgs& p) {
#define CDR_S32P_GO(Q_, M_, P_) \
  if (Q == Q_ && MT == M_ && PD == P_) \
    hipLaunchKernelGGL((screen32p<Q_, M_, P_>), grid, dim3(256), 0, s, p);
  CDR_S32P_ALL(CDR_S32P_GO)
#undef CDR_S32P_GO
}

#define CDR_S32B_ALL(X) X(1, 1) X(1, 2) X(2, 1) X(2, 2) X(3, 1) X(3, 2) X(4, 1) X(4, 2)

static int screen32b_blocks_per_cu(int Q, int MT) {
  static int cache[4][2] = {};
  int& nb = cache[Q - 1][MT - 1];
  if (!nb) {
    hipError_t e = hipErrorInvalidValue;
#define CDR_S32B_OCC(Q_, M_) \
    if (Q == Q_ && MT == M_) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, screen32b<Q_, M_>, 256, 0);
    CDR_S32B_ALL(CDR_S32B_OCC)
#undef CDR_S32B_OCC
    if (e != hipSuccess || nb < 1) nb = 2;
    if (nb > 8) nb = 8;
  }
  return nb;
}

static void screen32b_launch(int Q, int MT, dim3 grid, hipStream_t s, const S32BArgs& p) {
#define CDR_S32B_GO(Q_, M_) \
  if (Q == Q_ && MT == M_) hipLaunchKernelGGL((screen32b<Q_, M_>), grid, dim3(256), 0, s, p);
  CDR_S32B_ALL(CDR_S32B_GO)
#undef CDR_S32B_GO
}

static int screen32bs_blocks_per_cu(int Q, int MT) {
  static int cache[4][2] = {};
  int& nb = cache[Q - 1][MT - 1];
  if (!nb) {
    hipError_t e = hipErrorInvalidValue;
#define CDR_S32BS_OCC(Q_, M_) \
    if (Q == Q_ && MT == M_) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, screen32bs<Q_, M_>, 256, 0);
    CDR_S32B_ALL(CDR_S32BS_OCC)
#undef CDR_S32BS_OCC
    if (e != hipSuccess || nb < 1) nb = 2;
    if (nb > 8) nb = 8;
  }
  return nb;
}

static void screen32bs_launch(int Q, int MT, dim3 grid, hipStream_t s, const S32BArgs& p,
                              bool split) {
#define CDR_S32BS_GO(Q_, M_)                                                                  \
  if (Q == Q_ && MT == M_) {                                                                  \
    if (split) hipLaunchKernelGGL((screen32bs<Q_, M_, true>), grid, dim3(256), 0, s, p);      \
    else hipLaunchKernelGGL((screen32bs<Q_, M_>), grid, dim3(256), 0, s, p);                  \
  }
  CDR_S32B_ALL(CDR_S32BS_GO)
#undef CDR_S32BS_GO
}

// chunks in flight per wave of screen32bz (CDR_S32BZ_PD = 4 | 8 | 12)
static void screen32bz_launch(dim3 grid, hipStream_t s, const S32BArgs& p) {
  static const int pd = exp_env("CDR_S32BZ_PD") ? std::atoi(exp_env("CDR_S32BZ_PD")) : 8;
  if (pd == 4) hipLaunchKernelGGL(screen32bz<4>, grid, dim3(256), 0, s, p);
  else if (pd == 12) hipLaunchKernelGGL(screen32bz<12>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(screen32bz<8>, grid, dim3(256), 0, s, p);
}

// Prefetch depth of screen32d: CDR_S32D_PD=2|3|4 (comparisons), else the
// measured default per shape.
static int s32d_depth(int QH) {
  static const int env = exp_env("CDR_S32D_PD") ? std::atoi(exp_env("CDR_S32D_PD")) : 0;
  if (env >= 2 && env <= 4) return env;
  return QH == 1 ? 3 : 2;  // A/B at configs 2 and 3: 3 helps the d <= 8 screen (0.108 -> 0.102 ms), not d = 16
}

// A DELTA step on screen32d + fixup32 (labels and running sums as screen32's).
static void screen32d_step(Ctx& c, int QH, int MT, int k, const h8* dfrag, const float* dcinit,
                           const double* dcent, float thr0, float thr_rel, float Dv,
                           const float* dthr, long long* dout, long long* hout, bool prof,
                           long long* gate) {
  // d > 8: the hi-only screen (half the bytes; CDR_S32D_HO=0: the split copy)
  static const bool ho_env = !exp_env("CDR_S32D_HO") || std::atoi(exp_env("CDR_S32D_HO"));
  const bool HO = ho_env;
  // hi-only: LDS ring of CDR_S32H_LR slots per wave (2..4; 0: register prefetch);
  // A/B at config 3: 2 slots 0.90-0.91 ms, 3-4 slots 0.92-0.95, registers 0.93
  static const int lr_env = exp_env("CDR_S32H_LR") ? std::atoi(exp_env("CDR_S32H_LR")) : 2;
  const int LRn = HO && QH == 2 && lr_env >= 2 && lr_env <= 4 ? lr_env : 0;
  ensure_split(c, HO ? (QH == 2 ? 3 : 4) : QH);
  const int64_t groups = c.n_pad / 64;
  const int cus = lloyd_num_cus(c.device);
  // pruned screen (screen32p) on the hi-only copy: CDR_PRUNE=0 turns it off
  static const bool pr_env = !exp_env("CDR_PRUNE") || std::atoi(exp_env("CDR_PRUNE"));
  const bool PR = pr_env && HO && c.prune_on;
  const int PPD = 3;
  const int PQ = d4_of(c.d) / 4;
  // the fixup fused into screen32p's tail (CDR_PRUNE_FUSE=0: a separate fixup32)
  static const bool fuse_env =
      !exp_env("CDR_PRUNE_FUSE") || std::atoi(exp_env("CDR_PRUNE_FUSE"));
  // bounded screen (screen32b) in the device loop, where ll_finalize32 keeps
  // the drift bounds of every centroid move (CDR_BOUNDS=0 turns it off)
  const bool bnd_env = !std::getenv("CDR_BOUNDS") || std::atoi(std::getenv("CDR_BOUNDS"));
  const bool BND = PR && bnd_env && gate && dthr && c.ll_on && c.bnd_ok &&
                   c.n_pad < (int64_t(1) << 31);
  // the bounded screen deciding in registers (screen32bs; CDR_S32B_SPLIT=0:
  // screen32b with its queue and fused fixup)
  const bool BS = BND && (!std::getenv("CDR_S32B_SPLIT") || std::atoi(std::getenv("CDR_S32B_SPLIT")));
  if (!BND) c.zb_valid = false;  // another path decides this step's labels
  int bpc;
  const int PD = PR ? PPD : LRn ? LRn : s32d_depth(QH);
  if (BS) {
    bpc = screen32bs_blocks_per_cu(PQ, MT);
    // (experiments: fewer workgroups per CU, CDR_S32BS_BPC=1..3)
    static const int bsb_env = exp_env("CDR_S32BS_BPC") ? std::atoi(exp_env("CDR_S32BS_BPC")) : 0;
    if (bsb_env >= 1 && bsb_env < bpc) bpc = bsb_env;
  } else if (BND) {
    bpc = screen32b_blocks_per_cu(PQ, MT);
  } else if (PR) {
    bpc = screen32p_blocks_per_cu(PQ, MT, PPD);
    static const int bpc_env = exp_env("CDR_S32P_BPC") ? std::atoi(exp_env("CDR_S32P_BPC")) : 0;
    if (bpc_env >= 1 && bpc_env < bpc) bpc = bpc_env;
#ifndef CDR_EXPERIMENTS
  } else {
    // (the unpruned DELTA screens: CDR_PRUNE=0 / CDR_S32D_HO=0, experiments build)
    CDR_FAIL(CDR_ERR_STATE, "screen32d: the unpruned DELTA screens are in the experiments build");
  }
#else
  } else if (LRn) {
    if (PD == 2) bpc = MT == 1 ? s32d_blocks_per_cu<2, 1, 2, true, true>() : s32d_blocks_per_cu<2, 2, 2, true, true>();
    else if (PD == 3) bpc = MT == 1 ? s32d_blocks_per_cu<2, 1, 3, true, true>() : s32d_blocks_per_cu<2, 2, 3, true, true>();
    else bpc = MT == 1 ? s32d_blocks_per_cu<2, 1, 4, true, true>() : s32d_blocks_per_cu<2, 2, 4, true, true>();
  } else if (HO && QH == 1) {
    if (PD == 2) bpc = MT == 1 ? s32d_blocks_per_cu<1, 1, 2, true>() : s32d_blocks_per_cu<1, 2, 2, true>();
    else if (PD == 3) bpc = MT == 1 ? s32d_blocks_per_cu<1, 1, 3, true>() : s32d_blocks_per_cu<1, 2, 3, true>();
    else bpc = MT == 1 ? s32d_blocks_per_cu<1, 1, 4, true>() : s32d_blocks_per_cu<1, 2, 4, true>();
  } else if (HO) {
    if (PD == 2) bpc = MT == 1 ? s32d_blocks_per_cu<2, 1, 2, true>() : s32d_blocks_per_cu<2, 2, 2, true>();
    else if (PD == 3) bpc = MT == 1 ? s32d_blocks_per_cu<2, 1, 3, true>() : s32d_blocks_per_cu<2, 2, 3, true>();
    else bpc = MT == 1 ? s32d_blocks_per_cu<2, 1, 4, true>() : s32d_blocks_per_cu<2, 2, 4, true>();
  } else if (PD == 4) {
    if (QH == 1 && MT == 1) bpc = s32d_blocks_per_cu<1, 1, 4>();
    else if (QH == 1) bpc = s32d_blocks_per_cu<1, 2, 4>();
    else if (MT == 1) bpc = s32d_blocks_per_cu<2, 1, 4>();
    else bpc = s32d_blocks_per_cu<2, 2, 4>();
  } else if (PD == 3) {
    if (QH == 1 && MT == 1) bpc = s32d_blocks_per_cu<1, 1, 3>();
    else if (QH == 1) bpc = s32d_blocks_per_cu<1, 2, 3>();
    else if (MT == 1) bpc = s32d_blocks_per_cu<2, 1, 3>();
    else bpc = s32d_blocks_per_cu<2, 2, 3>();
  } else {
    if (QH == 1 && MT == 1) bpc = s32d_blocks_per_cu<1, 1, 2>();
    else if (QH == 1) bpc = s32d_blocks_per_cu<1, 2, 2>();
    else if (MT == 1) bpc = s32d_blocks_per_cu<2, 1, 2>();
    else bpc = s32d_blocks_per_cu<2, 2, 2>();
  }
#endif
  // (screen32b: a wave's unit is a chunk of kBChunk points, not a 64-point group)
  const int64_t units = BND ? c.n_pad / kBChunk : groups;
  const int unit_pts = BND ? kBChunk : 64;
  int nwg = (int)std::min<int64_t>(ceil_div(units, 4), (int64_t)cus * bpc);
  if (nwg < 1) nwg = 1;
  const int nwaves = nwg * 4;
  const int cap = (int)(ceil_div(units, nwaves) * unit_pts);
  c.fb_list.ensure(sizeof(int2) * (size_t)nwaves * cap);
  if (!BS) c.mv_list.ensure(sizeof(int2) * (size_t)nwaves * cap);  // (screen32bs: no move list)
  c.mv_count.ensure(sizeof(int32_t) * (size_t)nwaves);
  if (c.fb_count.bytes < sizeof(int32_t) * (nwaves + 3) || c.fb_layout != nwaves) {
    c.fb_count.ensure(sizeof(int32_t) * (nwaves + 3));
    HIP_CHECK(hipMemsetAsync(c.fb_count.p, 0, sizeof(int32_t) * (nwaves + 3), c.stream));
    c.fb_layout = nwaves;
  }
  c.fb_regions = nwaves;
  c.fb_total_slot = nwaves + 1;
  if (!c.lab8_valid) {  // first DELTA step since another path wrote the labels
    c.lab8.ensure((size_t)c.n_pad);
    hipLaunchKernelGGL(lab8_kernel, dim3(2048), dim3(256), 0, c.stream, c.labels.as<int32_t>(),
                       c.lab8.as<uint8_t>(), c.n_pad);
    HIP_CHECK(hipGetLastError());
    c.lab8_valid = true;
  }
  S32DArgs a;
  a.XS = c.xs16.as<unsigned char>();
  a.n = c.n;
  a.n_pad = c.n_pad;
  a.frag = dfrag;
  a.cinit = dcinit;
  a.thr0 = thr0;
  a.thr_rel = thr_rel;
  a.Dv = Dv;
  a.thr_dev = dthr;
  a.gate = gate;
  a.labels = c.labels.as<int32_t>();
  a.lab8 = c.lab8.as<uint8_t>();
  a.fb_list = c.fb_list.as<int2>();
  a.fb_count = c.fb_count.as<int32_t>();
  a.mv_list = c.mv_list.as<int2>();
  a.mv_count = c.mv_count.as<int32_t>();
  a.cap = cap;
  FixArgs f;
  f.XA = c.xa32.as<float>();
  f.n_pad = c.n_pad;
  f.cent = dcent;
  f.k = k;
  f.d = c.d;
  f.labels = c.labels.as<int32_t>();
  f.lab8 = c.lab8.as<uint8_t>();
  f.fb_list = c.fb_list.as<int2>();
  f.fb_count = c.fb_count.as<int32_t>();
  f.mv_list = c.mv_list.as<int2>();
  f.mv_count = c.mv_count.as<int32_t>();
  f.cap = cap;
  f.regions = nwaves;
  f.fx = std::ldexp(1.0, c.scale_bits);
  f.run_sums = c.run_sums.as<unsigned long long>();
  f.gate = gate;
  f.abl = 0;
  f.XS = c.xs16.as<unsigned char>();
  f.frag = dfrag;
  f.cinit = dcinit;
  f.thr0 = thr0;
  f.thr_rel = thr_rel;
  f.thr_dev = dthr;
  f.ho = HO;
  f.ms = c.mu_s.as<float>();
  f.sig = (float)std::ldexp(1.0, c.sigma);
  f.zb = nullptr;
#ifdef CDR_EXPERIMENTS
  if (const char* e = exp_env("CDR_FIX_ABL")) f.abl = std::atoi(e);
#endif
  const dim3 grid(nwg), blk(256);
  const bool fused = PR && fuse_env;
  if (PR) {
    S32PArgs p;
    p.XS = a.XS;
    p.n = c.n;
    p.n_pad = c.n_pad;
    p.k = k;
    p.d = c.d;
    p.prune = reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(dfrag) +
                                             plan32_layout(MT, k, c.d).prune);
    p.gate = gate;
    p.labels = a.labels;
    p.lab8 = a.lab8;
    p.fb_list = a.fb_list;
    p.fb_count = a.fb_count;
    p.mv_list = a.mv_list;
    p.mv_count = a.mv_count;
    p.cap = cap;
    p.frag = dfrag;
    p.cinit = dcinit;
    p.thr0 = thr0;
    p.thr_rel = thr_rel;
    p.Dv = Dv;
    p.thr_dev = dthr;
    if (c.prof_on && c.q_acc.bytes < sizeof(long long) * nwaves) {  // (zeroed when grown)
      c.q_acc.ensure(sizeof(long long) * nwaves);
      HIP_CHECK(hipMemsetAsync(c.q_acc.p, 0, c.q_acc.bytes, c.stream));
    }
    p.q_acc = c.prof_on ? c.q_acc.as<long long>() : nullptr;
    p.abl = 0;
#ifdef CDR_EXPERIMENTS
    if (const char* e = exp_env("CDR_S32P_ABL")) p.abl = std::atoi(e);
#endif
    p.fx = f;
    p.fx.fr = 4;
    p.fuse = fused ? 1 : 0;
    if (BND) {
      // bound words: reset (every point "no bound", labels from lab8) at the
      // first bounded step of a run; the row-major hi copy once per point set
      // the fused screen32bs keeps 2-byte words; the split
      // form (CDR_S32BS_SPLIT=1) and screen32b 4-byte ones
      const bool split_env =
          BS && std::getenv("CDR_S32BS_SPLIT") && std::atoi(std::getenv("CDR_S32BS_SPLIT"));
      const bool z16 = BS && !split_env;
      const int zfmt = z16 ? 16 : 32;
      if (c.zb_fmt != zfmt) c.zb_valid = false;
      c.zb_fmt = zfmt;
      c.zb.ensure(sizeof(uint32_t) * (size_t)c.n_pad);
      if (!c.zb_valid) {
        if (z16)
          hipLaunchKernelGGL(zh_reset_kernel, dim3(2048), dim3(256), 0, c.stream,
                             c.lab8.as<uint8_t>(), c.zb.as<uint16_t>(), c.n, c.n_pad, gate);
        else
          hipLaunchKernelGGL(zb_reset_kernel, dim3(2048), dim3(256), 0, c.stream,
                             c.lab8.as<uint8_t>(), c.zb.as<uint32_t>(), c.n, c.n_pad, gate);
        HIP_CHECK(hipGetLastError());
      }
      if (!BS && !c.xh_valid) {
        c.xh16.ensure((size_t)c.n_pad * (QH == 1 ? 16 : 32));
        if (QH == 1)
          hipLaunchKernelGGL(aos_hi_kernel<8>, dim3(4096), dim3(256), 0, c.stream,
                             c.xs16.as<unsigned char>(), c.n_pad, c.xh16.as<unsigned char>());
        else
          hipLaunchKernelGGL(aos_hi_kernel<16>, dim3(4096), dim3(256), 0, c.stream,
                             c.xs16.as<unsigned char>(), c.n_pad, c.xh16.as<unsigned char>());
        HIP_CHECK(hipGetLastError());
        c.xh_valid = true;
      }
      if (c.prof_on && c.t_acc.bytes < sizeof(long long) * nwaves) {  // (zeroed when grown)
        c.t_acc.ensure(sizeof(long long) * nwaves);
        HIP_CHECK(hipMemsetAsync(c.t_acc.p, 0, c.t_acc.bytes, c.stream));
      }
      S32BArgs b;
      f.zb = c.zb.as<uint32_t>();  // (the separate fixup32, CDR_PRUNE_FUSE=0)
      b.p = p;
      b.p.fx.zb = c.zb.as<uint32_t>();
      b.XH = c.xh16.as<unsigned char>();
      b.zb = c.zb.as<uint32_t>();
      b.wup = reinterpret_cast<const float*>(c.bnd.as<long long>() + 64);
      b.wdn = b.wup + 64;
      b.nchunks = c.n_pad / (z16 ? kZ16Chunk : kBChunk);
      b.zh = z16 ? c.zb.as<uint16_t>() : nullptr;
      b.bt = reinterpret_cast<const unsigned char*>(c.bnd.p);
      b.t_acc = c.prof_on ? c.t_acc.as<long long>() : nullptr;
      b.dbg = exp_env("CDR_BOUNDS_DBG") ? std::atoi(exp_env("CDR_BOUNDS_DBG")) : 0;
#ifndef CDR_EXPERIMENTS
      b.dbg &= 1;  // (the other bits are timing experiments: experiments build only)
#endif
      c.zb_valid = true;
      b.tprof = nullptr;
      b.slot_wg = 0;
      // chunk shares of screen32bs's 4 launch generations (workgroups per CU):
      // one region per generation (4-byte words, A/B at 100M: 180 -> 166 us
      // against one strided split; speed-proportional weights 100,82,68,61
      // 166 us); 2-byte words: 115,105,95,85 (0.161-0.163 ms per step against
      // 0.168-0.178 equal, profiles/r05_generation_weights.txt);
      // CDR_S32BS_W="w0,w1,w2,w3" sets them, CDR_S32BS_W=0 the split
      if (BS) {
        static int wenv[4] = {-1, 0, 0, 0};
        if (wenv[0] < 0) {
          const int wdef[4] = {115, 105, 95, 85};
          for (int q = 0; q < 4; ++q) wenv[q] = split_env ? 100 : wdef[q];
          if (const char* e = exp_env("CDR_S32BS_W")) {
            wenv[0] = 0;
            int v[4] = {0, 0, 0, 0};
            if (std::sscanf(e, "%d,%d,%d,%d", &v[0], &v[1], &v[2], &v[3]) == 4 && v[0] > 0 &&
                v[1] > 0 && v[2] > 0 && v[3] > 0)
              for (int q = 0; q < 4; ++q) wenv[q] = v[q];
          }
        }
        if (wenv[0] > 0 && nwg == cus * bpc && bpc == 4) {
          b.slot_wg = cus;
          for (int q = 0; q < 4; ++q) b.wsl[q] = wenv[q];
        }
        // contiguous chunk ranges per wave (CDR_S32BS_CONTIG=1)
        if (exp_env("CDR_S32BS_CONTIG") && std::atoi(exp_env("CDR_S32BS_CONTIG")))
          b.slot_wg = -1;
      }
      // the dynamic tail (2-byte words in generation regions): CDR_S32BS_DYN
      // = the statically streamed percent (100: off)
      b.dyn = nullptr;
      b.dyn_par = 0;
      b.dyn_pct = 100;
      if (BS && z16 && !split_env && b.slot_wg > 0) {
        static int dyn_env = -1;
        if (dyn_env < 0) {
          dyn_env = kS32DynPct;
          if (const char* e = exp_env("CDR_S32BS_DYN")) dyn_env = std::atoi(e);
          dyn_env = std::min(std::max(dyn_env, 0), 100);
        }
        if (dyn_env < 100 && bs_max_region(b, nwg) < (1 << 17) && b.slot_wg % 8 == 0 &&
            bs_max_chunks(b, nwg) >= kS32DynMinChunks) {
          if (c.s32_dyn.bytes < sizeof(unsigned) * 2 * 32 * 32) {
            c.s32_dyn.ensure(sizeof(unsigned) * 2 * 32 * 32);
            HIP_CHECK(hipMemsetAsync(c.s32_dyn.p, 0, c.s32_dyn.bytes, c.stream));
          }
          b.dyn = c.s32_dyn.as<unsigned>();
          b.dyn_par = c.s32_dyn_par;
          b.dyn_pct = dyn_env;
          c.s32_dyn_par ^= 1;
        }
      }
#ifdef CDR_EXPERIMENTS
      static unsigned long long* tprof_buf = nullptr;
      const bool tprof_on = BS && exp_env("CDR_S32BS_TPROF");
      if (tprof_on) {
        if (!tprof_buf) HIP_CHECK(hipMalloc(&tprof_buf, sizeof(unsigned long long) * 8 * 65536));
        b.tprof = tprof_buf;
      }
#endif
      if (BS) {
        // split form (CDR_S32BS_SPLIT=1; default: the fused kernel): screen32bz
        // streams the words and lists the failed points, screen32bs<.., true>
        // decides the lists.  Measured at config 3 (profiles/r05_split_ab.txt):
        // the stream alone takes ~80 us and the decisions ~100-130 us as their
        // own launch, so the fused kernel (~165-180 us) stays the default
        // the near-tie list holds at most the points of a wave's chunks
        // (the dynamic tail: twice the static share plus the two groups a
        // claiming wave may hold, so the waves' budgets cover the pool)
        const int64_t need =
            (b.dyn ? 2 * bs_max_chunks(b, nwg) + 2 * kBPD + 1 : bs_max_chunks(b, nwg)) *
            (z16 ? kZ16Chunk : kBChunk);
        if (need > b.p.cap) {
          c.fb_list.ensure(sizeof(int2) * (size_t)nwaves * (size_t)need);
          b.p.fb_list = c.fb_list.as<int2>();
          b.p.cap = (int)need;
        }
        b.zl = nullptr;
        b.zn = nullptr;
        b.zcap = 0;
        if (split_env) {
          b.zcap = ceil_div(bs_max_chunks(b, nwg) * kBChunk, 64) * 64;
          c.zl.ensure(sizeof(uint32_t) * (size_t)nwaves * (size_t)b.zcap);
          c.zn.ensure(sizeof(int32_t) * (size_t)nwaves);
          b.zl = c.zl.as<uint32_t>();
          b.zn = c.zn.as<int32_t>();
        }
        snprintf(c.prof_kernel, sizeof(c.prof_kernel),
                 split_env ? "screen32bs<%d,%d>split" : "screen32bs16<%d,%d>", PQ, MT);
        if (prof) prof_mark(c, 0);
        if (split_env) {
          screen32bz_launch(grid, c.stream, b);
          if (prof) prof_mark_sub(c);
        }
        screen32bs_launch(PQ, MT, grid, c.stream, b, split_env);
#ifdef CDR_EXPERIMENTS
        if (tprof_on) {  // per-wave phase times (100 MHz counter), to stderr
          std::vector<unsigned long long> h((size_t)nwaves * 8);
          HIP_CHECK(hipStreamSynchronize(c.stream));
          HIP_CHECK(hipMemcpy(h.data(), tprof_buf, h.size() * 8, hipMemcpyDeviceToHost));
          unsigned long long t0 = ~0ull, t4 = 0;
          double sum[6] = {}, mx[6] = {}, mv = 0, nb = 0, mvt = 0;
          for (int w = 0; w < nwaves; ++w) {
            const unsigned long long* r = &h[(size_t)w * 8];
            t0 = std::min(t0, r[0]);
            t4 = std::max(t4, r[4]);
          }
          for (int w = 0; w < nwaves; ++w) {
            const unsigned long long* r = &h[(size_t)w * 8];
            const double v[6] = {double(r[0] - t0), double(r[1] - r[0]), double(r[2] - r[1]),
                                 double(r[3] - r[2]), double(r[4] - r[3]), double(t4 - r[4])};
            for (int q = 0; q < 6; ++q) {
              sum[q] += v[q];
              mx[q] = std::max(mx[q], v[q]);
            }
            mvt += double(r[5]);
            nb += double(r[6]);
            mv += double(r[7]);
          }
          if (const char* path = exp_env("CDR_S32BS_TPROF_FILE")) {  // raw, appended
            if (FILE* fo = std::fopen(path, "ab")) {
              std::fwrite(h.data(), 8, h.size(), fo);
              std::fclose(fo);
            }
          }
          std::fprintf(stderr,
                       "TPROF waves %d span %.1f us | avg/max us: start %.1f/%.1f prologue %.1f/%.1f "
                       "phases %.1f/%.1f tail %.1f/%.1f flush %.1f/%.1f idle-end %.1f/%.1f | "
                       "| (split form: tail batches/wave, moves/wave, move us/wave; fused: batches/wave, "
                       "row-wait us/wave, decide us/wave) %.2f %.1f %.2f\n",
                       nwaves, (t4 - t0) / 100.0, sum[0] / nwaves / 100, mx[0] / 100,
                       sum[1] / nwaves / 100, mx[1] / 100, sum[2] / nwaves / 100, mx[2] / 100,
                       sum[3] / nwaves / 100, mx[3] / 100, sum[4] / nwaves / 100, mx[4] / 100,
                       sum[5] / nwaves / 100, mx[5] / 100, nb / nwaves, split_env ? mv / nwaves : mv / nwaves / 100,
                       mvt / nwaves / 100);
        }
#endif
      } else {
        snprintf(c.prof_kernel, sizeof(c.prof_kernel), "screen32b<%d,%d>%s", PQ, MT,
                 fused ? "+fixup" : "");
        if (prof) prof_mark(c, 0);
        screen32b_launch(PQ, MT, grid, c.stream, b);
      }
    } else {
    snprintf(c.prof_kernel, sizeof(c.prof_kernel), "screen32p<%d,%d,%d>%s", PQ, MT, PPD,
             fused ? "+fixup" : "");
    if (prof) prof_mark(c, 0);
    screen32p_launch(PQ, MT, PPD, grid, c.stream, p);
    }
  } else {
#ifdef CDR_EXPERIMENTS
  if (LRn)
    snprintf(c.prof_kernel, sizeof(c.prof_kernel), "screen32h<%d,%d>lds", MT, PD);
  else if (HO)
    snprintf(c.prof_kernel, sizeof(c.prof_kernel), QH == 1 ? "screen32h1<%d,%d>" : "screen32h<%d,%d>",
             MT, PD);
  else
    snprintf(c.prof_kernel, sizeof(c.prof_kernel), "screen32d<%d,%d,%d>", QH, MT, PD);
  if (prof) prof_mark(c, 0);
#define CDR_S32D_LAUNCH(P)                                                                  \
  if (LRn && MT == 1) hipLaunchKernelGGL((screen32d<2, 1, P, true, true>), grid, blk, 0, c.stream, a); \
  else if (LRn) hipLaunchKernelGGL((screen32d<2, 2, P, true, true>), grid, blk, 0, c.stream, a);       \
  else if (HO && QH == 1 && MT == 1) hipLaunchKernelGGL((screen32d<1, 1, P, true>), grid, blk, 0, c.stream, a); \
  else if (HO && QH == 1) hipLaunchKernelGGL((screen32d<1, 2, P, true>), grid, blk, 0, c.stream, a); \
  else if (HO && MT == 1) hipLaunchKernelGGL((screen32d<2, 1, P, true>), grid, blk, 0, c.stream, a); \
  else if (HO) hipLaunchKernelGGL((screen32d<2, 2, P, true>), grid, blk, 0, c.stream, a);      \
  else if (QH == 1 && MT == 1) hipLaunchKernelGGL((screen32d<1, 1, P>), grid, blk, 0, c.stream, a); \
  else if (QH == 1) hipLaunchKernelGGL((screen32d<1, 2, P>), grid, blk, 0, c.stream, a);       \
  else if (MT == 1) hipLaunchKernelGGL((screen32d<2, 1, P>), grid, blk, 0, c.stream, a);       \
  else hipLaunchKernelGGL((screen32d<2, 2, P>), grid, blk, 0, c.stream, a);
  if (PD == 4) {
    CDR_S32D_LAUNCH(4)
  } else if (PD == 3) {
    CDR_S32D_LAUNCH(3)
  } else {
    CDR_S32D_LAUNCH(2)
  }
#undef CDR_S32D_LAUNCH
#endif
  }
  HIP_CHECK(hipGetLastError());
  if (prof) prof_mark(c, 1);
  // list regions per fixup workgroup: CDR_FIX_FR (1..16); A/B at config 3 (100M and
  // the 12.5M shard): 8 leaves 79-82 / 34 us beside the screen, 4 91-93 / 42, 16 106 / 39
  static const int fr_env = exp_env("CDR_FIX_FR") ? std::atoi(exp_env("CDR_FIX_FR")) : 8;
  f.fr = fr_env >= 1 && fr_env <= kFixMaxR ? fr_env : 8;
  const dim3 fgrid((nwaves + f.fr - 1) / f.fr);
#ifdef CDR_EXPERIMENTS
  if (!fused && !BS) switch (d4_of(c.d) / 4) {  // (screen32bs applies its own moves)
#define CDR_FIX(Q_)                                                                  \
  case Q_:                                                                           \
    if (MT == 1) hipLaunchKernelGGL((fixup32<Q_, 1>), fgrid, blk, 0, c.stream, f);    \
    else hipLaunchKernelGGL((fixup32<Q_, 2>), fgrid, blk, 0, c.stream, f);            \
    break;
    CDR_FIX(1) CDR_FIX(2) CDR_FIX(3) CDR_FIX(4)
#undef CDR_FIX
    default: CDR_FAIL(CDR_ERR_STATE, "screen32d: d > 16");
  }
#endif
  HIP_CHECK(hipGetLastError());
  const int len = k * (c.d + 1);
  long long* hout_dev = nullptr;
  if (hout) {
    void* hp = nullptr;
    HIP_CHECK(hipHostGetDevicePointer(&hp, hout, 0));
    hout_dev = static_cast<long long*>(hp);
  }
  c.fb_accum.ensure(2 * sizeof(long long));
  if (dout || hout_dev || !gate) {
    hipLaunchKernelGGL(publish32, dim3((unsigned)std::max(1, (len + 255) / 256)), dim3(256), 0,
                       c.stream, c.run_sums.as<long long>(),
                       len, dout, hout_dev, gate ? nullptr : c.fb_count.as<int32_t>(), nwaves,
                       c.prof_on ? c.fb_accum.as<long long>() : nullptr, gate);
    HIP_CHECK(hipGetLastError());
  }
}

// One F32X Lloyd step through screen32.  C != null: host plan (built here,
// uploaded with the step); returns false (nothing launched) when the
// centroids are out of the fp16 split range.  C == null: device-resident loop
// (loop.hip) — plan32_kernel builds the plan from c.ll_C on the device and
// every kernel of the step runs only while gate[0] != 0.
bool screen32_step(Ctx& c, const double* C, int k, long long* dout, long long* hout, bool prof,
                   float* dbg, float* thr_out, long long* gate) {
  const bool devplan = C == nullptr;
  Plan32 pl;
  if (devplan) {
    const int Q4 = d4_of(c.d) / 4;
    pl.QH = Q4 <= 2 ? 1 : 2;
    pl.MT = k <= 32 ? 1 : 2;
    pl.thr0 = 0.0f;
    pl.thr_rel = 1.0f + std::ldexp(1.0f, -16);
  } else if (!build_plan32(c, C, k, pl)) {
    return false;
  }
  // incremental update when the device labels and running sums belong to the
  // previous step of this point set and k
  const bool delta = c.run_valid && c.run_k == k && !dbg && !std::getenv("CDR_NO_DELTA");
  const int len = k * (c.d + 1);
  c.run_sums.ensure(sizeof(long long) * len * kRunSlices);
  if (!delta) {
    if (gate) {
      hipLaunchKernelGGL(zero_gated, dim3(4), dim3(256), 0, c.stream, c.run_sums.as<long long>(),
                         len * kRunSlices, gate);
      HIP_CHECK(hipGetLastError());
    } else {
      HIP_CHECK(hipMemsetAsync(c.run_sums.p, 0, sizeof(long long) * len * kRunSlices, c.stream));
    }
  }
  c.run_valid = false;
  c.big_valid = false;  // screen32 writes the labels the large-k running sums follow
  c.last_delta = delta;
  if (thr_out) {
    thr_out[0] = pl.thr0;
    thr_out[1] = 0.0f;
  }
  const int d = c.d, Q = d4_of(d) / 4;
  const int KP = 32 * pl.MT, NF = 8 * pl.QH;
  // plan buffer: fragments | C operand | centroids (fp64, for the fused
  // exact fallback) | thr0 (device plan only)
  const Plan32Layout PL = plan32_layout(pl.MT, k, c.d);
  const size_t b_frag = PL.cinit;
  const size_t b_cinit = PL.cent - PL.cinit;
  const size_t b_cent = PL.thr - PL.cent;
  const size_t b_all = PL.thr;
  c.frag.ensure(PL.all);
  if (!devplan) {  // (device plan: built by plan32_kernel / ll_finalize)
    // one pinned upload per step; the previous step's copy must have left the
    // staging buffer
    if (c.up_pending) HIP_CHECK(hipEventSynchronize(c.up_event));
    c.h_up.ensure(PL.all);
    memcpy(c.h_up.p, pl.frag.data(), b_frag);
    memcpy(static_cast<char*>(c.h_up.p) + b_frag, pl.cinit.data(), b_cinit);
    memcpy(static_cast<char*>(c.h_up.p) + b_frag + b_cinit, C, b_cent);
    memcpy(static_cast<char*>(c.h_up.p) + PL.prune, pl.prune.data(), kPrBytes);
    // the device pulls the staging buffer itself (pinned, mapped host memory)
    // with one small kernel on the stream: no DMA-engine copy in the step (a
    // runtime H2D copy here stalled the host for 7-16 ms once per run)
    void* hdev = nullptr;
    HIP_CHECK(hipHostGetDevicePointer(&hdev, c.h_up.p, 0));
    const int64_t n16 = (int64_t)(PL.all / 16);
    hipLaunchKernelGGL(pull_host_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0,
                       c.stream, static_cast<const uint4*>(hdev), static_cast<uint4*>(c.frag.p),
                       n16);
    HIP_CHECK(hipGetLastError());
    if (!c.up_event) HIP_CHECK(hipEventCreateWithFlags(&c.up_event, hipEventDisableTiming));
    HIP_CHECK(hipEventRecord(c.up_event, c.stream));
    c.up_pending = true;
  }
  h8* dfrag = c.frag.as<h8>();
  float* dcinit = reinterpret_cast<float*>(static_cast<char*>(c.frag.p) + b_frag);
  const double* dcent =
      reinterpret_cast<const double*>(static_cast<char*>(c.frag.p) + b_frag + b_cinit);
  const float* dthr =
      devplan ? reinterpret_cast<const float*>(static_cast<char*>(c.frag.p) + b_all) : nullptr;
  const bool lean = delta && !dbg && !exp_env("CDR_NO_LEAN");
  if (lean) {
    screen32d_step(c, pl.QH, pl.MT, k, dfrag, dcinit, dcent, pl.thr0, pl.thr_rel, pl.Dv, dthr,
                   dout, hout, prof, gate);
    c.run_valid = true;
    c.run_k = k;
    return true;
  }
  c.lab8_valid = false;  // the full screen writes the labels alone
  const size_t lds = (size_t)NF * KP * 8 + (size_t)KP * 4 + (size_t)k * 17 * 8;
  const int64_t groups = c.n_pad / 64;
  const int cus = lloyd_num_cus(c.device);
  const int bpc = s32_blocks_per_cu(pl.QH, pl.MT, lds);
  int nwg = (int)std::min<int64_t>(ceil_div(groups, 4), (int64_t)cus * bpc);
  if (nwg < 1) nwg = 1;
  const int nwaves = nwg * 4;
  const int cap = (int)(ceil_div(groups, nwaves) * 64);
  c.fb_list.ensure(sizeof(int32_t) * (size_t)nwaves * cap);
  // per-wave counts | running total (screen) | published total: zeroed once
  // per layout; publish32 clears the running total every step
  if (c.fb_count.bytes < sizeof(int32_t) * (nwaves + 3) || c.fb_layout != nwaves) {
    c.fb_count.ensure(sizeof(int32_t) * (nwaves + 3));
    HIP_CHECK(hipMemsetAsync(c.fb_count.p, 0, sizeof(int32_t) * (nwaves + 3), c.stream));
    c.fb_layout = nwaves;
  }
  c.fb_regions = nwaves;
  c.fb_total_slot = nwaves + 1;
  // pre-centred screen copy (exact; built once per point set)
  const bool pre = c.pre_ok && !exp_env("CDR_NO_PRE");
  if (pre) ensure_precentered(c);
  S32Args a;
  a.X = pre ? c.xt32.as<float>() : c.x32.as<float>();
  a.X0 = c.x32.as<float>();
  a.cent = dcent;
  a.n = c.n;
  a.n_pad = c.n_pad;
  a.d = d;
  a.k = k;
  a.Q = Q;
  a.frag = dfrag;
  a.cinit = dcinit;
  a.mu_s = c.mu_s.as<float>();
  a.sig = (float)std::ldexp(1.0, c.sigma);
  a.thr0 = pl.thr0;
  a.thr_rel = pl.thr_rel;
  a.labels = c.labels.as<int32_t>();
  a.run_sums = c.run_sums.as<unsigned long long>();
  a.muf = pre ? c.muf.as<long long>() : nullptr;
  a.fx = std::ldexp(1.0, c.scale_bits - (pre ? c.sigma : 0));
  a.KP = KP;
  a.fb_list = c.fb_list.as<int32_t>();
  a.fb_count = c.fb_count.as<int32_t>();
  a.fb_cap = cap;
  a.dbg = dbg;
  a.dbg_ld = (k + 15) / 16 * 16;
  a.gate = gate;
  a.thr_dev = dthr;
  snprintf(c.prof_kernel, sizeof(c.prof_kernel), "screen32<%d,%d,%s,%s,%s,%s>", pl.QH, pl.MT,
           Q == 2 * pl.QH ? "true" : "false", delta ? "true" : "false", dbg ? "true" : "false",
           pre ? "true" : "false");
  if (prof) prof_mark(c, 0);
  const dim3 grid(nwg), blk(256);
  const bool fullq = Q == 2 * pl.QH;
#ifdef CDR_EXPERIMENTS
#define CDR_S32P(QH_, MT_, P_)                                                                  \
  if (dbg) hipLaunchKernelGGL((screen32<QH_, MT_, false, false, true, P_>), grid, blk, lds, c.stream, a); \
  else if (fullq && delta) hipLaunchKernelGGL((screen32<QH_, MT_, true, true, false, P_>), grid, blk, lds, c.stream, a); \
  else if (fullq) hipLaunchKernelGGL((screen32<QH_, MT_, true, false, false, P_>), grid, blk, lds, c.stream, a); \
  else if (delta) hipLaunchKernelGGL((screen32<QH_, MT_, false, true, false, P_>), grid, blk, lds, c.stream, a); \
  else hipLaunchKernelGGL((screen32<QH_, MT_, false, false, false, P_>), grid, blk, lds, c.stream, a);
#else
  // (product: DELTA steps take the lean path above, CDR_NO_LEAN is experiments-only)
  if (delta) CDR_FAIL(CDR_ERR_STATE, "screen32: the full DELTA screen is in the experiments build");
#define CDR_S32P(QH_, MT_, P_)                                                                  \
  if (dbg) hipLaunchKernelGGL((screen32<QH_, MT_, false, false, true, P_>), grid, blk, lds, c.stream, a); \
  else if (fullq) hipLaunchKernelGGL((screen32<QH_, MT_, true, false, false, P_>), grid, blk, lds, c.stream, a); \
  else hipLaunchKernelGGL((screen32<QH_, MT_, false, false, false, P_>), grid, blk, lds, c.stream, a);
#endif
#define CDR_S32(QH_, MT_) \
  if (pre) { CDR_S32P(QH_, MT_, true) } else { CDR_S32P(QH_, MT_, false) }
#ifdef CDR_EXPERIMENTS
  const int abl = c.screen_ablate;
  if (abl && pl.QH == 2 && pl.MT == 2 && fullq && delta && pre) {  // timing experiments only
    switch (abl) {
      case 1: hipLaunchKernelGGL((screen32<2, 2, true, true, false, true, 1>), grid, blk, lds, c.stream, a); break;
      case 2: hipLaunchKernelGGL((screen32<2, 2, true, true, false, true, 2>), grid, blk, lds, c.stream, a); break;
      case 3: hipLaunchKernelGGL((screen32<2, 2, true, true, false, true, 3>), grid, blk, lds, c.stream, a); break;
      case 8: hipLaunchKernelGGL((screen32<2, 2, true, true, false, true, 8>), grid, blk, lds, c.stream, a); break;
      case 9: hipLaunchKernelGGL((screen32<2, 2, true, true, false, true, 9>), grid, blk, lds, c.stream, a); break;
      case 11: hipLaunchKernelGGL((screen32<2, 2, true, true, false, true, 11>), grid, blk, lds, c.stream, a); break;
      default: hipLaunchKernelGGL((screen32<2, 2, true, true, false, true, 0>), grid, blk, lds, c.stream, a); break;
    }
  } else
#endif
  if (pl.QH == 1 && pl.MT == 1) { CDR_S32(1, 1) }
  else if (pl.QH == 1) { CDR_S32(1, 2) }
  else if (pl.MT == 1) { CDR_S32(2, 1) }
  else { CDR_S32(2, 2) }
#undef CDR_S32P
#undef CDR_S32
  HIP_CHECK(hipGetLastError());
  if (prof) prof_mark(c, 1);
  long long* hout_dev = nullptr;
  if (hout) {
    void* hp = nullptr;
    HIP_CHECK(hipHostGetDevicePointer(&hp, hout, 0));
    hout_dev = static_cast<long long*>(hp);
  }
  c.fb_accum.ensure(2 * sizeof(long long));
  if (dout || hout_dev || !gate) {
    // (device loop with no all-reduce buffer: ll_finalize reads the slices and
    // moves the fallback counter itself)
    hipLaunchKernelGGL(publish32, dim3((unsigned)std::max(1, (len + 255) / 256)), dim3(256), 0,
                       c.stream, c.run_sums.as<long long>(),
                       len, dout, hout_dev, gate ? nullptr : c.fb_count.as<int32_t>(), nwaves,
                       c.prof_on ? c.fb_accum.as<long long>() : nullptr, gate);
    HIP_CHECK(hipGetLastError());
  }
  c.run_valid = dbg == nullptr;
  c.run_k = k;
  return true;
}

}  // namespace cdr
