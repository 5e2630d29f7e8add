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
  int32_t* fb_list;
  int32_t* fb_count;
  float* dbg;  // optional: screen values (n_pad x KT*16) for tests
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
          xr[p][c][i] = fok[c][i] ? a.X[(int64_t)f * a.n_pad + base + 16 * p + col] : 0.0f;
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
#pragma unroll
        for (int c = 0; c < DCH; ++c) {
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1[c], b1[p][c], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(A2[c], b2[p][c], acc, 0, 0, 0);
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
      const bool cert = vs > lim;  // NaN-safe: a NaN runner-up never certifies
      const int64_t pt = base + 16 * p + col;
      const bool real = pt < a.n;
      if (g == 0 && real) a.labels[pt] = label;
      const bool need = (g == 0) && real && !cert;
      const unsigned long long m = __ballot(need);
      if (m) {
        const int leader = __builtin_ctzll(m);
        int basei = 0;
        if (lane == leader) basei = atomicAdd(a.fb_count, __popcll(m));
        basei = __shfl(basei, leader);
        const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        if (need) a.fb_list[basei + rank] = (int32_t)pt;
      }
      if (real && cert) {
        unsigned long long* row = tbl + (size_t)label * kd1;
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
  __syncthreads();
  unsigned long long* dst = a.partials + (size_t)blockIdx.x * a.k * kd1;
  for (int i = threadIdx.x; i < a.k * kd1; i += blockDim.x) dst[i] = tbl[i];
}

__global__ void reduce_partials(const long long* __restrict__ part, int nwg, int len,
                                long long* __restrict__ out) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x) {
    long long s = 0;
    for (int w = 0; w < nwg; ++w) s += part[(size_t)w * len + i];
    out[i] = s;
  }
}

// Exact NumPy-order argmin over k centroids (row-major fp64 C).  sqrt is only
// evaluated when the squared distance drops, which keeps first-index ties of
// the *square roots* exactly as np.argmin(np.linalg.norm(...)) sees them.
template <typename XF>
__device__ __forceinline__ int exact_argmin(XF xv, const double* __restrict__ C, int k,
                                            int d) {
  double Rb = INFINITY, rb = INFINITY;
  int jb = 0;
  for (int j = 0; j < k; ++j) {
    const double* cj = C + (size_t)j * d;
    const double R = np_sqdist(xv, [&](int f) { return cj[f]; }, d);
    if (R < Rb) {
      const double r = sqrt(R);
      if (r < rb) {
        rb = r;
        Rb = R;
        jb = j;
      }
    }
  }
  return jb;
}

__global__ void fallback_exact_f32x(const float* __restrict__ X, int64_t n_pad, int d,
                                    const double* __restrict__ C, int k,
                                    const int32_t* __restrict__ list,
                                    const int32_t* __restrict__ count,
                                    int32_t* __restrict__ labels,
                                    unsigned long long* __restrict__ out, float fx) {
  const int cnt = *count;
  const int kd1 = d + 1;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < cnt;
       idx += gridDim.x * blockDim.x) {
    const int64_t pt = list[idx];
    auto xv = [&](int f) { return (double)X[(int64_t)f * n_pad + pt]; };
    const int jb = exact_argmin(xv, C, k, d);
    labels[pt] = jb;
    for (int f = 0; f < d; ++f) {
      const long long u = (long long)(int)(X[(int64_t)f * n_pad + pt] * fx);
      atomicAdd(&out[(size_t)jb * kd1 + f], (unsigned long long)u);
    }
    atomicAdd(&out[(size_t)jb * kd1 + d], 1ull);
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
    auto xv = [&](int f) { return (double)X[(int64_t)f * n_pad + pt]; };
    labels[pt] = exact_argmin(xv, C, k, d);
  }
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
      atomicAdd(&row[f], (unsigned long long)(long long)(int)(X[(int64_t)f * n_pad + pt] * fx));
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
  const double* col = X + (int64_t)f * n_pad;
  if (d >= 2) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i)
      if (labels[i] == j) s = s + col[i];
    sums[(size_t)j * d + f] = s;
    return;
  }
  // d == 1: res = 0; res += pairwise(block) for each 8192-block of the selection.
  const long long m = counts_in[j];
  int64_t cursor = 0;
  auto next = [&](int64_t) -> double {
    while (labels[cursor] != j) ++cursor;
    return col[cursor++];
  };
  double res = 0.0;
  for (long long done = 0; done < m; done += kSeedBlock) {
    const long long blk = (m - done) < kSeedBlock ? (m - done) : kSeedBlock;
    res = res + np_pairwise(next, blk);
  }
  sums[j] = res;
}

__global__ void count_labels(const int32_t* __restrict__ labels, int64_t n, int k,
                             unsigned long long* __restrict__ counts) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&counts[labels[i]], 1ull);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static int num_cus(int device) {
  static int cached[64] = {0};
  if (device >= 0 && device < 64 && cached[device]) return cached[device];
  int v = 0;
  HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device));
  if (device >= 0 && device < 64) cached[device] = v;
  return v;
}

struct ScreenPlan {
  int DCH, KT;
  bool pack6;
  float thrA0, thrA1;
  std::vector<h8> frag;
};

// Build the fp16 A-operand fragments and the certification constants
// (derivation: DESIGN.md §3 "screen error bound").
static void build_screen_plan(const Ctx& c, const double* C, int k, ScreenPlan& pl) {
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

  pl.frag.assign((size_t)pl.KT * pl.DCH * 2 * 64, h8{});
  for (int t = 0; t < pl.KT; ++t)
    for (int cch = 0; cch < pl.DCH; ++cch)
      for (int lane = 0; lane < 64; ++lane) {
        const int j = 16 * t + (lane & 15);
        const int g = lane >> 4;
        h8 A1 = {}, A2 = {};
        for (int i = 0; i < 4; ++i) {
          const int f = 16 * cch + 4 * g + i;
          if (j < k && f < d) {
            const double v = ch[(size_t)j * d + f];
            const _Float16 hi = (_Float16)v;
            const _Float16 lo = (_Float16)(v - (double)hi);
            A1[2 * i] = (_Float16)(-2.0 * (double)hi);
            A1[2 * i + 1] = (_Float16)(-2.0 * (double)hi);
            A2[2 * i] = (_Float16)(-2.0 * (double)lo);
          }
        }
        if (cch == 0) {
          if (g == 0) {
            A2[1] = A2[3] = A2[5] = (_Float16)1.0f;
          } else if (g == 1) {
            if (j < k) {
              const double v = cc[j] + eps;
              const _Float16 p0 = (_Float16)v;
              const double r1 = v - (double)p0;
              const _Float16 p1 = (_Float16)r1;
              const double r2 = r1 - (double)p1;
              const _Float16 p2 = (_Float16)r2;
              A2[1] = p0;
              A2[3] = p1;
              A2[5] = p2;
            } else {
              A2[1] = (_Float16)30000.0f;  // padding centroid: never the best
            }
          }
        }
        pl.frag[(((size_t)t * pl.DCH + cch) * 2 + 0) * 64 + lane] = A1;
        pl.frag[(((size_t)t * pl.DCH + cch) * 2 + 1) * 64 + lane] = A2;
      }
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

// Fold the last step's event pair into the profile accumulators.
void prof_collect(Ctx& c) {
  if (!c.prof_pending) return;
  HIP_CHECK(hipEventSynchronize(c.pe[2]));
  float a = 0.f, b = 0.f;
  HIP_CHECK(hipEventElapsedTime(&a, c.pe[0], c.pe[1]));
  HIP_CHECK(hipEventElapsedTime(&b, c.pe[0], c.pe[2]));
  c.prof_screen_ms += a;
  c.prof_step_ms += b;
  c.prof_launches += 1;
  c.prof_pending = false;
}

void lloyd_step_f32x(Ctx& c, const double* C, int32_t k, int64_t* out, bool out_dev) {
  check_k(c, k);
  if (c.mode != CDR_MODE_F32X) CDR_FAIL(CDR_ERR_STATE, "lloyd_step: points are not F32X");
  const int d = c.d, kd1 = d + 1, len = k * kd1;
  upload_centroids(c, C, k);
  long long* dout;
  if (out_dev) {
    dout = reinterpret_cast<long long*>(out);
  } else {
    c.out_sums.ensure(sizeof(long long) * len);
    dout = c.out_sums.as<long long>();
  }
  c.fb_count.ensure(16);
  HIP_CHECK(hipMemsetAsync(c.fb_count.p, 0, 16, c.stream));
  c.fb_list.ensure(sizeof(int32_t) * (c.n > 0 ? c.n : 1));
  const float fx = (float)std::ldexp(1.0, c.scale_bits);
  const int cus = num_cus(c.device);

  prof_collect(c);
  const bool prof = c.prof_on;
  if (screen_supported(c, k)) {
    ScreenPlan pl;
    build_screen_plan(c, C, k, pl);
    c.frag.ensure(pl.frag.size() * sizeof(h8));
    HIP_CHECK(hipMemcpyAsync(c.frag.p, pl.frag.data(), pl.frag.size() * sizeof(h8),
                             hipMemcpyHostToDevice, c.stream));
    const size_t lds = screen_lds_bytes(pl.KT, pl.DCH, k, d);
    const int64_t groups = c.n_pad / 64;
    int nwg = (int)std::min<int64_t>(ceil_div(groups, 4), (int64_t)cus * 4);
    if (nwg < 1) nwg = 1;
    c.partials.ensure(sizeof(long long) * (size_t)nwg * len);
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
    a.dbg = g_dbg_ptr;
    const bool dbg = g_dbg_ptr != nullptr;
    if (prof) HIP_CHECK(hipEventRecord(c.pe[0], c.stream));
    switch (pl.DCH) {
      case 1: launch_screen<1>(pl.pack6, dbg, dim3(nwg), lds, c.stream, a); break;
      case 2: launch_screen<2>(pl.pack6, dbg, dim3(nwg), lds, c.stream, a); break;
      case 3: launch_screen<3>(pl.pack6, dbg, dim3(nwg), lds, c.stream, a); break;
      default: launch_screen<4>(pl.pack6, dbg, dim3(nwg), lds, c.stream, a); break;
    }
    HIP_CHECK(hipGetLastError());
    if (prof) HIP_CHECK(hipEventRecord(c.pe[1], c.stream));
    hipLaunchKernelGGL(reduce_partials, dim3((len + 255) / 256), dim3(256), 0, c.stream,
                       c.partials.as<long long>(), nwg, len, dout);
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(fallback_exact_f32x, dim3(cus * 4), dim3(256), 0, c.stream,
                       c.x32.as<float>(), c.n_pad, d, c.cent64.as<double>(), k,
                       c.fb_list.as<int32_t>(), c.fb_count.as<int32_t>(),
                       c.labels.as<int32_t>(), reinterpret_cast<unsigned long long*>(dout), fx);
    HIP_CHECK(hipGetLastError());
  } else {
    // exact assignment for every point, then fixed-point sums from labels
    hipLaunchKernelGGL(assign_exact_all<float>, dim3(std::max(1, (int)std::min<int64_t>(ceil_div(c.n, 256), cus * 8))),
                       dim3(256), 0, c.stream, c.x32.as<float>(), c.n, c.n_pad, d,
                       c.cent64.as<double>(), k, c.labels.as<int32_t>());
    HIP_CHECK(hipGetLastError());
    const size_t lds = (size_t)len * 8;
    if (lds > 64 * 1024) CDR_FAIL(CDR_ERR_UNSUPPORTED, "k*(d+1) too large for the update table");
    int nwg = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(c.n, 256), cus * 2));
    c.partials.ensure(sizeof(long long) * (size_t)nwg * len);
    hipLaunchKernelGGL(update_from_labels_f32x, dim3(nwg), dim3(256), lds, c.stream,
                       c.x32.as<float>(), c.n, c.n_pad, d, k, c.labels.as<int32_t>(), fx,
                       c.partials.as<unsigned long long>());
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(reduce_partials, dim3((len + 255) / 256), dim3(256), 0, c.stream,
                       c.partials.as<long long>(), nwg, len, dout);
    HIP_CHECK(hipGetLastError());
  }
  if (prof && screen_supported(c, k)) {
    HIP_CHECK(hipEventRecord(c.pe[2], c.stream));
    c.prof_pending = true;
  }
  c.last_k = k;
  c.have_labels = true;
  if (!out_dev) {
    c.h_small.ensure(sizeof(long long) * len + 64);
    HIP_CHECK(hipMemcpyAsync(c.h_small.p, dout, sizeof(long long) * len,
                             hipMemcpyDeviceToHost, c.stream));
    int32_t fb = 0;
    HIP_CHECK(hipMemcpyAsync(&fb, c.fb_count.p, sizeof(int32_t), hipMemcpyDeviceToHost,
                             c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    memcpy(out, c.h_small.p, sizeof(long long) * len);
    c.last_fallback = screen_supported(c, k) ? fb : c.n;
    if (c.prof_pending) c.prof_fb_points += fb;
    prof_collect(c);
  } else {
    c.last_fallback = -1;  // unknown until cdr_lloyd_stats synchronises
  }
}

void lloyd_step_f64(Ctx& c, const double* C, int32_t k, double* sums, int64_t* counts) {
  check_k(c, k);
  if (c.mode != CDR_MODE_F64) CDR_FAIL(CDR_ERR_STATE, "lloyd_step_f64: points are not F64");
  const int d = c.d;
  const int cus = num_cus(c.device);
  upload_centroids(c, C, k);
  hipLaunchKernelGGL(assign_exact_all<double>,
                     dim3(std::max(1, (int)std::min<int64_t>(ceil_div(c.n, 256), cus * 8))),
                     dim3(256), 0, c.stream, c.x64.as<double>(), c.n, c.n_pad, d,
                     c.cent64.as<double>(), k, c.labels.as<int32_t>());
  HIP_CHECK(hipGetLastError());
  c.f64_sums.ensure(sizeof(double) * (size_t)k * d);
  c.f64_counts.ensure(sizeof(long long) * k * 2);
  long long* cnt_pre = c.f64_counts.as<long long>() + k;
  HIP_CHECK(hipMemsetAsync(cnt_pre, 0, sizeof(long long) * k, c.stream));
  hipLaunchKernelGGL(count_labels, dim3(std::max(1, (int)std::min<int64_t>(ceil_div(c.n, 256), 1024))),
                     dim3(256), 0, c.stream, c.labels.as<int32_t>(), c.n, k,
                     reinterpret_cast<unsigned long long*>(cnt_pre));
  HIP_CHECK(hipGetLastError());
  const int threads = k * (d + 1);
  hipLaunchKernelGGL(seq_sums_f64, dim3((threads + 63) / 64), dim3(64), 0, c.stream,
                     c.x64.as<double>(), c.n, c.n_pad, d, k, c.labels.as<int32_t>(), cnt_pre,
                     c.f64_sums.as<double>(), c.f64_counts.as<long long>());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(sums, c.f64_sums.p, sizeof(double) * (size_t)k * d,
                           hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(counts, c.f64_counts.p, sizeof(long long) * k,
                           hipMemcpyDeviceToHost, c.stream));
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

int cdr_lloyd_stats(cdr_ctx* h, int64_t* n_fallback) {
  CDR_TRY
  if (!h || !n_fallback) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  if (c.last_fallback < 0) {
    HIP_CHECK(hipSetDevice(c.device));
    int32_t fb = 0;
    HIP_CHECK(hipMemcpyAsync(&fb, c.fb_count.p, sizeof(int32_t), hipMemcpyDeviceToHost,
                             c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    c.last_fallback = screen_supported(c, c.last_k) ? fb : c.n;
  }
  *n_fallback = c.last_fallback;
  CDR_CATCH
}

int cdr_profile_reset(cdr_ctx* h, int32_t enable) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  for (int i = 0; i < 3; ++i)
    if (!c.pe[i]) HIP_CHECK(hipEventCreate(&c.pe[i]));
  if (c.prof_pending) HIP_CHECK(hipEventSynchronize(c.pe[2]));
  c.prof_pending = false;
  c.prof_on = enable != 0;
  c.prof_screen_ms = c.prof_step_ms = c.prof_fb_points = 0.0;
  c.prof_launches = 0;
  CDR_CATCH
}

int cdr_profile_read(cdr_ctx* h, double* out) {
  CDR_TRY
  if (!h || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  prof_collect(c);
  out[0] = c.prof_screen_ms;
  out[1] = (double)c.prof_launches;
  out[2] = c.prof_step_ms;
  out[3] = c.prof_fb_points;
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
    ScreenPlan pl;
    build_screen_plan(c, C, k, pl);
    thr_a0a1[0] = pl.thrA0;
    thr_a0a1[1] = pl.thrA1;
  }
  CDR_CATCH
}

}  // extern "C"
