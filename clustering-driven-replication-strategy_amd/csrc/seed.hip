// seed.hip — k-means++ D^2 seeding (reference src/kmeans_plusplus.py:3-22).
//
// Per step i (one new centre c):
//   dist_sq = min(dist_sq, norm(X - c)**2)        :14-17  (running min is exact:
//                                                         min is order free)
//   total   = dist_sq.sum()                        :18     NumPy add.reduce: 8192-
//             element chunks, pairwise inside each chunk, chunks added left to right
//   idx     = rng.choice(n, p=dist_sq/total)       :19     = searchsorted(cumsum(p) /
//             cumsum(p)[-1], rng.random(), 'right') (one draw; u comes from host)
//
// The cumulative sum is where a parallel scan would change the rounding.  We
// emulate NumPy's strictly sequential fp64 accumulation exactly:
//   while the running value c stays inside one binade [2^e, 2^(e+1)), every
//   fl(c + p) lands on the grid g = 2^(e-52), so c/g = N is an integer and
//   N' = N + rne(p/g) — independent of N except for exact ties, where round-
//   half-even looks at the parity of N.  A run of elements is therefore a
//   *transfer* (D0, D1): the increment of N when N enters even / odd.  Two
//   transfers compose as D_q = L_q + R_{q ^ (L_q & 1)} (associative), so
//   blocks are reduced in parallel; a single wave then walks the blocks,
//   applying whole blocks inside a binade and walking element by element only
//   across the ~log2(c_last/c_first) binade crossings.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hip/hip_fp16.h>

#include "cdr_internal.h"
#include "exact_math.h"

namespace cdr {

void ensure_rowmajor(Ctx& c);  // screen32.hip: the row-major copy xa32

struct Xfer {
  long long d0, d1;
  int e;      // binade exponent the transfer was computed for
  int valid;  // 0: some element would leave the binade / overflow
  long long pad;
};

constexpr int kSub = 128;  // elements per lane in a block (8192 = 64 x 128)

__global__ void fill_inf(double* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = INFINITY;
}

// Pairwise tree skeleton of NumPy's pairwise_sum with leaves produced by a
// functor leaf(off, m) (m <= 128) — same recursion as np_pairwise.
template <typename LF>
__device__ double pw_tree(int64_t n, LF leaf) {
  if (n <= 128) return leaf((int64_t)0, (int)n);
  struct Frame {
    int64_t off, n;
    int state;
    double left;
  };
  Frame st[48];
  int sp = 0;
  st[0] = {0, n, 0, 0.0};
  double ret = 0.0;
  bool have = false;
  while (sp >= 0) {
    Frame& fr = st[sp];
    if (have) {
      if (fr.state == 1) {
        fr.left = ret;
        fr.state = 2;
        have = false;
        int64_t n2 = fr.n / 2;
        n2 -= n2 % 8;
        st[sp + 1] = {fr.off + n2, fr.n - n2, 0, 0.0};
        ++sp;
      } else {
        ret = fr.left + ret;
        --sp;
      }
      continue;
    }
    if (fr.n <= 128) {
      ret = leaf(fr.off, (int)fr.n);
      have = true;
      --sp;
      continue;
    }
    int64_t n2 = fr.n / 2;
    n2 -= n2 % 8;
    fr.state = 1;
    st[sp + 1] = {fr.off, n2, 0, 0.0};
    ++sp;
  }
  return ret;
}

// One workgroup (256 threads) per 8192-point block.  The block is handled in
// two halves of 4096 (pw(8192) = pw(4096) + pw(4096)); each half's values sit
// in LDS (one pad slot per 16).
//
// Full blocks: the 32 pairwise leaves of 128 of a half are
// summed by 8 threads each — thread (leaf L, j) adds NumPy's accumulator r_j
// = a(j) + a(j + 8) + ... sequentially, shfl_xor 1, 2, 4 forms
// ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), shfl_xor 8, 16, 32 and
// then a 4-wave LDS step combine the leaves in the balanced tree of
// pw(4096).
// The one partial block (m < 8192) is the grid's last workgroup: it updates
// its dmin values with the others and leaves its pairwise sum to
// seed_tail_sum_kernel (a stack walk of the tree: scratch memory, kept out
// of this kernel).
// D > 0 (float points, d == D <= 16): each thread takes 4 points per
// iteration with all their 16-byte feature-quad loads and dmin loads issued
// before any arithmetic, and the NumPy-order distance unrolled for that d.
// Exact pruning of the running minimum (the k-means++ D^2 step,
// src/kmeans_plusplus.py:14-17): the point's nearest centre so far, c_a =
// near[i], is at distance r with dmin = fl(r^2); if the new centre is at
// least 2 r (1 + 2^-30) from c_a, the triangle inequality puts it at least
// r (1 + 2^-30) from the point, so its computed squared distance (NumPy
// order, relative error < 2^-45 at d <= 128) is >= dmin and min(dmin, .)
// leaves dmin unchanged bit for bit: the point is not read at all.
// ccd[j] = ||c_j - c_new|| (fp64, relative error < 2^-48).  dmin = +inf (no
// centre yet) never prunes.
__device__ __forceinline__ bool seed_prunable(double ccd_a, double dmin_old) {
  return ccd_a >= 2.0 * sqrt(dmin_old) * (1.0 + 0x1p-30);
}

// ccd[j] = ||cents[j] - cen|| for the j < count centres so far.
__global__ void seed_ccd_kernel(const double* __restrict__ cents, int count, int d,
                                const double* __restrict__ cen, double* __restrict__ ccd) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < count; j += gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int f = 0; f < d; ++f) {
      const double t = cents[(size_t)j * d + f] - cen[f];
      s += t * t;
    }
    ccd[j] = sqrt(s);
  }
}

template <typename T, int D>
__global__ __launch_bounds__(256) void seed_update_kernel(
    const T* __restrict__ X, int64_t n, int64_t n_pad, int d, const double* __restrict__ cen,
    double* __restrict__ dmin, double* __restrict__ blocksums, int32_t* __restrict__ near,
    const double* __restrict__ ccd, int cidx) {
  constexpr int kHalf = 4096;
  __shared__ double sdm[kHalf + kHalf / 16];
  __shared__ double swave[4];
  const int64_t b = blockIdx.x;
  const int64_t base = b * kSeedBlock;
  const int m = (n - base) < kSeedBlock ? (int)(n - base) : kSeedBlock;
  const bool TAIL = m < kSeedBlock;  // workgroup-uniform: the partial last block
  auto spos = [](int q) { return q + (q >> 4); };
  double halves[2] = {0.0, 0.0};
  for (int h = 0; h < 2; ++h) {
    if constexpr (D > 0) {
      constexpr int Q = (D + 3) / 4;
      // points per thread and iteration: all their loads issue before any
      // arithmetic (fewer for wide rows: registers)
      constexpr int U = D <= 16 ? 4 : (D <= 32 ? 2 : 1);
      // the centre in registers for narrow rows, else uniform (scalar) loads
      constexpr int CR = D <= 16 ? D : 1;
      typedef float f4v __attribute__((ext_vector_type(4)));
      const f4v* X4 = reinterpret_cast<const f4v*>(X);
      double cr[CR];
#pragma unroll
      for (int f = 0; f < CR; ++f) cr[f] = cen[f];
      for (int q0 = threadIdx.x; q0 < kHalf; q0 += U * 256) {
        f4v xv[U][Q];
        double old[U];
        bool go[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int qi = h * kHalf + q0 + 256 * u;
          const int64_t i = base + qi;
          go[u] = false;
          if (!TAIL || qi < m) {
            old[u] = dmin[i];
            go[u] = cidx == 0 || !seed_prunable(ccd[near[i]], old[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = base + h * kHalf + q0 + 256 * u;
          if (go[u]) {
#pragma unroll
            for (int qq = 0; qq < Q; ++qq) xv[u][qq] = X4[(int64_t)qq * n_pad + i];
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int q = q0 + 256 * u;
          const int qi = h * kHalf + q;
          double v = 0.0;
          if (!TAIL || qi < m) {
            v = old[u];
            if (go[u]) {
              auto xf = [&](int f) { return (double)xv[u][f >> 2][f & 3]; };
              auto cf = [&](int f) { return D <= 16 ? cr[f < CR ? f : 0] : cen[f]; };
              const double R = np_sqdist(xf, cf, D);
              const double r = sqrt(R);
              const double t = r * r;
              if (t < old[u]) {
                v = t;
                dmin[base + qi] = t;
                near[base + qi] = cidx;
              }
            }
          }
          sdm[spos(q)] = v;
        }
      }
    } else {
      for (int q = threadIdx.x; q < kHalf; q += blockDim.x) {
        const int qi = h * kHalf + q;
        const int64_t i = base + qi;
        double v = 0.0;
        if (!TAIL || qi < m) {
          const double old = dmin[i];
          v = old;
          if (cidx == 0 || !seed_prunable(ccd[near[i]], old)) {
            auto xv = [&](int f) { return (double)X[xidx(X, f, i, n_pad)]; };
            auto cv = [&](int f) { return cen[f]; };
            const double R = np_sqdist(xv, cv, d);
            const double r = sqrt(R);
            const double t = r * r;
            if (t < old) {
              v = t;
              dmin[i] = t;
              near[i] = cidx;
            }
          }
        }
        sdm[spos(q)] = v;
      }
    }
    __syncthreads();
    if (!TAIL) {
      const int t = threadIdx.x;
      const int L = t >> 3, j = t & 7;
      double r = sdm[spos(128 * L + j)];
#pragma unroll
      for (int i = 1; i < 16; ++i) r = r + sdm[spos(128 * L + j + 8 * i)];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) r = r + __shfl_xor(r, o);
      if ((t & 63) == 0) swave[t >> 6] = r;
      __syncthreads();
      if (t == 0) halves[h] = (swave[0] + swave[1]) + (swave[2] + swave[3]);
      __syncthreads();
    }
  }
  if (!TAIL && threadIdx.x == 0) blocksums[b] = halves[0] + halves[1];
}

// ---- fp16-certified update (F32X points, d in {8, 16, 32, 64}) --------------
// A k-means++ step changes few minima: most points are farther from the new
// centre than from their nearest one.  A half-size copy proves that for most
// points without reading them in fp32: x16 = fp16 of xh = (x - mu) 2^tau
// (tau = sigma + 14, |xh| < 2^14), grouped by 8 features, [G][n_pad] x 16 B,
// with e16[i] >= ||xh_i - x16_i|| (computed exactly in fp64 when the copy is
// built, rounded up to fp16).  With ch = (c - mu) 2^tau rounded to fp32 (Ec >=
// ||ch32 - ch||), the fp32 a = ||x16_i - ch32|| has relative error below
// (D + 8) 2^-23, so
//     ||x_i - c|| >= (a (1 - (D + 8) 2^-23) - e16[i] - Ec) 2^-tau = r_lo,
// and r_lo^2 >= dmin (1 + 2^-30) proves the NumPy-order distance (relative
// error < 2^-45, as seed_prunable) is >= dmin: min(dmin, .) leaves it
// unchanged.  Only the points it cannot prove read the fp32 row and take the
// exact path; the triangle-inequality pruning (seed_prunable) runs first.
constexpr int kSeed16Tau = 14;

__global__ __launch_bounds__(256) void seed16_pack_kernel(const float* __restrict__ x32,
                                                          int64_t n, int64_t n_pad, int d,
                                                          const float* __restrict__ mu,
                                                          double scale,
                                                          uint4* __restrict__ x16,
                                                          unsigned short* __restrict__ e16) {
  const int G = (d + 7) / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad;
       i += (int64_t)gridDim.x * blockDim.x) {
    double err = 0.0;
    for (int g = 0; g < G; ++g) {
      unsigned short hv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = 8 * g + j;
        double v = 0.0;
        if (f < d && i < n) v = ((double)x32[xidx(x32, f, i, n_pad)] - (double)mu[f]) * scale;
        const __half h = __float2half_rn((float)v);
        const double dv = v - (double)__half2float(h);
        err += dv * dv;
        hv[j] = __half_as_ushort(h);
      }
      uint4 w;
      w.x = hv[0] | ((unsigned)hv[1] << 16);
      w.y = hv[2] | ((unsigned)hv[3] << 16);
      w.z = hv[4] | ((unsigned)hv[5] << 16);
      w.w = hv[6] | ((unsigned)hv[7] << 16);
      x16[(int64_t)g * n_pad + i] = w;
    }
    // stored as fp16 rounded up (an upper bound; 2 bytes a point, not 4);
    // non-finite (an fp16 overflow) and anything past fp16's range is +inf,
    // which never certifies
    const double e = sqrt(err) * (1.0 + 0x1p-20) + 0x1p-60;
    unsigned short eb = 0x7C00u;
    if (isfinite(e) && e < 65504.0) {
      const __half h = __float2half_rn((float)e);
      eb = __half_as_ushort(h);
      if ((double)__half2float(h) < e) ++eb;  // the next fp16 up (e > 0)
    }
    e16[i] = eb;
  }
}

// The centre in the copy's coordinates: ch = fp32 of (c - mu) 2^tau and Ec >=
// ||ch - (c - mu) 2^tau|| (rounded up), from the device copy of the centre.
__global__ void seed_ch_kernel(const double* __restrict__ cen, const float* __restrict__ mu,
                               int d, double scale, float* __restrict__ ch,
                               float* __restrict__ Ec) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double ec = 0.0;
  for (int f = 0; f < d; ++f) {
    const double v = (cen[f] - (double)mu[f]) * scale;
    const float h = (float)v;
    ch[f] = h;
    const double r = v - (double)h;
    ec += r * r;
  }
  Ec[0] = (float)(sqrt(ec) * (1.0 + 0x1p-20) + 0x1p-60);
}

// PR: the triangle-inequality pruning (seed_prunable) first, so that a pruned
// point does not read its copy — worth it for wide rows; for d <= 16 the
// dependent near / ccd loads cost more than the 32-byte copy they save, and
// dmin and the copy are loaded together in one round trip instead.
template <int D, int UU = 0, bool PR = (D > 16)>
__global__ __launch_bounds__(256) void seed_update16_kernel(
    const float* __restrict__ X, const uint4* __restrict__ x16, const unsigned short* __restrict__ e16,
    int64_t n, int64_t n_pad, const double* __restrict__ cen, const float* __restrict__ ch,
    const float* __restrict__ Ecp, double rscale, double* __restrict__ dmin,
    double* __restrict__ blocksums,
    int32_t* __restrict__ near, const double* __restrict__ ccd, int cidx) {
  constexpr int kHalf = 4096;
  constexpr int G = (D + 7) / 8;
  constexpr int Q = (D + 3) / 4;
  constexpr int U = UU ? UU : (D <= 8 ? 4 : (D <= 32 ? 2 : 1));
  constexpr float kRel = 1.0f - (float)(D + 8) * 0x1p-23f;
  const float Ec = Ecp[0];
  __shared__ double sdm[kHalf + kHalf / 16];
  __shared__ double swave[4];
  const int64_t b = blockIdx.x;
  const int64_t base = b * kSeedBlock;
  const int m = (n - base) < kSeedBlock ? (int)(n - base) : kSeedBlock;
  const bool TAIL = m < kSeedBlock;
  auto spos = [](int q) { return q + (q >> 4); };
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v* X4 = reinterpret_cast<const f4v*>(X);
  double halves[2] = {0.0, 0.0};
  for (int h = 0; h < 2; ++h) {
    for (int q0 = threadIdx.x; q0 < kHalf; q0 += U * 256) {
      double old[U];
      bool go[U];
      uint4 hv[U][G];
      float ev[U];
      if constexpr (PR) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int qi = h * kHalf + q0 + 256 * u;
          const int64_t i = base + qi;
          go[u] = false;
          old[u] = 0.0;
          if (qi < m) {
            old[u] = dmin[i];
            go[u] = cidx == 0 || !seed_prunable(ccd[near[i]], old[u]);
          }
        }
        // the fp16 certificate
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = base + h * kHalf + q0 + 256 * u;
          if (go[u]) {
#pragma unroll
            for (int g = 0; g < G; ++g) hv[u][g] = x16[(int64_t)g * n_pad + i];
            ev[u] = __half2float(__ushort_as_half(e16[i]));
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int qi = h * kHalf + q0 + 256 * u;
          const int64_t i = base + qi;
          go[u] = qi < m;
          old[u] = 0.0;
          if (go[u]) {
            old[u] = dmin[i];
#pragma unroll
            for (int g = 0; g < G; ++g) hv[u][g] = x16[(int64_t)g * n_pad + i];
            ev[u] = __half2float(__ushort_as_half(e16[i]));
          }
        }
      }
      bool need[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        need[u] = go[u];
        if (go[u] && cidx > 0) {
          float s = 0.0f;
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const unsigned w[4] = {hv[u][g].x, hv[u][g].y, hv[u][g].z, hv[u][g].w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              if (8 * g + j < D) {
                const float xv = __half2float(
                    __ushort_as_half((unsigned short)(w[j >> 1] >> (16 * (j & 1)))));
                const float t = xv - ch[8 * g + j];
                s = fmaf(t, t, s);
              }
            }
          }
          const float lo = sqrtf(s) * kRel - ev[u] - Ec;
          if (lo > 0.0f) {
            const double r = (double)lo * rscale;
            need[u] = !(r * r >= old[u] * (1.0 + 0x1p-30));
          }
        }
      }
      // the exact path for the points left
      f4v xv[U][Q];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + h * kHalf + q0 + 256 * u;
        if (need[u]) {
#pragma unroll
          for (int qq = 0; qq < Q; ++qq) xv[u][qq] = X4[(int64_t)qq * n_pad + i];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + 256 * u;
        const int qi = h * kHalf + q;
        double v = old[u];
        if (need[u]) {
          auto xf = [&](int f) { return (double)xv[u][f >> 2][f & 3]; };
          auto cf = [&](int f) { return cen[f]; };
          const double R = np_sqdist(xf, cf, D);
          const double r = sqrt(R);
          const double t = r * r;
          if (t < old[u]) {
            v = t;
            dmin[base + qi] = t;
            near[base + qi] = cidx;
          }
        }
        sdm[spos(q)] = qi < m ? v : 0.0;
      }
    }
    __syncthreads();
    if (!TAIL) {
      const int t = threadIdx.x;
      const int L = t >> 3, j = t & 7;
      double r = sdm[spos(128 * L + j)];
#pragma unroll
      for (int i = 1; i < 16; ++i) r = r + sdm[spos(128 * L + j + 8 * i)];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) r = r + __shfl_xor(r, o);
      if ((t & 63) == 0) swave[t >> 6] = r;
      __syncthreads();
      if (t == 0) halves[h] = (swave[0] + swave[1]) + (swave[2] + swave[3]);
      __syncthreads();
    }
  }
  if (!TAIL && threadIdx.x == 0) blocksums[b] = halves[0] + halves[1];
}

// The update with the block's pairwise tree kept in registers (the default
// for d = 8 and 16; CDR_SEED16_LDS=1: seed_update16_kernel).  One
// 512-thread workgroup per 8192-row block; thread (half h, leaf L, j) owns
// NumPy's accumulator j of the 128-element leaf L of half h, i.e. the rows
// 128 L + j + 8 i (i = 0 .. 15), and adds its 16 updated minima in NumPy's
// order (r = v_0, then r += v_i) from registers: no LDS staging of the
// half's 4096 values (34 KB per workgroup capped seed_update16_kernel at 4
// workgroups per CU) and no transposed re-read.  Accumulators combine by
// shuffles ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) and the leaves
// and waves by the same perfect tree, exactly seed_update16_kernel's sums.
// A wave's load instruction reads 8 runs of 8 consecutive rows (64 B of
// dmin, 128 B of each copy group).  Rows are taken 4 per batch, the batch's
// loads issued together; the fp32 row is read only where the fp16
// certificate cannot prove the minimum unchanged.
// The exact path is compacted per wave (round 6).  PMC put the previous form
// (each batch gathering its uncertified rows in place) at TD 97 % / TA 81 %
// busy with 44K vector-memory instructions per CU and launch, ~19K of them
// the exact path's row gathers: a batch ran them whenever any lane of the
// wave could not certify a row, with one or two lanes active.  Here phase 1 streams every row of the thread (certificate
// only) and keeps its 16 current minima in registers with a 16-bit mask of
// the rows left; phase 2 lists the wave's (lane, row) pairs in LDS and
// evaluates them 64 at a time, one per lane (a full-width gather); phase 3
// adds the thread's 16 values in NumPy's order as before.  Same values, same
// order: dmin, near and the block sums are bit-identical.  1.15 -> 1.08 ms per
// launch on average at config 3 (the converged steps stay ~0.91 ms: the
// streamed 42 B per row at ~4.8 TB/s), seeding 0.1075 -> 0.1055 s.
template <int D>
__global__ __launch_bounds__(512) void seed_update16c_kernel(
    const float* __restrict__ X, const uint4* __restrict__ x16, const unsigned short* __restrict__ e16,
    int64_t n, int64_t n_pad, const double* __restrict__ cen, const float* __restrict__ ch,
    const float* __restrict__ Ecp, double rscale, double* __restrict__ dmin,
    double* __restrict__ blocksums, int32_t* __restrict__ near, int cidx,
    const float* __restrict__ XA) {
  constexpr int G = (D + 7) / 8;
  constexpr int Q = (D + 3) / 4;
  constexpr int kB = D <= 8 ? 4 : 2;
  constexpr float kRel = 1.0f - (float)(D + 8) * 0x1p-23f;
  constexpr int kCap = 256;  // exact rows per wave and round
  __shared__ double swave[8];
  __shared__ unsigned short slist[8][kCap];
  __shared__ double supd[8][kCap];
  const float Ec = Ecp[0];
  const int64_t b = blockIdx.x;
  const int64_t base = b * kSeedBlock;
  const int m = (n - base) < kSeedBlock ? (int)(n - base) : kSeedBlock;
  const int t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  const int h = t >> 8, L = (t >> 3) & 31, j = t & 7;
  const int r0 = h * 4096 + 128 * L + j;  // row of i = 0 (row of i: r0 + 8 i)
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v* X4 = reinterpret_cast<const f4v*>(X);
  const f4v* XA4 = reinterpret_cast<const f4v*>(XA);
  float chv[D];
#pragma unroll
  for (int f = 0; f < D; ++f) chv[f] = ch[f];
  struct SB {
    double old[kB];
    uint4 hv[kB][G];
    float ev[kB];
  };
  auto sload = [&](SB& sb, int i0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int r = r0 + 8 * (i0 + u);
      const int64_t i = base + (r < m ? r : 0);
      sb.old[u] = dmin[i];
#pragma unroll
      for (int g = 0; g < G; ++g) sb.hv[u][g] = x16[(int64_t)g * n_pad + i];
      sb.ev[u] = __half2float(__ushort_as_half(e16[i]));
    }
  };
  // phase 1: the certificate over the thread's 16 rows
  double ov[16];
  unsigned nm = 0;
  if (cidx == 0) {
    // the first centre: every minimum is +inf, nothing to certify - the
    // exact distances straight from the rows, 4 rows' loads in flight (not
    // the stream of copies and bounds plus a list of every row)
#pragma unroll
    for (int i0 = 0; i0 < 16; i0 += 4) {
      f4v xv[4][Q];
      double old[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = r0 + 8 * (i0 + u);
        const int64_t row = base + (r < m ? r : 0);
        old[u] = dmin[row];
#pragma unroll
        for (int qq = 0; qq < Q; ++qq)
          xv[u][qq] = XA4 ? XA4[row * Q + qq] : X4[(int64_t)qq * n_pad + row];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = r0 + 8 * (i0 + u);
        double v = 0.0;
        if (r < m) {
          auto xf = [&](int f) { return (double)xv[u][f >> 2][f & 3]; };
          auto cf = [&](int f) { return cen[f]; };
          const double R = np_sqdist(xf, cf, D);
          const double rt = sqrt(R);
          const double tt = rt * rt;
          v = old[u];
          if (tt < old[u]) {
            v = tt;
            dmin[base + r] = tt;
            near[base + r] = cidx;
          }
        }
        ov[i0 + u] = v;
      }
    }
  } else {
    SB sbuf[2];
    sload(sbuf[0], 0);
#pragma unroll
    for (int bi = 0; bi < 16 / kB; ++bi) {
      const int i0 = bi * kB;
      if (bi + 1 < 16 / kB) sload(sbuf[(bi + 1) & 1], i0 + kB);
      const SB& sb = sbuf[bi & 1];
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        const bool in = r0 + 8 * (i0 + u) < m;
        bool need = in;
        if (in && cidx > 0) {
          float sacc = 0.0f;
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const unsigned w[4] = {sb.hv[u][g].x, sb.hv[u][g].y, sb.hv[u][g].z, sb.hv[u][g].w};
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              if (8 * g + q < D) {
                const float xv = __half2float(
                    __ushort_as_half((unsigned short)(w[q >> 1] >> (16 * (q & 1)))));
                const float dd = xv - chv[8 * g + q];
                sacc = fmaf(dd, dd, sacc);
              }
            }
          }
          const float lo = sqrtf(sacc) * kRel - sb.ev[u] - Ec;
          if (lo > 0.0f) {
            const double rr = (double)lo * rscale;
            need = !(rr * rr >= sb.old[u] * (1.0 + 0x1p-30));
          }
        }
        ov[i0 + u] = in ? sb.old[u] : 0.0;
        if (need) nm |= 1u << (i0 + u);
      }
    }
  }
  // phase 2: the wave's uncertified rows, one per lane
  const int cnt = __popc(nm);
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  const int total = __shfl(incl, 63);
  const int myoff = incl - cnt;
  for (int e0 = 0; e0 < total; e0 += kCap) {  // (wave-uniform)
    {
      unsigned mm = nm;
      int e = myoff;
      while (mm) {
        const int i = __builtin_ctz(mm);
        mm &= mm - 1u;
        if (e >= e0 && e < e0 + kCap) slist[wv][e - e0] = (unsigned short)((lane << 4) | i);
        ++e;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int nr = total - e0 < kCap ? total - e0 : kCap;
    for (int k0 = 0; k0 < nr; k0 += 64) {
      const int k = k0 + lane;
      if (k < nr) {
        const int ent = slist[wv][k];
        const int ts = wv * 64 + (ent >> 4), i = ent & 15;
        const int64_t row =
            base + (ts >> 8) * 4096 + 128 * ((ts >> 3) & 31) + (ts & 7) + 8 * i;
        f4v xv[Q];
#pragma unroll
        for (int qq = 0; qq < Q; ++qq)
          xv[qq] = XA4 ? XA4[row * Q + qq] : X4[(int64_t)qq * n_pad + row];
        const double old = dmin[row];
        auto xf = [&](int f) { return (double)xv[f >> 2][f & 3]; };
        auto cf = [&](int f) { return cen[f]; };
        const double R = np_sqdist(xf, cf, D);
        const double rt = sqrt(R);
        const double tt = rt * rt;
        double v = old;
        if (tt < old) {
          v = tt;
          dmin[row] = tt;
          near[row] = cidx;
        }
        supd[wv][k] = v;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if ((nm >> i) & 1u) {
        const int e = myoff + __popc(nm & ((1u << i) - 1u));
        if (e >= e0 && e < e0 + kCap) ov[i] = supd[wv][e - e0];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (m < kSeedBlock) return;  // the partial last block: seed_tail_sum_kernel sums it
  // phase 3: NumPy's accumulator j of its leaf: r = v_0, then r += v_i
  double acc = ov[0];
#pragma unroll
  for (int i = 1; i < 16; ++i) acc = acc + ov[i];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) acc = acc + __shfl_xor(acc, o);
  if ((t & 63) == 0) swave[t >> 6] = acc;
  __syncthreads();
  if (t == 0)
    blocksums[b] = ((swave[0] + swave[1]) + (swave[2] + swave[3])) +
                   ((swave[4] + swave[5]) + (swave[6] + swave[7]));
}

// The partial last block's pairwise sum (m < 8192 elements at base): its
// pairwise tree depends on m alone, so the host lays it out once
// (seed_tail_plan): the leaves' (offset, length) pairs, then the internal
// nodes grouped by height (node ids: leaves 0..L-1, internal nodes L.. in
// height order; each internal node = (left id, right id)).  The block is
// staged in LDS with coalesced loads, the leaves are summed in parallel, and
// each height's nodes are added in parallel (<= 7 heights for m < 8192).
// Its dmin values come from the seed_update_kernel launch before it (the
// block is that grid's last workgroup, updated with the other blocks).
constexpr int kTailLeaves = 160;
constexpr int kTailHeights = 16;
__global__ __launch_bounds__(256) void seed_tail_sum_kernel(const double* __restrict__ dmin,
                                                            int64_t b,
                                                            const int* __restrict__ plan,
                                                            int nleaves, int nheights,
                                                            double* __restrict__ blocksums) {
  __shared__ double snode[2 * kTailLeaves];
  __shared__ double sv[kSeedBlock];
  const int64_t base = b * kSeedBlock;
  const int t = threadIdx.x;
  {
    // the whole block, coalesced, 32 loads per thread in flight (dmin is
    // allocated to n_pad: padding slots load, the leaves never read them)
    double v[kSeedBlock / 256];
#pragma unroll
    for (int j = 0; j < kSeedBlock / 256; ++j) v[j] = dmin[base + j * 256 + t];
#pragma unroll
    for (int j = 0; j < kSeedBlock / 256; ++j) sv[j * 256 + t] = v[j];
  }
  __syncthreads();
  if (t < nleaves) {
    const int off = plan[2 * t], len = plan[2 * t + 1];
    snode[t] = np_pw_leaf([&](int i) { return sv[off + i]; }, len);
  }
  const int* hstart = plan + 2 * nleaves;  // nheights + 1 entries
  const int* nodes = hstart + nheights + 1;
  for (int h = 0; h < nheights; ++h) {
    __syncthreads();
    const int a = hstart[h] + t;
    if (a < hstart[h + 1]) snode[nleaves + a] = snode[nodes[2 * a]] + snode[nodes[2 * a + 1]];
  }
  __syncthreads();
  if (t == 0) blocksums[b] = snode[nleaves > 1 ? nleaves + hstart[nheights] - 1 : 0];
}

// ---- cumulative-sum emulation --------------------------------------------

__device__ __forceinline__ void compose(long long L0, long long L1, long long R0, long long R1,
                                        long long& o0, long long& o1) {
  o0 = L0 + ((L0 & 1) ? R1 : R0);
  o1 = L1 + ((L1 & 1) ? R0 : R1);
}

// Transfer of elements [lo, hi) (values v(i)) under binade exponent e.
template <typename V>
__device__ __forceinline__ void range_transfer_v(V v, double S, int64_t lo, int64_t hi, int e,
                                                 long long& D0, long long& D1, int& valid) {
  D0 = 0;
  D1 = 0;
  valid = 1;
  for (int64_t i = lo; i < hi; ++i) {
    const double p = v(i) / S;
    const double f = ldexp(p, 52 - e);
    if (!(f < 4503599627370496.0)) {  // >= 2^52 (or NaN): leaves the binade
      valid = 0;
      continue;
    }
    const double fl = floor(f);
    const double frac = f - fl;
    const long long k = (long long)fl;
    const long long up = frac > 0.5 ? 1 : 0;
    const bool tie = frac == 0.5;
    // incoming parity q = 0
    {
      const long long par = (D0 ^ k) & 1;  // parity of N + fl with N even + D0
      D0 += k + up + ((tie && par) ? 1 : 0);
    }
    {
      const long long par = (1 ^ D1 ^ k) & 1;
      D1 += k + up + ((tie && par) ? 1 : 0);
    }
  }
  if (D0 >= (1ll << 52) || D1 >= (1ll << 52)) valid = 0;
}

__device__ void range_transfer(const double* __restrict__ dmin, double S, int64_t lo,
                               int64_t hi, int e, long long& D0, long long& D1, int& valid) {
  range_transfer_v([&](int64_t i) { return dmin[i]; }, S, lo, hi, e, D0, D1, valid);
}

__device__ __forceinline__ bool binade_of(double c, int& e, long long& N) {
  const unsigned long long bits = __double_as_longlong(c);
  const int ef = (int)((bits >> 52) & 0x7FF);
  if (ef == 0 || ef >= 2046 || (bits >> 63)) return false;  // zero/subnormal/huge/neg
  e = ef - 1023;
  N = (long long)((bits & 0xFFFFFFFFFFFFFull) | (1ull << 52));
  return true;
}
__device__ __forceinline__ double from_binade(int e, long long N) {
  const unsigned long long bits =
      ((unsigned long long)(e + 1023) << 52) | ((unsigned long long)N & 0xFFFFFFFFFFFFFull);
  return __longlong_as_double(bits);
}

// Per-block transfers under the guessed binade of the block's start.  One
// wave per 8192-element block, in 8 passes of 1024: the pass is loaded
// coalesced (16 B per lane per load) into LDS with one pad slot per 16
// elements, then lane l walks elements [16 l, 16 l + 16) of the pass from LDS
// (conflict-free ds_read_b64), the 64 lane transfers are composed in order and
// the pass transfer is composed onto the block's.
// Device-resident seeding (seed_run): the total S, the running value at the
// shard's end and the uniform of the draw live in device memory, written by
// the kernels before; a non-zero *gate (the program's success flag) turns the
// block-walk fallback kernels into no-ops.  Null pointers: the by-value
// arguments hold.
struct SeedDev {
  const double* S = nullptr;
  const double* gate = nullptr;
  const double* c_last = nullptr;
  const double* u = nullptr;
  const double* c_in = nullptr;  // (sharded device seeding: the shard's exact start)
};

constexpr int kPass = 1024;
constexpr int kPassPad = kPass + kPass / 16;

__global__ __launch_bounds__(256) void xfer_kernel(const double* __restrict__ dmin, int64_t n,
                                                   double S, const double* __restrict__ approx,
                                                   int64_t nblocks, Xfer* __restrict__ out,
    SeedDev dv) {
  if (dv.gate && dv.gate[0] != 0.0) return;
  if (dv.S) S = dv.S[0];
  __shared__ double sbuf[4][kPassPad];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t b = (int64_t)blockIdx.x * 4 + w;
  const bool live = b < nblocks;
  double* sb = sbuf[w];
  int e = 0;
  long long Ndummy;
  const bool okg = live && binade_of(approx[b], e, Ndummy);
  const int64_t base = b * kSeedBlock;
  long long T0 = 0, T1 = 0;
  int tv = okg ? 1 : 0;
  for (int ps = 0; ps < kSeedBlock / kPass; ++ps) {
    const int64_t pb = base + (int64_t)ps * kPass;
    const bool act = okg && pb < n;  // wave-uniform
    if (act) {
      // dmin is allocated to n_pad (a multiple of the block): whole passes load
      const double2* src = reinterpret_cast<const double2*>(dmin + pb);
#pragma unroll
      for (int j = 0; j < kPass / 128; ++j) {
        const double2 v = src[j * 64 + lane];
        const int el = j * 128 + 2 * lane;
        const int pos = el + (el >> 4);
        sb[pos] = v.x;
        sb[pos + 1] = v.y;
      }
    }
    __syncthreads();
    if (act) {
      const int64_t lo = pb + (int64_t)lane * 16;
      const int64_t hi = (lo + 16) < n ? (lo + 16) : n;
      long long D0 = 0, D1 = 0;
      int valid = 1;
      const double* sl = sb + lane * 17;
      if (lo < hi)
        range_transfer_v([&](int64_t i) { return sl[i - lo]; }, S, lo, hi, e, D0, D1, valid);
      // ordered reduction over lanes: lane l absorbs lane l+o
      for (int o = 1; o < 64; o <<= 1) {
        const long long r0 = __shfl_down(D0, o), r1 = __shfl_down(D1, o);
        const int rv = __shfl_down(valid, o);
        if ((lane & (2 * o - 1)) == 0 && lane + o < 64) {
          long long n0, n1;
          compose(D0, D1, r0, r1, n0, n1);
          D0 = n0;
          D1 = n1;
          valid &= rv;
        }
      }
      long long n0, n1;
      compose(T0, T1, D0, D1, n0, n1);
      tv &= valid;
      // saturate: keeps the composition of later passes from overflowing
      if (n0 >= (1ll << 52) || n1 >= (1ll << 52)) {
        tv = 0;
        n0 = n1 = 0;
      }
      T0 = n0;
      T1 = n1;
    }
    __syncthreads();
  }
  if (live && lane == 0) out[b] = Xfer{T0, T1, e, tv, 0};
}

// approx[b] = c_in + sum_{b' < b} blocksums[b'] / S   (guesses only: any
// summation order will do).  Each thread's run of block sums is loaded 8 at a
// time (the loads in flight together), the 1024 partials are scanned by waves
// (shfl) and then across the 16 waves.
__global__ __launch_bounds__(1024) void approx_prefix_kernel(const double* __restrict__ bs,
                                                             int64_t nb, double S, double c_in,
                                                             double* __restrict__ approx,
    SeedDev dv) {
  if (dv.gate && dv.gate[0] != 0.0) return;
  if (dv.S) S = dv.S[0];
  if (dv.c_in) c_in = dv.c_in[0];
  __shared__ double wsum[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t per = (nb + 1023) / 1024;
  const int64_t lo = t * per, hi = (lo + per) < nb ? (lo + per) : nb;
  constexpr int kB = 8;
  double s = 0.0;
  for (int64_t b0 = lo; b0 < hi; b0 += kB) {
    double v[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) v[j] = bs[b0 + j < hi ? b0 + j : lo];
#pragma unroll
    for (int j = 0; j < kB; ++j)
      if (b0 + j < hi) s += v[j] / S;
  }
  double inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  double acc = c_in;
  for (int i = 0; i < w; ++i) acc += wsum[i];
  acc += inc - s;  // the exclusive prefix of this thread's run
  for (int64_t b0 = lo; b0 < hi; b0 += kB) {
    double v[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) v[j] = bs[b0 + j < hi ? b0 + j : lo];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      if (b0 + j < hi) {
        approx[b0 + j] = acc;
        acc += v[j] / S;
      }
    }
  }
}

// Wave-parallel exact walk of elements [lo, hi) starting from running value c.
// If `search`, stops at the first element m with fl(c_m / c_last) > u and
// returns its index in *found (else *found stays -1).  Returns the running
// value after the last element processed.  Executed by all 64 lanes of a
// single-wave workgroup (it synchronises the workgroup).
//
// The range is taken in segments of 4096: p = fl(dmin / S) of the segment is
// staged in LDS (coalesced loads, one pad slot per 64 so that lane l's
// sub-chunk [64 l, 64 l + 64) reads conflict-free), then sub-chunk transfers
// are applied in bulk while they stay in the binade and the sub-chunk that
// leaves it is walked element by element.
constexpr int kSeg = 4096;
constexpr int kSegSub = kSeg / 64;

__device__ double fine_walk(const double* __restrict__ dmin, double S, int64_t lo, int64_t hi,
                            double c, bool search, double c_last, double u, int64_t* found) {
  __shared__ double sp[kSeg + kSeg / kSegSub];
  const int lane = threadIdx.x & 63;
  for (int64_t s0 = lo; s0 < hi; s0 += kSeg) {
    const int m = (int)((hi - s0) < kSeg ? (hi - s0) : kSeg);
    __syncthreads();  // the previous segment's reads are done
    if (m == kSeg && (s0 & 1) == 0) {
      // whole segment: 32 independent 16-byte loads per lane in flight
      // (a rolled load/divide/store loop would pay the full HBM latency per
      // element pair)
      const double2* src = reinterpret_cast<const double2*>(dmin + s0);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double2 v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = src[(h * 16 + j) * 64 + lane];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int i = ((h * 16 + j) * 64 + lane) * 2;
          sp[i + i / kSegSub] = v[j].x / S;
          sp[i + 1 + (i + 1) / kSegSub] = v[j].y / S;
        }
      }
    } else {
      for (int i0 = 0; i0 < m; i0 += 64 * 8) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = i0 + j * 64 + lane;
          v[j] = i < m ? dmin[s0 + i] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = i0 + j * 64 + lane;
          if (i < m) sp[i + i / kSegSub] = v[j] / S;
        }
      }
    }
    __syncthreads();
    auto pv = [&](int i) { return sp[i + i / kSegSub]; };
    int pos = 0;
    while (pos < m) {
      int e;
      long long N;
      const bool inb = binade_of(c, e, N);
      int L = 0;  // sub-chunks applied in bulk
      if (inb) {
        const int slo = pos + lane * kSegSub;
        const int shi = (slo + kSegSub) < m ? (slo + kSegSub) : m;
        long long D0 = 0, D1 = 0;
        int valid = 1;
        if (slo < m)
          range_transfer_v([&](int64_t i) { return pv((int)i); }, 1.0, slo, shi, e, D0, D1,
                           valid);
        else
          valid = 0;
        // inclusive ordered prefix over lanes
        for (int o = 1; o < 64; o <<= 1) {
          const long long l0 = __shfl_up(D0, o), l1 = __shfl_up(D1, o);
          const int lv = __shfl_up(valid, o);
          if (lane >= o) {
            long long n0, n1;
            compose(l0, l1, D0, D1, n0, n1);
            D0 = n0;
            D1 = n1;
            valid &= lv;
          }
        }
        const long long Dq = (N & 1) ? D1 : D0;
        const long long Nend = N + Dq;
        bool ok = valid && slo < m && Dq < (1ll << 52) && Nend < (1ll << 53);
        bool hit = false;
        if (ok && search) hit = (from_binade(e, Nend) / c_last) > u;
        const unsigned long long okm = __ballot(ok && !hit);
        // number of leading lanes that are ok and not yet past the target
        L = (okm == ~0ull) ? 64 : __builtin_ctzll(~okm);
        if (L > 0) {
          const long long DL = __shfl(Dq, L - 1);
          c = from_binade(e, N + DL);
          pos += L * kSegSub;
          if (pos > m) pos = m;
        }
        if (pos >= m) break;
        if (L == 64) continue;  // every sub-chunk applied: next bulk round
      }
      // element-wise over (at most) one sub-chunk; lane 0 computes, broadcasts
      const int ehi = (pos + kSegSub) < m ? (pos + kSegSub) : m;
      double cc = c;
      int hitidx = -1;
      if (lane == 0) {
        for (int i = pos; i < ehi; ++i) {
          cc = cc + pv(i);
          if (search && (cc / c_last) > u) {
            hitidx = i;
            break;
          }
        }
      }
      cc = __shfl(cc, 0);
      hitidx = __shfl(hitidx, 0);
      c = cc;
      if (hitidx >= 0) {
        *found = s0 + hitidx;
        return c;
      }
      pos = ehi;
    }
  }
  return c;
}

// Single wave: exact running value through every block, cend[b] = value after
// block b.  Each round takes the next 64 blocks: the leading run of blocks
// whose transfers apply in the current binade is applied at once (an ordered
// prefix of the transfers), the first block that does not is done alone
// (its transfer if it applies from the new value, else an element walk), and
// the next round starts after it.
constexpr int kXWin = 1024;  // block transfers staged in LDS per window (32 KB)

__global__ __launch_bounds__(64) void walk_kernel(const double* __restrict__ dmin, int64_t n,
                                                  double S, const Xfer* __restrict__ xf,
                                                  int64_t nblocks, double c_in,
                                                  double* __restrict__ cend,
                                                  double* __restrict__ c_out,
                                                  long long* __restrict__ stats,
    SeedDev dv) {
  if (dv.gate && dv.gate[0] != 0.0) return;
  if (dv.S) S = dv.S[0];
  __shared__ Xfer sx[kXWin];
  const int lane = threadIdx.x;
  double c = c_in;
  int64_t dummy = -1;
  int64_t b0 = 0;
  int64_t win0 = -1;  // first block of the staged window
  long long st_rounds = 0, st_single = 0, st_fine = 0, st_fcyc = 0;
  const long long st_t0 = stats ? (long long)clock64() : 0;
  while (b0 < nblocks) {
    const int nb = (int)((nblocks - b0) < 64 ? (nblocks - b0) : 64);
    if (win0 < 0 || b0 + nb > win0 + kXWin) {
      // restage [b0, b0 + kXWin): 16 independent loads per lane in flight
      __syncthreads();
      win0 = b0;
      Xfer v[kXWin / 64];
#pragma unroll
      for (int j = 0; j < kXWin / 64; ++j) {
        const int64_t bb = b0 + j * 64 + lane;
        v[j] = bb < nblocks ? xf[bb] : Xfer{0, 0, 0, 0, 0};
      }
#pragma unroll
      for (int j = 0; j < kXWin / 64; ++j) sx[j * 64 + lane] = v[j];
      __syncthreads();
    }
    const Xfer r = lane < nb ? sx[b0 - win0 + lane] : Xfer{0, 0, 0, 0, 0};
    int e;
    long long N;
    const bool inb = binade_of(c, e, N);
    // inclusive ordered prefix of the round's transfers
    long long D0 = r.d0, D1 = r.d1;
    int valid = (lane < nb) && r.valid && inb && r.e == e;
    for (int o = 1; o < 64; o <<= 1) {
      const long long l0 = __shfl_up(D0, o), l1 = __shfl_up(D1, o);
      const int lv = __shfl_up(valid, o);
      if (lane >= o) {
        long long n0, n1;
        compose(l0, l1, D0, D1, n0, n1);
        D0 = n0;
        D1 = n1;
        valid &= lv;
      }
    }
    const long long Dq = (N & 1) ? D1 : D0;
    const bool ok = inb && valid && Dq < (1ll << 52) && (N + Dq) < (1ll << 53);
    const unsigned long long okm = __ballot(ok);
    int L = (okm == ~0ull) ? 64 : __builtin_ctzll(~okm);
    if (L > nb) L = nb;
    if (L > 0) {
      if (lane < L) cend[b0 + lane] = from_binade(e, N + Dq);
      c = from_binade(e, N + __shfl(Dq, L - 1));
    }
    ++st_rounds;
    if (L == nb) {
      b0 += nb;
      continue;
    }
    ++st_single;
    // block bj alone
    const int64_t bj = b0 + L;
    const Xfer rj = sx[bj - win0];
    int ej;
    long long Nj;
    bool done = false;
    if (binade_of(c, ej, Nj) && rj.valid && rj.e == ej) {
      const long long Dj = (Nj & 1) ? rj.d1 : rj.d0;
      if (Dj < (1ll << 52) && Nj + Dj < (1ll << 53)) {
        c = from_binade(ej, Nj + Dj);
        done = true;
      }
    }
    if (!done) {
      const int64_t lo = bj * kSeedBlock;
      const int64_t hi = (lo + kSeedBlock) < n ? (lo + kSeedBlock) : n;
      const long long tf = stats ? (long long)clock64() : 0;
      c = fine_walk(dmin, S, lo, hi, c, false, 1.0, 0.0, &dummy);
      if (stats) st_fcyc += (long long)clock64() - tf;
      ++st_fine;
    }
    if (lane == 0) cend[bj] = c;
    b0 = bj + 1;
  }
  if (lane == 0) *c_out = c;
  if (stats && lane == 0) {
    stats[0] += st_rounds;
    stats[1] += st_single;
    stats[2] += st_fine;
    stats[3] += st_fcyc;
    stats[4] += (long long)clock64() - st_t0;
  }
}

// Single wave: first local index m with fl(c_m / c_last) > u (or -1).  The
// running values cend are non-decreasing, so hit(b) = fl(cend[b] / c_last) > u
// is monotone in b: a 64-ary search (64 probes per round) finds the first hit
// block, then an exact walk of that block finds the element.
__global__ __launch_bounds__(64) void search_kernel(const double* __restrict__ dmin, int64_t n,
                                                    double S, const double* __restrict__ cend,
                                                    int64_t nblocks, double c_in, double c_last,
                                                    double u, int64_t* __restrict__ result,
    SeedDev dv) {
  if (dv.S) S = dv.S[0];
  if (dv.c_last) c_last = dv.c_last[0];
  if (dv.u) u = dv.u[0];
  if (dv.c_in) c_in = dv.c_in[0];
  const int lane = threadIdx.x;
  // invariant: every block < lo misses, block hi hits (hi == nblocks: none)
  int64_t lo = 0, hi = nblocks;
  while (hi - lo > 0) {
    const int64_t span = hi - lo;
    const int64_t step = (span + 63) / 64;
    const int64_t pb = lo + (int64_t)lane * step;
    const bool probe = pb < hi;
    const bool hit = probe && (cend[pb] / c_last) > u;
    const unsigned long long m = __ballot(hit);
    const unsigned long long pm = __ballot(probe);
    if (step == 1) {
      if (m) hi = lo + __builtin_ctzll(m);
      break;
    }
    // first probing lane that hits: the answer is in (probe[j-1], probe[j]]
    if (m) {
      const int j = __builtin_ctzll(m);
      hi = lo + (int64_t)j * step;
      lo = j > 0 ? lo + (int64_t)(j - 1) * step + 1 : lo;
    } else {
      const int jl = 63 - __builtin_clzll(pm);  // last probe misses
      lo = lo + (int64_t)jl * step + 1;
    }
  }
  const int64_t bstar = hi < nblocks ? hi : -1;
  int64_t found = -1;
  if (bstar >= 0) {
    const double c0 = bstar == 0 ? c_in : cend[bstar - 1];
    const int64_t lo2 = bstar * kSeedBlock;
    const int64_t hi2 = (lo2 + kSeedBlock) < n ? (lo2 + kSeedBlock) : n;
    fine_walk(dmin, S, lo2, hi2, c0, true, c_last, u, &found);
  }
  if (lane == 0) *result = found;
}

// ---- cumulative-sum programs ----------------------------------------------
//
// The exact running value through the shard in three parallel passes and one
// short sequential one, instead of walk_kernel's block-by-block walk (which
// also stays, as the fallback):
//  seg_block_kernel  per block: the binade of every element's running value
//                    is guessed from an approximate prefix (approx[b] plus
//                    in-block sums).  An element whose guessed value stays in
//                    one binade joins the current run (a transfer, as above);
//                    one whose guessed value changes binade is a crossing,
//                    added exactly at evaluation.  The block becomes
//                    run x run x ... run (at most kKC crossings; more, or a
//                    guess that breaks a run, make it opaque: walked element
//                    by element at evaluation).
//  seg_plan_kernel   a segmented scan of the block tails over the blocks
//                    (segments start at blocks with crossings) and the
//                    shard's program: RUN / CROSS / FINE / MARK items, a few
//                    per crossing (~log2(c_last / c_first) of them).
//  seg_eval_kernel   one wave runs the program from the exact c_in.  A RUN
//                    applies when the running value is in its binade and
//                    stays there (N + D < 2^53), the transfer test above; a
//                    failed test is a wrong guess and the scan falls back to
//                    walk_kernel.
//  seg_fill_kernel   cend[b] from the value at the block's segment head and
//                    the scanned transfer.
// A program without FINE items is the shard's exact function c_in -> c_out:
// sharded seeding all-gathers the programs and every rank composes them
// (cdr_seed_program_eval) instead of a rank-ordered chain of scans.

struct Part {
  long long d0, d1;
  int e;   // binade exponent (kNoE when empty)
  int st;  // 0 empty (identity), 1 transfer, 2 broken (the guess cannot hold)
};
constexpr int kNoE = -100000;
constexpr long long kD52 = 1ll << 52;

// cdr_seed_item (include/cdr.h)
struct SeedItem {
  long long d0, d1;
  double p;
  int e;
  int kind;
};
static_assert(sizeof(SeedItem) == sizeof(cdr_seed_item), "cdr_seed_item layout");
enum : int {
  kItRun = CDR_SEED_RUN,
  kItCross = CDR_SEED_CROSS,
  kItConst = CDR_SEED_CONST,
  kItFine = CDR_SEED_FINE,
  kItMark = CDR_SEED_MARK,
  kItEnd = CDR_SEED_END,
  kItSkip = CDR_SEED_SKIP,
  kItBad = CDR_SEED_BAD
};

__host__ __device__ __forceinline__ Part part_empty() { return Part{0, 0, kNoE, 0}; }

// L then R
__host__ __device__ __forceinline__ Part part_compose(const Part& L, const Part& R) {
  if (L.st == 0) return R;
  if (R.st == 0) return L;
  if (L.st != 1 || R.st != 1 || L.e != R.e) return Part{0, 0, L.e, 2};
  Part o{L.d0 + ((L.d0 & 1) ? R.d1 : R.d0), L.d1 + ((L.d1 & 1) ? R.d0 : R.d1), L.e, 1};
  if (o.d0 >= kD52 || o.d1 >= kD52) o.st = 2;
  return o;
}

__host__ __device__ __forceinline__ bool sp_binade(double c, int& e, long long& N) {
  const unsigned long long bits = __builtin_bit_cast(unsigned long long, c);
  const int ef = (int)((bits >> 52) & 0x7FF);
  if (ef == 0 || ef >= 2046 || (bits >> 63)) return false;
  e = ef - 1023;
  N = (long long)((bits & 0xFFFFFFFFFFFFFull) | (1ull << 52));
  return true;
}
__host__ __device__ __forceinline__ double sp_value(int e, long long N) {
  const unsigned long long bits =
      ((unsigned long long)(e + 1023) << 52) | ((unsigned long long)N & 0xFFFFFFFFFFFFFull);
  return __builtin_bit_cast(double, bits);
}

// One RUN / SKIP / BAD / CROSS / CONST item applied to the running value c
// (MARK and END leave it; FINE cannot be applied here).  False: the item does
// not hold for this c (the guessed binade was wrong).
__host__ __device__ __forceinline__ bool item_apply(const SeedItem& it, double& c) {
  switch (it.kind) {
    case kItRun: {
      int e;
      long long N;
      if (!sp_binade(c, e, N) || e != it.e) return false;
      const long long N2 = N + ((N & 1) ? it.d1 : it.d0);
      if (N2 >= (1ll << 53)) return false;
      c = sp_value(e, N2);
      return true;
    }
    case kItSkip:
    case kItMark:
    case kItEnd:
      return true;
    case kItCross:
      c = c + it.p;
      return true;
    case kItConst:
      c = it.p;
      return true;
    default:
      return false;
  }
}

__host__ __device__ __forceinline__ SeedItem run_item(const Part& P) {
  return SeedItem{P.d0, P.d1, 0.0, P.e, P.st == 0 ? kItSkip : (P.st == 1 ? kItRun : kItBad)};
}

// Element p joins run P under binade e (range_transfer_v's step).
__device__ __forceinline__ void part_add(Part& P, double p, int e) {
  if (P.st == 0) P = Part{0, 0, e, 1};
  if (P.st != 1) return;
  if (P.e != e) {
    P.st = 2;
    return;
  }
  const double f = ldexp(p, 52 - e);
  if (!(f < 4503599627370496.0)) {
    P.st = 2;
    return;
  }
  const double fl = floor(f);
  const double frac = f - fl;
  const long long k = (long long)fl;
  const long long up = frac > 0.5 ? 1 : 0;
  const bool tie = frac == 0.5;
  P.d0 += k + up + ((tie && ((P.d0 ^ k) & 1)) ? 1 : 0);
  P.d1 += k + up + ((tie && ((1 ^ P.d1 ^ k) & 1)) ? 1 : 0);
  if (P.d0 >= kD52 || P.d1 >= kD52) P.st = 2;
}

// part_add with the run's counts kept as fp64 integers (exact below 2^53; a
// run stops at 2^52) and their parities as bits: no fp64 -> int64 conversion
// per element (seg_block's loop is VALU-bound); to_part gives the Part that
// part_add would have built from the same elements.
struct PartD {
  double d0, d1;
  int p0, p1;  // parities of d0, d1
  int e, st;
};
__device__ __forceinline__ PartD partd_empty() { return PartD{0.0, 0.0, 0, 0, kNoE, 0}; }
__device__ __forceinline__ void partd_add(PartD& P, double p, int e) {
  if (P.st == 0) P = PartD{0.0, 0.0, 0, 0, e, 1};
  if (P.st != 1) return;
  if (P.e != e) {
    P.st = 2;
    return;
  }
  const double f = ldexp(p, 52 - e);
  if (!(f < 4503599627370496.0)) {
    P.st = 2;
    return;
  }
  const double fl = floor(f);
  const double frac = f - fl;
  // fl < 2^52: in fl + 2^52 the last significand bit is fl's parity
  const int kp = (int)(__double_as_longlong(fl + 4503599627370496.0) & 1);
  const int up = frac > 0.5 ? 1 : 0;
  const int tie = frac == 0.5 ? 1 : 0;
  const int i0 = up | (tie & (P.p0 ^ kp));
  const int i1 = up | (tie & (1 ^ P.p1 ^ kp));
  P.d0 = (P.d0 + fl) + (double)i0;
  P.d1 = (P.d1 + fl) + (double)i1;
  P.p0 ^= kp ^ i0;
  P.p1 ^= kp ^ i1;
  if (P.d0 >= 4503599627370496.0 || P.d1 >= 4503599627370496.0) P.st = 2;
}
__device__ __forceinline__ Part to_part(const PartD& P) {
  return Part{(long long)P.d0, (long long)P.d1, P.e, P.st};
}

__device__ __forceinline__ Part shfl_up_part(const Part& P, int o) {
  return Part{__shfl_up(P.d0, o), __shfl_up(P.d1, o), __shfl_up(P.e, o), __shfl_up(P.st, o)};
}
__device__ __forceinline__ Part shfl_part(const Part& P, int l) {
  return Part{__shfl(P.d0, l), __shfl(P.d1, l), __shfl(P.e, l), __shfl(P.st, l)};
}

__device__ __forceinline__ int gbin(double c) {
  int e;
  long long N;
  return sp_binade(c, e, N) ? e : kNoE;
}

// A guessed running value within 2^-24 (relative) of its binade's edges: the
// exact value may sit on either side (a sequential fp64 sum of n terms is
// within n 2^-53 of the real sum, < 2^-24 for n < 2^29), so elements next to
// it are crossings, added exactly whatever the binade turns out to be.
__device__ __forceinline__ bool gnear(double c) {
  const unsigned long long m = __builtin_bit_cast(unsigned long long, c) & 0xFFFFFFFFFFFFFull;
  return m < (1ull << 28) || m > (1ull << 52) - (1ull << 28);
}

constexpr int kKC = 32;  // crossings recorded per block
struct SegTail {
  Part t;      // the run after the block's last crossing (the whole block: none)
  int ncross;  // crossings in the block
  int opaque;  // walked element by element at evaluation
};
struct SegEnt {
  Part pre;  // the run before the crossing (from the block start or the previous crossing)
  double p;  // the crossing element
};
struct SegScan {
  Part s;        // transfer from the block's segment head (exclusive) through the block
  long long lh;  // segment head block (-1: the shard start)
};

// One workgroup per block, one wave per 1024-element pass (8 waves); lane l
// of wave w owns elements [1024 w + 16 l, +16).  The passes are linked
// through LDS: their sums (the guessed running value at each pass start),
// their crossing counts (where each pass's entries go) and their tail runs
// (the run open at each pass start).
constexpr int kSegWaves = kSeedBlock / kPass;  // 8
__global__ __launch_bounds__(512) void seg_block_kernel(const double* __restrict__ dmin,
                                                        int64_t n, double S,
                                                        const double* __restrict__ approx,
                                                        int64_t nblocks,
                                                        SegTail* __restrict__ tails,
                                                        SegEnt* __restrict__ ents,
    SeedDev dv) {
  if (dv.S) S = dv.S[0];
  __shared__ double s_sum[kSegWaves];
  __shared__ int s_m[kSegWaves], s_bad[kSegWaves], s_h[kSegWaves];
  __shared__ Part s_t[kSegWaves];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t b = blockIdx.x;
  const int64_t base = b * kSeedBlock;
  SegEnt* eb = ents + b * kKC;
  const int64_t lo = base + (int64_t)w * kPass + (int64_t)lane * 16;
  const int cnt = lo >= n ? 0 : (n - lo < 16 ? (int)(n - lo) : 16);
  // dmin is allocated to n_pad (a multiple of the block): whole lanes load
  double p[16];
  {
    const double2* src = reinterpret_cast<const double2*>(dmin + lo);
    double2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = src[j];
    // p = fl(dmin / S) by Markstein's correction from y = fl(1 / S): q0 =
    // fl(a y), r = a - S q0 (exact in one fma), fl(q0 + r y) is the correctly
    // rounded quotient (no underflow: a >= 2^-960, S < 2^1000; others divide).
    // 3 fp64 instructions per element instead of the ~11 of a division
    // (tools/markstein_div_fuzz.cpp: 3.2e8 quotients, none differs).
    const double y = 1.0 / S;
    const bool fastS = S < 0x1p1000;
    auto quo = [&](double a) {
      const double q0 = a * y;
      double q = fma(fma(-q0, S, a), y, q0);
      if (!(fastS && a >= 0x1p-960)) q = a / S;
      return q;
    };
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      p[2 * j] = 2 * j < cnt ? quo(v[j].x) : 0.0;
      p[2 * j + 1] = 2 * j + 1 < cnt ? quo(v[j].y) : 0.0;
    }
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += p[j];
  double inc = s;
  for (int o = 1; o < 64; o <<= 1) {
    const double t = __shfl_up(inc, o);
    if (lane >= o) inc += t;
  }
  if (lane == 63) s_sum[w] = inc;
  __syncthreads();
  // guessed running value at each pass start: the same sequence in every wave
  double A = approx[b], Anext = 0.0;
  for (int v = 0; v <= w; ++v) {
    Anext = A + s_sum[v];
    if (v < w) A = Anext;
  }
  const double Aend = (b + 1 < nblocks) ? approx[b + 1] : -1.0;
  const double ex = __shfl_up(inc, 1);
  const double a0 = A + (lane ? ex : 0.0);
  double a1 = __shfl_down(a0, 1);
  if (lane == 63) a1 = (w == kSegWaves - 1 && Aend >= 0.0) ? Aend : Anext;
  // crossings under the guess
  unsigned xm = 0;
  {
    double cb = a0;
    int gb = gbin(cb);
    bool nb_ = gnear(cb);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < cnt) {
        const double ca = (j == cnt - 1) ? a1 : cb + p[j];
        const int ga = gbin(ca);
        const bool na = gnear(ca);
        if (gb == kNoE || ga != gb || nb_ || na) xm |= 1u << j;
        cb = ca;
        gb = ga;
        nb_ = na;
      }
    }
  }
  const int m = __popc(xm);
  int mi = m;
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(mi, o);
    if (lane >= o) mi += t;
  }
  if (lane == 63) s_m[w] = mi;
  __syncthreads();
  int basew = 0, mtot = 0;
  for (int v = 0; v < kSegWaves; ++v) {
    if (v < w) basew += s_m[v];
    mtot += s_m[v];
  }
  const bool over = mtot > kKC;  // block-uniform
  Part Sx = part_empty();
  Part F = part_empty();
  double p0 = 0.0;
  bool bad = false;
  const int bl = basew + mi - m;  // this lane's first entry
  if (!over) {
    PartD cur = partd_empty();
    int jj = 0;
    double cb = a0;
    int gb = gbin(cb);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < cnt) {
        const double ca = (j == cnt - 1) ? a1 : cb + p[j];
        if ((xm >> j) & 1) {
          if (jj == 0) {
            F = to_part(cur);
            p0 = p[j];
          } else {
            eb[bl + jj] = SegEnt{to_part(cur), p[j]};
            bad |= cur.st == 2;
          }
          ++jj;
          cur = partd_empty();
        } else {
          partd_add(cur, p[j], gb);
        }
        cb = ca;
        gb = gbin(ca);
      }
    }
    // segmented inclusive scan of the lane tails (heads: lanes with a crossing)
    Sx = to_part(cur);
    int hs = m > 0;
    for (int o = 1; o < 64; o <<= 1) {
      const Part L = shfl_up_part(Sx, o);
      const int hl = __shfl_up(hs, o);
      if (lane >= o) {
        if (!hs) Sx = part_compose(L, Sx);
        hs |= hl;
      }
    }
  }
  const unsigned long long hm = __ballot(m > 0);
  const Part S63 = shfl_part(Sx, 63);
  if (lane == 0) {
    s_t[w] = S63;
    s_h[w] = hm != 0ull;
  }
  Part Sp = shfl_up_part(Sx, 1);
  if (lane == 0) Sp = part_empty();
  const int anybad = __ballot(bad) != 0ull;
  if (lane == 0) s_bad[w] = anybad;
  __syncthreads();
  // the run open at this pass's start: passes since the last one with a crossing
  Part open = part_empty();
  for (int v = 0; v < w; ++v) open = s_h[v] ? s_t[v] : part_compose(open, s_t[v]);
  bool badw = false;
  if (!over && m > 0) {
    const bool prevh = (hm & ((1ull << lane) - 1)) != 0;
    const Part pre = part_compose(prevh ? Sp : part_compose(open, Sp), F);
    eb[bl] = SegEnt{pre, p0};
    badw = pre.st == 2;
  }
  const int badf = __ballot(badw) != 0ull;
  __syncthreads();
  if (lane == 0 && badf) s_bad[w] = 1;
  __syncthreads();
  if (threadIdx.x == 0) {
    Part t = part_empty();
    int anyb = 0;
    for (int v = 0; v < kSegWaves; ++v) {
      t = s_h[v] ? s_t[v] : part_compose(t, s_t[v]);
      anyb |= s_bad[v];
    }
    const bool opq = over || anyb || t.st == 2;
    tails[b] = SegTail{t, opq ? 0 : mtot, opq ? 1 : 0};
  }
}

constexpr int kPlanT = 1024;
constexpr int64_t kItemCap = 1 << 16;  // program items per shard (more: fallback)

// Single workgroup: segmented scan of the block tails and the program.
__global__ __launch_bounds__(1024) void seg_plan_kernel(const SegTail* __restrict__ tails,
                                                        const SegEnt* __restrict__ ents,
                                                        int64_t nb, SegScan* __restrict__ scan,
                                                        SeedItem* __restrict__ items, int64_t cap,
                                                        long long* __restrict__ meta) {
  __shared__ Part sP[kPlanT];
  __shared__ int sH[kPlanT];
  __shared__ long long sI[kPlanT], sL[kPlanT], sF[kPlanT];
  const int t = threadIdx.x;
  const int64_t per = (nb + kPlanT - 1) / kPlanT;
  const int64_t lo = (int64_t)t * per;
  const int64_t hi = (lo + per) < nb ? (lo + per) : nb;
  // a thread's tails are loaded kPB at a time, the loads in flight together
  // (one at a time paid a memory latency per block: 60 us at 12 208 blocks)
  constexpr int kPB = 4;
  auto load_tails = [&](int64_t b0, SegTail (&T)[kPB]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kPB; ++j) T[j] = tails[b0 + j < hi ? b0 + j : lo];
  };
  {
    Part agg = part_empty();
    int hh = 0;
    long long ni = 0, lh = -1, nf = 0;
    for (int64_t b0 = lo; b0 < hi; b0 += kPB) {
      SegTail TT[kPB];
      load_tails(b0, TT);
#pragma unroll
      for (int j = 0; j < kPB; ++j) {
        const int64_t b = b0 + j;
        if (b >= hi) break;
        const SegTail& T = TT[j];
        if (T.ncross > 0 || T.opaque) {
          agg = T.opaque ? part_empty() : T.t;
          hh = 1;
          lh = b;
          ni += T.opaque ? 3 : 2 + 2 * (long long)T.ncross;
          nf += T.opaque;
        } else {
          agg = part_compose(agg, T.t);
        }
      }
    }
    sP[t] = agg;
    sH[t] = hh;
    sI[t] = ni;
    sL[t] = lh;
    sF[t] = nf;
  }
  __syncthreads();
  for (int o = 1; o < kPlanT; o <<= 1) {
    Part L = part_empty();
    int hl = 0;
    long long il = 0, ll = -1, fl = 0;
    if (t >= o) {
      L = sP[t - o];
      hl = sH[t - o];
      il = sI[t - o];
      ll = sL[t - o];
      fl = sF[t - o];
    }
    __syncthreads();
    if (t >= o) {
      if (!sH[t]) sP[t] = part_compose(L, sP[t]);
      sH[t] |= hl;
      sI[t] += il;
      if (ll > sL[t]) sL[t] = ll;
      sF[t] += fl;
    }
    __syncthreads();
  }
  Part run = t ? sP[t - 1] : part_empty();
  long long off = t ? sI[t - 1] : 0;
  long long lastH = t ? sL[t - 1] : -1;
  const long long total = sI[kPlanT - 1];
  const bool over = total + 2 > cap;
  for (int64_t b0 = lo; b0 < hi; b0 += kPB) {
    SegTail TT[kPB];
    load_tails(b0, TT);
#pragma unroll
    for (int jb = 0; jb < kPB; ++jb) {
      const int64_t b = b0 + jb;
      if (b >= hi) break;
      const SegTail& T = TT[jb];
      if (T.ncross > 0 || T.opaque) {
        if (!over) {
          items[off++] = run_item(run);
          if (T.opaque) {
            items[off++] = SeedItem{b, 0, 0.0, 0, kItFine};
          } else {
            for (int j = 0; j < T.ncross; ++j) {
              const SegEnt E = ents[b * kKC + j];
              items[off++] = run_item(E.pre);
              items[off++] = SeedItem{0, 0, E.p, 0, kItCross};
            }
          }
          items[off++] = SeedItem{b, 0, 0.0, 0, kItMark};
        }
        run = T.opaque ? part_empty() : T.t;
        lastH = b;
      } else {
        run = part_compose(run, T.t);
      }
      scan[b] = SegScan{run, lastH};
    }
  }
  if (t == 0) {
    if (!over) {
      items[total] = run_item(sP[kPlanT - 1]);
      items[total + 1] = SeedItem{0, 0, 0.0, 0, kItEnd};
    }
    meta[0] = total + 2;
    meta[1] = sF[kPlanT - 1];
    meta[2] = over ? 1 : 0;
  }
}

// Single wave: the program from the exact c_in.  Items are staged through
// LDS a window at a time (one round trip for the whole window); each item's
// fields go to scalar registers (readfirstlane) so the walk over the items is
// uniform scalar control flow with no per-item memory latency.
// res[0] = running value after the shard, res[1] = 1 when every item held.
constexpr int kEvalWin = 256;
__device__ __forceinline__ long long sgpr64(long long v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)v >> 32));
  return (long long)(((unsigned long long)hi << 32) | lo);
}
__global__ __launch_bounds__(64) void seg_eval_kernel(const double* __restrict__ dmin, int64_t n,
                                                      double S,
                                                      const SeedItem* __restrict__ items,
                                                      const long long* __restrict__ meta,
                                                      double c_in, double* __restrict__ markc,
                                                      double* __restrict__ res,
    SeedDev dv) {
  if (dv.S) S = dv.S[0];
  if (dv.c_in) c_in = dv.c_in[0];
  __shared__ SeedItem sit[kEvalWin];
  const int lane = threadIdx.x;
  double c = c_in;
  bool ok = meta[2] == 0;
  const long long cnt = ok ? meta[0] : 0;
  int64_t dummy = -1;
  bool end = false;
  for (long long w0 = 0; ok && !end && w0 < cnt; w0 += kEvalWin) {
    const int m = (int)((cnt - w0) < kEvalWin ? (cnt - w0) : kEvalWin);
    __syncthreads();
    {
      const double4* src = reinterpret_cast<const double4*>(items + w0);
      double4* dst = reinterpret_cast<double4*>(sit);
      double4 v[kEvalWin / 64];
#pragma unroll
      for (int j = 0; j < kEvalWin / 64; ++j)
        if (j * 64 + lane < m) v[j] = src[j * 64 + lane];
#pragma unroll
      for (int j = 0; j < kEvalWin / 64; ++j)
        if (j * 64 + lane < m) dst[j * 64 + lane] = v[j];
    }
    __syncthreads();
    for (int i = 0; i < m; ++i) {
      const int kind = __builtin_amdgcn_readfirstlane(sit[i].kind);
      if (kind == kItEnd) {
        end = true;
        break;
      }
      if (kind == kItFine) {
        const int64_t lo = sgpr64(sit[i].d0) * kSeedBlock;
        const int64_t hi = (lo + kSeedBlock) < n ? (lo + kSeedBlock) : n;
        c = fine_walk(dmin, S, lo, hi, c, false, 1.0, 0.0, &dummy);
      } else if (kind == kItMark) {
        if (lane == 0) markc[sgpr64(sit[i].d0)] = c;
      } else {
        SeedItem it;
        it.kind = kind;
        it.e = __builtin_amdgcn_readfirstlane(sit[i].e);
        it.d0 = sgpr64(sit[i].d0);
        it.d1 = sgpr64(sit[i].d1);
        it.p = __builtin_bit_cast(double, sgpr64(__builtin_bit_cast(long long, sit[i].p)));
        if (!item_apply(it, c)) {
          ok = false;
          break;
        }
      }
    }
  }
  if (lane == 0) {
    res[0] = c;
    res[1] = ok ? 1.0 : 0.0;
  }
}

__global__ __launch_bounds__(256) void seg_fill_kernel(const SegScan* __restrict__ scan,
                                                       int64_t nb,
                                                       const double* __restrict__ markc,
                                                       const double* __restrict__ res,
                                                       double c_in, double* __restrict__ cend,
                                                       const double* __restrict__ c_in_dev) {
  if (res[1] == 0.0) return;
  if (c_in_dev) c_in = c_in_dev[0];
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const SegScan s = scan[b];
  const double c0 = s.lh < 0 ? c_in : markc[s.lh];
  double v = c0;
  if (s.s.st == 1) {
    int e;
    long long N;
    sp_binade(c0, e, N);
    v = sp_value(e, N + ((N & 1) ? s.s.d1 : s.s.d0));
  }
  cend[b] = v;
}

// ---- device-resident seeding (seed_run) -----------------------------------

// The left-to-right sum of v[0 .. n) in one wave (the value in every lane).
// The chain of n dependent fp64 (or fp32) adds is the whole cost, so each add
// takes its operand from LDS (a broadcast read, in order under lgkmcnt) and
// the values arrive in chunks: the wave loads chunk c + 1 into registers
// (coalesced, one value per lane per load) while the chain runs over chunk c,
// then writes it to the other LDS buffer.  (Round 5 read each value through
// two v_readlane into SGPRs: three VALU instructions and a hazard wait per
// add, ~2.5x slower.)  Padding past n adds +0.0, which leaves a sum of
// non-negative terms unchanged.
template <typename T>
__device__ __forceinline__ T wave_seq_sum(const T* __restrict__ v, int64_t n) {
  constexpr int kChunk = 1024;       // values per chunk
  constexpr int kPer = kChunk / 64;  // per lane
  __shared__ __attribute__((aligned(16))) T buf[2][kChunk];
  const int lane = threadIdx.x & 63;
  T r[kPer];
  // lane l holds values c0 + l + 64 j of the chunk at c0 (coalesced; no
  // branches: a clamped address and a select, so the loads stay in flight)
  auto load = [&](int64_t c0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t i = c0 + lane + 64 * j;
      r[j] = v[i < n ? i : n - 1];
    }
  };
  // (the select past n here, after the chain: not at the load, where it
  // would wait for the data)
  auto store = [&](T* dst, int64_t c0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kPer; ++j) dst[lane + 64 * j] = c0 + lane + 64 * j < n ? r[j] : T(0);
  };
  T s = T(0);
  if (n <= 0) return s;
  load(0);
  store(buf[0], 0);
  int cb = 0;
  for (int64_t c0 = 0; c0 < n; c0 += kChunk) {
    const bool more = c0 + kChunk < n;  // (uniform)
    if (more) load(c0 + kChunk);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const T* src = buf[cb];
    const int m = n - c0 < kChunk ? (int)(n - c0) : kChunk;
    if (m == kChunk) {
      // 16-byte reads kP ahead of the chain (the LDS latency covered by the
      // adds of the kP - 1 reads before)
      constexpr int kVec = 16 / sizeof(T);
      constexpr int kNV = kChunk / kVec;
      constexpr int kP = 8;
      typedef T tv __attribute__((ext_vector_type(kVec)));
      const tv* q = reinterpret_cast<const tv*>(src);
      tv pipe[kP];
#pragma unroll
      for (int i = 0; i < kP; ++i) pipe[i] = q[i];
#pragma unroll
      for (int i = 0; i < kNV; ++i) {
        const tv cur = pipe[i % kP];
        if (i + kP < kNV) pipe[i % kP] = q[i + kP];
#pragma unroll
        for (int e = 0; e < kVec; ++e) s = s + cur[e];
      }
    } else {
      for (int j = 0; j < m; ++j) s = s + src[j];
    }
    if (more) store(buf[cb ^ 1], c0 + kChunk);
    cb ^= 1;
  }
  return s;
}

// total = dist_sq.sum() (:18): the block sums added left to right, as the host
// does (cdr_host_seq_sum).  A total that is not finite and positive raises
// "Probabilities contain NaN" on the host at the end; S = 1 keeps the rest of
// the run finite meanwhile.
__global__ __launch_bounds__(64) void seed_total_kernel(const double* __restrict__ bs,
                                                        int64_t nb, double* __restrict__ S,
                                                        double* __restrict__ bad) {
  const double s = wave_seq_sum(bs, nb);
  if (threadIdx.x == 0) {
    const bool ok = s > 0.0 && !isinf(s);
    S[0] = ok ? s : 1.0;
    if (!ok) bad[0] = 1.0;
  }
}

// The picked row (exact as fp64) into the centre slot; a missing pick (-1,
// impossible for a finite total: cdf[-1] == 1 > u) is flagged, row 0 used.
__global__ __launch_bounds__(64) void seed_gather_kernel(const float* __restrict__ x32,
                                                         const double* __restrict__ x64,
                                                         int64_t* __restrict__ pick, int d,
                                                         int64_t n_pad,
                                                         double* __restrict__ out,
                                                         double* __restrict__ bad) {
  int64_t i = pick[0];
  if (i < 0) {
    i = 0;
    if (threadIdx.x == 0) {
      bad[1] = 1.0;
      pick[0] = 0;
    }
  }
  for (int f = threadIdx.x; f < d; f += 64)
    out[f] = x32 ? (double)x32[xidx(x32, f, i, n_pad)] : x64[xidx(x64, f, i, n_pad)];
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static void check_points(const Ctx& c) {
  if (c.mode == 0) CDR_FAIL(CDR_ERR_STATE, "no points loaded");
  if (c.d > 128) CDR_FAIL(CDR_ERR_UNSUPPORTED, "d > 128 is not supported yet");
}

void seed_reset(Ctx& c) {
  check_points(c);
  c.dmin.ensure(sizeof(double) * c.n_pad);
  hipLaunchKernelGGL(fill_inf, dim3(1024), dim3(256), 0, c.stream, c.dmin.as<double>(), c.n_pad);
  HIP_CHECK(hipGetLastError());
  c.seed_near.ensure(sizeof(int32_t) * c.n_pad);
  HIP_CHECK(hipMemsetAsync(c.seed_near.p, 0, sizeof(int32_t) * c.n_pad, c.stream));
  c.seed_count = 0;
  c.seed_scanned = false;
}

// Append the new centre (device copy in seed_scalar) to the centre list and
// compute its distances to the earlier ones (the pruning table).
static void seed_track(Ctx& c) {
  const int d = c.d;
  const size_t need = sizeof(double) * (size_t)(c.seed_count + 1) * d;
  if (c.seed_cents.bytes < need) {
    DevBuf grown;
    grown.ensure(std::max(need, 2 * c.seed_cents.bytes));
    if (c.seed_count > 0)
      HIP_CHECK(hipMemcpyAsync(grown.p, c.seed_cents.p, sizeof(double) * (size_t)c.seed_count * d,
                               hipMemcpyDeviceToDevice, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    c.seed_cents.release();
    c.seed_cents = grown;
    grown.p = nullptr;
    grown.bytes = 0;
  }
  c.seed_ccd.ensure(sizeof(double) * (size_t)(c.seed_count + 1));
  if (c.seed_count > 0)
    hipLaunchKernelGGL(seed_ccd_kernel, dim3((c.seed_count + 255) / 256), dim3(256), 0, c.stream,
                       c.seed_cents.as<double>(), c.seed_count, d, c.seed_scalar.as<double>(),
                       c.seed_ccd.as<double>());
  HIP_CHECK(hipMemcpyAsync(c.seed_cents.as<double>() + (size_t)c.seed_count * d,
                           c.seed_scalar.p, sizeof(double) * d, hipMemcpyDeviceToDevice,
                           c.stream));
}

// NumPy's pairwise tree over m elements (np_pairwise): leaves of <= 128, split
// at n/2 rounded down to a multiple of 8.  Returns the node's height (leaves
// 0); internal nodes are collected as (height, left, right) with leaf ids
// and internal ids (-1 - index into `inner`).
static int pw_layout(int64_t off, int64_t m, std::vector<int>& leaves,
                     std::vector<std::array<int, 3>>& inner, int& id) {
  if (m <= 128) {
    id = (int)leaves.size() / 2;
    leaves.push_back((int)off);
    leaves.push_back((int)m);
    return 0;
  }
  int64_t m2 = m / 2;
  m2 -= m2 % 8;
  int l, r;
  const int hl = pw_layout(off, m2, leaves, inner, l);
  const int hr = pw_layout(off + m2, m - m2, leaves, inner, r);
  const int h = 1 + (hl > hr ? hl : hr);
  inner.push_back({h, l, r});
  id = -(int)inner.size();  // internal node -1 - index
  return h;
}

static void seed_tail_plan(Ctx& c, int64_t m) {
  if (c.seed_tail_m == m) return;
  std::vector<int> leaves;
  std::vector<std::array<int, 3>> inner;
  int root;
  const int H = pw_layout(0, m, leaves, inner, root);
  const int nl = (int)leaves.size() / 2;
  if (nl > kTailLeaves || H > kTailHeights)
    CDR_FAIL(CDR_ERR_UNSUPPORTED, "pairwise tail layout too large");
  // internal nodes in height order; ids: leaves 0..nl-1, internal nl + rank
  std::vector<int> order(inner.size()), rank(inner.size());
  for (size_t i = 0; i < inner.size(); ++i) order[i] = (int)i;
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return inner[a][0] < inner[b][0]; });
  for (size_t r = 0; r < order.size(); ++r) rank[order[r]] = (int)r;
  auto nid = [&](int x) { return x >= 0 ? x : nl + rank[-1 - x]; };
  std::vector<int> plan(leaves);
  std::vector<int> hstart(H + 1, 0);
  for (int h = 1, r = 0; h <= H; ++h) {
    hstart[h - 1] = r;
    while (r < (int)order.size() && inner[order[r]][0] == h) ++r;
    hstart[h] = r;
  }
  plan.insert(plan.end(), hstart.begin(), hstart.end());
  for (int r : order) {
    plan.push_back(nid(inner[r][1]));
    plan.push_back(nid(inner[r][2]));
  }
  c.seed_tail_plan.ensure(sizeof(int) * plan.size());
  HIP_CHECK(hipMemcpy(c.seed_tail_plan.p, plan.data(), sizeof(int) * plan.size(),
                      hipMemcpyHostToDevice));
  c.seed_tail_nleaves = nl;
  c.seed_tail_nheights = H;
  c.seed_tail_m = m;
}

// cen: the new centre on the host, or nullptr when seed_run has already put
// it at the start of c.seed_scalar on the device.
void seed_update(Ctx& c, const double* cen) {
  check_points(c);
  if (!c.dmin.p) seed_reset(c);
  const int64_t nb = c.nblocks();
  c.blocksums.ensure(sizeof(double) * (nb > 0 ? nb : 1));
  c.seed_scalar.ensure(sizeof(double) * (2 * c.d + 8));
  if (cen)
    HIP_CHECK(hipMemcpyAsync(c.seed_scalar.p, cen, sizeof(double) * c.d, hipMemcpyHostToDevice,
                             c.stream));
  if (!c.seed_near.p) {  // dmin from an earlier session without the tracking buffers
    c.seed_near.ensure(sizeof(int32_t) * c.n_pad);
    HIP_CHECK(hipMemsetAsync(c.seed_near.p, 0, sizeof(int32_t) * c.n_pad, c.stream));
  }
  seed_track(c);
  int32_t* near = c.seed_near.as<int32_t>();
  const double* ccd = c.seed_ccd.as<double>();
  const int cidx = c.seed_count;
  if (nb > 0) {
    typedef void (*SeedFn)(const float*, int64_t, int64_t, int, const double*, double*, double*,
                           int32_t*, const double*, int);
#define CDR_SU(D_) seed_update_kernel<float, D_>
    static const SeedFn fns[17] = {CDR_SU(0),  CDR_SU(1),  CDR_SU(2),  CDR_SU(3),  CDR_SU(4),
                                   CDR_SU(5),  CDR_SU(6),  CDR_SU(7),  CDR_SU(8),  CDR_SU(9),
                                   CDR_SU(10), CDR_SU(11), CDR_SU(12), CDR_SU(13), CDR_SU(14),
                                   CDR_SU(15), CDR_SU(16)};
#undef CDR_SU
    const int64_t nfull = c.n / kSeedBlock;
    static const bool no16 = exp_env("CDR_SEED16") && std::atoi(exp_env("CDR_SEED16")) == 0;
    const int d = c.d;
    if (c.mode == CDR_MODE_F32X && (d == 8 || d == 16 || d == 32 || d == 64) && !no16) {
      const int tau = c.sigma + kSeed16Tau;
      const int G = (d + 7) / 8;
      if (!c.seed16_valid) {
        c.seed_x16.ensure(sizeof(uint4) * (size_t)G * c.n_pad);
        c.seed_e16.ensure(sizeof(unsigned short) * c.n_pad);
        c.seed_mu.ensure(sizeof(float) * d);
        HIP_CHECK(hipMemcpyAsync(c.seed_mu.p, c.mu.data(), sizeof(float) * d,
                                 hipMemcpyHostToDevice, c.stream));
        hipLaunchKernelGGL(seed16_pack_kernel, dim3(4096), dim3(256), 0, c.stream,
                           c.x32.as<float>(), c.n, c.n_pad, d, c.seed_mu.as<float>(),
                           std::ldexp(1.0, tau), c.seed_x16.as<uint4>(), c.seed_e16.as<unsigned short>());
        HIP_CHECK(hipGetLastError());
        c.seed16_valid = true;
      }
      // the centre in the copy's coordinates (fp32) and its rounding error
      float* dch = reinterpret_cast<float*>(c.seed_scalar.as<double>() + d + 8);
      float* dEc = dch + d;
      hipLaunchKernelGGL(seed_ch_kernel, dim3(1), dim3(64), 0, c.stream,
                         c.seed_scalar.as<double>(), c.seed_mu.as<float>(), d,
                         std::ldexp(1.0, tau), dch, dEc);
      typedef void (*S16Fn)(const float*, const uint4*, const unsigned short*, int64_t, int64_t,
                            const double*, const float*, const float*, double, double*,
                            double*, int32_t*, const double*, int);
      static const int u16 = exp_env("CDR_SEED16_U") ? std::atoi(exp_env("CDR_SEED16_U")) : 0;
      static const bool pr16 = exp_env("CDR_SEED16_PR") != nullptr;  // A/B: prune at d <= 16
      // the pairwise tree in registers (d = 8, 16; CDR_SEED16_LDS=1: staged in LDS)
      const bool lds16 = exp_env("CDR_SEED16_LDS") && std::atoi(exp_env("CDR_SEED16_LDS"));
      if ((d == 8 || d == 16) && !lds16 && !pr16 && !u16) {
        // the exact path's rows from the row-major copy (built once per point
        // set; the bounded Lloyd screen gathers from it too); CDR_SEED_XA=0:
        // from the quad planes
        const bool xa = !exp_env("CDR_SEED_XA") || std::atoi(exp_env("CDR_SEED_XA"));
        if (xa) ensure_rowmajor(c);
        hipLaunchKernelGGL(d == 8 ? seed_update16c_kernel<8> : seed_update16c_kernel<16>,
                           dim3(nb), dim3(512), 0, c.stream, c.x32.as<float>(),
                           c.seed_x16.as<uint4>(), c.seed_e16.as<unsigned short>(), c.n, c.n_pad,
                           c.seed_scalar.as<double>(), dch, dEc, std::ldexp(1.0, -tau),
                           c.dmin.as<double>(), c.blocksums.as<double>(), near, cidx,
                           xa ? c.xa32.as<float>() : nullptr);
        HIP_CHECK(hipGetLastError());
        if (nb > nfull) {
          seed_tail_plan(c, c.n - nfull * kSeedBlock);
          hipLaunchKernelGGL(seed_tail_sum_kernel, dim3(1), dim3(256), 0, c.stream,
                             c.dmin.as<double>(), nfull, c.seed_tail_plan.as<int>(),
                             c.seed_tail_nleaves, c.seed_tail_nheights, c.blocksums.as<double>());
          HIP_CHECK(hipGetLastError());
        }
        c.seed_count += 1;
        c.seed_scanned = false;
        return;
      }
      const S16Fn f16 = d == 8    ? (pr16 ? seed_update16_kernel<8, 0, true> : seed_update16_kernel<8>)
                        : d == 16 ? (pr16       ? seed_update16_kernel<16, 0, true>
                                     : u16 == 1 ? seed_update16_kernel<16, 1>
                                     : u16 == 4 ? seed_update16_kernel<16, 4>
                                                : seed_update16_kernel<16>)
                        : d == 32 ? seed_update16_kernel<32>
                                  : seed_update16_kernel<64>;
      hipLaunchKernelGGL(f16, dim3(nb), dim3(256), 0, c.stream, c.x32.as<float>(),
                         c.seed_x16.as<uint4>(), c.seed_e16.as<unsigned short>(), c.n, c.n_pad,
                         c.seed_scalar.as<double>(), dch, dEc, std::ldexp(1.0, -tau),
                         c.dmin.as<double>(), c.blocksums.as<double>(), near, ccd, cidx);
      HIP_CHECK(hipGetLastError());
      if (nb > nfull) {
        seed_tail_plan(c, c.n - nfull * kSeedBlock);
        hipLaunchKernelGGL(seed_tail_sum_kernel, dim3(1), dim3(256), 0, c.stream,
                           c.dmin.as<double>(), nfull, c.seed_tail_plan.as<int>(),
                           c.seed_tail_nleaves, c.seed_tail_nheights, c.blocksums.as<double>());
        HIP_CHECK(hipGetLastError());
      }
      c.seed_count += 1;
      c.seed_scanned = false;
      return;
    }
    const SeedFn fn = c.d <= 16 ? fns[c.d]
                      : c.d == 32 ? seed_update_kernel<float, 32>
                      : c.d == 64 ? seed_update_kernel<float, 64>
                                  : fns[0];
    if (c.mode == CDR_MODE_F32X)
      hipLaunchKernelGGL(fn, dim3(nb), dim3(256), 0, c.stream,
                         c.x32.as<float>(), c.n, c.n_pad, c.d, c.seed_scalar.as<double>(),
                         c.dmin.as<double>(), c.blocksums.as<double>(), near, ccd, cidx);
    else
      hipLaunchKernelGGL((seed_update_kernel<double, 0>), dim3(nb), dim3(256), 0, c.stream,
                         c.x64.as<double>(), c.n, c.n_pad, c.d, c.seed_scalar.as<double>(),
                         c.dmin.as<double>(), c.blocksums.as<double>(), near, ccd, cidx);
    HIP_CHECK(hipGetLastError());
    if (nb > nfull) {
      seed_tail_plan(c, c.n - nfull * kSeedBlock);
      hipLaunchKernelGGL(seed_tail_sum_kernel, dim3(1), dim3(256), 0, c.stream,
                         c.dmin.as<double>(), nfull, c.seed_tail_plan.as<int>(),
                         c.seed_tail_nleaves, c.seed_tail_nheights, c.blocksums.as<double>());
      HIP_CHECK(hipGetLastError());
    }
  }
  c.seed_count += 1;
  c.seed_scanned = false;
}

// The block-by-block walk (exact from any c_in; the fallback of the program).
// Device-resident mode (seed_run): dv carries S / gate, the running value at
// the end goes to dres_dev, and nothing is read back (c_out == nullptr).
static void seed_scan_walk(Ctx& c, double total, double c_in, double* c_out,
                           const SeedDev& dv = SeedDev{}, double* dres_dev = nullptr) {
  const int64_t nb = c.nblocks();
  c.xfer.ensure(sizeof(Xfer) * nb);
  c.cend.ensure(sizeof(double) * nb * 2);
  double* approx = c.cend.as<double>() + nb;
  hipLaunchKernelGGL(approx_prefix_kernel, dim3(1), dim3(1024), 0, c.stream,
                     c.blocksums.as<double>(), nb, total, c_in, approx, dv);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(xfer_kernel, dim3((int)ceil_div(nb, 4)), dim3(256), 0, c.stream,
                     c.dmin.as<double>(), c.n, total, approx, nb, c.xfer.as<Xfer>(), dv);
  HIP_CHECK(hipGetLastError());
  c.seed_scalar.ensure(sizeof(double) * (2 * c.d + 8));
  double* dres = dres_dev ? dres_dev : c.seed_scalar.as<double>() + c.d;
  static const bool want_stats = exp_env("CDR_SEED_STATS") != nullptr;
  long long* dstats = nullptr;
  if (want_stats) {
    static long long* ds = nullptr;
    if (!ds) {
      HIP_CHECK(hipMalloc(&ds, 8 * sizeof(long long)));
      HIP_CHECK(hipMemset(ds, 0, 8 * sizeof(long long)));
    }
    dstats = ds;
  }
  hipLaunchKernelGGL(walk_kernel, dim3(1), dim3(64), 0, c.stream, c.dmin.as<double>(), c.n,
                     total, c.xfer.as<Xfer>(), nb, c_in, c.cend.as<double>(), dres, dstats, dv);
  if (!c_out) {
    HIP_CHECK(hipGetLastError());
    return;
  }
  if (want_stats) {
    long long hs[8];
    HIP_CHECK(hipMemcpyAsync(hs, dstats, sizeof(hs), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    fprintf(stderr,
            "seed walk stats (cumulative): rounds %lld single %lld fine %lld nb %lld "
            "fine_cycles %lld total_cycles %lld\n",
            hs[0], hs[1], hs[2], (long long)nb, hs[3], hs[4]);
  }
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(c_out, dres, sizeof(double), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.seed_c_in = c_in;
  c.seed_total = total;
  c.seed_scanned = true;
}

// This shard's cumsum program under the guess c_guess of the running value at
// its first element (seg_block_kernel, seg_plan_kernel).
static void seed_scan_program(Ctx& c, double total, double c_guess,
                              const SeedDev& dv = SeedDev{}) {
  const int64_t nb = c.nblocks();
  c.cend.ensure(sizeof(double) * nb * 2);
  double* approx = c.cend.as<double>() + nb;
  c.seg_tails.ensure(sizeof(SegTail) * nb);
  c.seg_ents.ensure(sizeof(SegEnt) * nb * kKC);
  c.seg_scan.ensure(sizeof(SegScan) * nb);
  c.seg_items.ensure(sizeof(SeedItem) * kItemCap);
  c.seg_meta.ensure(sizeof(long long) * 8);
  SeedDev dvs;  // the program is always built (no gate)
  dvs.S = dv.S;
  dvs.c_in = dv.c_in;
  hipLaunchKernelGGL(approx_prefix_kernel, dim3(1), dim3(1024), 0, c.stream,
                     c.blocksums.as<double>(), nb, total, c_guess, approx, dvs);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(seg_block_kernel, dim3((int)nb), dim3(kSegWaves * 64), 0, c.stream,
                     c.dmin.as<double>(), c.n, total, approx, nb, c.seg_tails.as<SegTail>(),
                     c.seg_ents.as<SegEnt>(), dvs);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(seg_plan_kernel, dim3(1), dim3(kPlanT), 0, c.stream,
                     c.seg_tails.as<SegTail>(), c.seg_ents.as<SegEnt>(), nb,
                     c.seg_scan.as<SegScan>(), c.seg_items.as<SeedItem>(), kItemCap,
                     c.seg_meta.as<long long>());
  HIP_CHECK(hipGetLastError());
  c.seed_prog_total = total;
  c.seed_prog_ready = true;
  ++c.seed_programs;
}

// Runs the program from the exact c_in and fills cend; false when a guess
// failed (nothing usable written).
// Device-resident mode: c_out == nullptr, nothing is read back (res[0] the
// running value, res[1] the success flag stay on the device).
static double* seed_res(Ctx& c) {
  return reinterpret_cast<double*>(c.seg_meta.as<long long>() + 4);
}
static bool seed_scan_finish(Ctx& c, double c_in, double* c_out,
                             const SeedDev& dv = SeedDev{}) {
  const int64_t nb = c.nblocks();
  double* markc = c.cend.as<double>() + nb;  // the guesses are consumed
  double* res = seed_res(c);
  SeedDev dvs;
  dvs.S = dv.S;
  dvs.c_in = dv.c_in;
  hipLaunchKernelGGL(seg_eval_kernel, dim3(1), dim3(64), 0, c.stream, c.dmin.as<double>(), c.n,
                     c.seed_prog_total, c.seg_items.as<SeedItem>(), c.seg_meta.as<long long>(),
                     c_in, markc, res, dvs);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(seg_fill_kernel, dim3((int)ceil_div(nb, 256)), dim3(256), 0, c.stream,
                     c.seg_scan.as<SegScan>(), nb, markc, res, c_in, c.cend.as<double>(), dv.c_in);
  HIP_CHECK(hipGetLastError());
  if (!c_out) return true;
  double h[2];
  HIP_CHECK(hipMemcpyAsync(h, res, sizeof(h), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  static const bool want_stats = exp_env("CDR_SEED_STATS") != nullptr;
  if (want_stats) {
    long long m[3];
    HIP_CHECK(hipMemcpy(m, c.seg_meta.p, sizeof(m), hipMemcpyDeviceToHost));
    fprintf(stderr, "seed program: items %lld fine %lld over %lld ok %d\n", m[0], m[1], m[2],
            h[1] != 0.0);
  }
  if (h[1] == 0.0) return false;
  *c_out = h[0];
  return true;
}

static void seed_scan_done(Ctx& c, double total, double c_in) {
  c.seed_c_in = c_in;
  c.seed_total = total;
  c.seed_scanned = true;
  c.seed_prog_ready = false;
}

void seed_scan(Ctx& c, double total, double c_in, double* c_out) {
  check_points(c);
  const int64_t nb = c.nblocks();
  if (nb == 0) {
    *c_out = c_in;
    return;
  }
  static const bool walk_only = exp_env("CDR_SEED_WALK") != nullptr;
  bool done = false;
  if (!walk_only) {
    seed_scan_program(c, total, c_in);
    done = seed_scan_finish(c, c_in, c_out);
    if (!done) ++c.seed_fallbacks;
  }
  if (!done) seed_scan_walk(c, total, c_in, c_out);
  seed_scan_done(c, total, c_in);
}

void seed_scan_begin(Ctx& c, double total, double c_guess, int64_t* n_items, int64_t* n_fine) {
  check_points(c);
  const int64_t nb = c.nblocks();
  c.seed_scanned = false;
  if (nb == 0) {
    *n_items = 0;
    *n_fine = 0;
    c.seed_prog_total = total;
    c.seed_prog_ready = true;
    return;
  }
  seed_scan_program(c, total, c_guess);
  long long m[3];
  HIP_CHECK(hipMemcpyAsync(m, c.seg_meta.p, sizeof(m), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  *n_items = m[2] ? -1 : m[0];
  *n_fine = m[1];
}

void seed_scan_items(Ctx& c, cdr_seed_item* out, int64_t cap, int64_t* n_items) {
  if (!c.seed_prog_ready) CDR_FAIL(CDR_ERR_STATE, "cdr_seed_scan_items before cdr_seed_scan_begin");
  const int64_t nb = c.nblocks();
  if (nb == 0) {
    *n_items = 0;
    return;
  }
  long long m[3];
  HIP_CHECK(hipMemcpyAsync(m, c.seg_meta.p, sizeof(m), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  if (m[2]) CDR_FAIL(CDR_ERR_UNSUPPORTED, "seed program over its item capacity");
  if (m[0] > cap) CDR_FAIL(CDR_ERR_ARG, "output capacity below the program's item count");
  HIP_CHECK(hipMemcpyAsync(out, c.seg_items.p, sizeof(SeedItem) * m[0], hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  *n_items = m[0];
}

void seed_scan_end(Ctx& c, double c_in, double* c_out) {
  if (!c.seed_prog_ready) CDR_FAIL(CDR_ERR_STATE, "cdr_seed_scan_end before cdr_seed_scan_begin");
  const double total = c.seed_prog_total;
  const int64_t nb = c.nblocks();
  if (nb == 0) {
    *c_out = c_in;
  } else if (!seed_scan_finish(c, c_in, c_out)) {
    ++c.seed_fallbacks;
    seed_scan_walk(c, total, c_in, c_out);
  }
  seed_scan_done(c, total, c_in);
}

void seed_search(Ctx& c, double c_last, double u, int64_t* idx) {
  check_points(c);
  if (!c.seed_scanned) CDR_FAIL(CDR_ERR_STATE, "cdr_seed_search before cdr_seed_scan");
  const int64_t nb = c.nblocks();
  if (nb == 0) {
    *idx = -1;
    return;
  }
  c.seed_scalar.ensure(sizeof(double) * (c.d + 8));
  int64_t* dres = reinterpret_cast<int64_t*>(c.seed_scalar.as<double>() + c.d + 1);
  hipLaunchKernelGGL(search_kernel, dim3(1), dim3(64), 0, c.stream, c.dmin.as<double>(), c.n,
                     c.seed_total, c.cend.as<double>(), nb, c.seed_c_in, c_last, u, dres,
                     SeedDev{});
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(idx, dres, sizeof(int64_t), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
}

// kmeans_plusplus_init (:3-22) on one shard with no host round trip per step:
// every step's centre, total, cumsum program (with its fallback gated on the
// device), draw and pick stay on the device; picks[0] = first, picks[1..k) the
// drawn rows; u[0..k-1) the host's rng.random() draws in order.
void seed_run(Ctx& c, int64_t first, int k, const double* u, int64_t* picks) {
  check_points(c);
  if (k < 1) CDR_FAIL(CDR_ERR_ARG, "k >= 1");
  if (first < 0 || first >= c.n) CDR_FAIL(CDR_ERR_ARG, "first row out of range");
  picks[0] = first;
  if (k == 1) return;
  const int64_t nb = c.nblocks();
  // [u: k-1][picks: k][S][bad x2][pad]
  const size_t words = (size_t)(k - 1) + (size_t)k + 8;
  c.seed_run_buf.ensure(sizeof(double) * words);
  double* du = c.seed_run_buf.as<double>();
  int64_t* dpick = reinterpret_cast<int64_t*>(du + (k - 1));
  double* dS = du + (k - 1) + k;
  double* dbad = dS + 1;
  HIP_CHECK(hipMemcpyAsync(du, u, sizeof(double) * (k - 1), hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipMemcpyAsync(dpick, &first, sizeof(int64_t), hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipMemsetAsync(dbad, 0, sizeof(double) * 2, c.stream));
  seed_reset(c);
  c.seed_scalar.ensure(sizeof(double) * (2 * c.d + 8));
  c.cend.ensure(sizeof(double) * nb * 2);
  c.seg_meta.ensure(sizeof(long long) * 8);
  static const bool walk_only = exp_env("CDR_SEED_WALK") != nullptr;
  const float* x32 = c.mode == CDR_MODE_F32X ? c.x32.as<float>() : nullptr;
  const double* x64 = c.mode == CDR_MODE_F64 ? c.x64.as<double>() : nullptr;
  for (int i = 1; i < k; ++i) {
    hipLaunchKernelGGL(seed_gather_kernel, dim3(1), dim3(64), 0, c.stream, x32, x64,
                       dpick + (i - 1), c.d, c.n_pad, c.seed_scalar.as<double>(), dbad);
    HIP_CHECK(hipGetLastError());
    seed_update(c, nullptr);
    hipLaunchKernelGGL(seed_total_kernel, dim3(1), dim3(64), 0, c.stream,
                       c.blocksums.as<double>(), nb, dS, dbad);
    HIP_CHECK(hipGetLastError());
    double* res = seed_res(c);
    SeedDev dv;
    dv.S = dS;
    if (!walk_only) {
      seed_scan_program(c, 1.0, 0.0, dv);
      seed_scan_finish(c, 0.0, nullptr, dv);
      dv.gate = res + 1;  // the fallback runs only when the program failed
    } else {
      HIP_CHECK(hipMemsetAsync(res, 0, sizeof(double) * 2, c.stream));
    }
    seed_scan_walk(c, 1.0, 0.0, nullptr, dv, res);
    SeedDev ds;
    ds.S = dS;
    ds.c_last = res;
    ds.u = du + (i - 1);
    hipLaunchKernelGGL(search_kernel, dim3(1), dim3(64), 0, c.stream, c.dmin.as<double>(), c.n,
                       1.0, c.cend.as<double>(), nb, 0.0, 1.0, 0.5, dpick + i, ds);
    HIP_CHECK(hipGetLastError());
  }
  double bad[2];
  HIP_CHECK(hipMemcpyAsync(picks, dpick, sizeof(int64_t) * k, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(bad, dbad, sizeof(bad), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.seed_scanned = false;
  c.seed_prog_ready = false;
  if (bad[0] != 0.0) CDR_FAIL(CDR_ERR_NAN, "Probabilities contain NaN");
  if (bad[1] != 0.0) CDR_FAIL(CDR_ERR_STATE, "k-means++ sampler found no index");
}

// ---- device-resident seeding over sharded rows ------------------------------
//
// kmeans_plusplus_init (:3-22) with the rows sharded over nranks ranks (whole
// 8192-row blocks each, so every shard block is a global block) and no host
// round trip per step.  One step = three phases with a collective after each:
//   phase 0: the previous pick's row (from the SUM all-reduce: its owner sent
//            it, every other rank zeros) becomes the new centre; dmin update;
//            this shard's block sums into its slot of [nranks][nbmax]
//            -> all-gather
//   phase 1: the total = every global block sum left to right (zero padding
//            adds nothing), exactly the host's dist_sq.sum(); this shard's
//            cumsum program from a guessed start (the earlier shards' sums /
//            total), packed into its slot of [nranks][kShardProgCap] items
//            -> all-gather
//   phase 2: every rank composes the programs in rank order (its exact start
//            c_mine and the global c_last), runs its own program from c_mine
//            (checked against the composition), searches u c_last in its
//            shard and sends {row, global index + 1, flags} if it holds the
//            pick, zeros otherwise
//            -> SUM all-reduce
// The steps' picks stay on the device; one readback at the end.  A program
// that cannot be composed (over capacity, opaque blocks, a wrong guess) or a
// program / scan mismatch on any rank sets a flag that every rank sees in the
// all-reduce; the host then runs the host protocol instead (cdr_dist.py).
constexpr int kShardProgCap = 1024;  // program items per rank (item 0: the header)
constexpr int kShardRed = 4;         // red buffer: row (d) | index + 1 | fail | nan | pad
enum : int { kSsS = 0, kSsGuess, kSsMine, kSsAfter, kSsLast, kSsFail, kSsNan, kSsNoHit, kSsWords };

// phase 0: the centre (and the previous pick) from the all-reduced buffer
__global__ __launch_bounds__(64) void shard_center_kernel(const double* __restrict__ red, int d,
                                                          double* __restrict__ centre,
                                                          int64_t* __restrict__ pick,
                                                          double* __restrict__ sc) {
  for (int f = threadIdx.x; f < d; f += 64) centre[f] = red[f];
  if (threadIdx.x == 0) {
    const double g1 = red[d];  // global index + 1 (0: nobody held it)
    pick[0] = g1 >= 1.0 ? (int64_t)g1 - 1 : 0;
    if (!(g1 >= 1.0)) sc[kSsNoHit] = 1.0;
    if (red[d + 1] != 0.0) sc[kSsFail] = 1.0;
    if (red[d + 2] != 0.0) sc[kSsNan] = 1.0;
  }
}

// this shard's block sums into its slot, zero padded to nbmax
__global__ __launch_bounds__(256) void shard_bs_kernel(const double* __restrict__ bs, int64_t nb,
                                                       int64_t nbmax, double* __restrict__ out) {
  for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < nbmax; b += (int64_t)gridDim.x * 256)
    out[b] = b < nb ? bs[b] : 0.0;
}

// phase 1: the guessed start of this shard (earlier shards' sums / total;
// any order: only a guess) — exactly 0 on rank 0
__global__ __launch_bounds__(256) void shard_guess_kernel(const double* __restrict__ gbs,
                                                          int64_t before,
                                                          double* __restrict__ sc) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < before; i += 256) s += gbs[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) sc[kSsGuess] = before ? red[0] / sc[kSsS] : 0.0;
}

// this shard's program into its slot: item 0 = {count, 0, 0, 0, 0} (count -1
// when it cannot be composed elsewhere: over capacity or opaque blocks)
__global__ __launch_bounds__(256) void shard_pack_kernel(const SeedItem* __restrict__ items,
                                                         const long long* __restrict__ meta,
                                                         SeedItem* __restrict__ out) {
  const long long cnt = meta[0];
  const bool ok = meta[2] == 0 && meta[1] == 0 && cnt <= kShardProgCap - 1;
  if (threadIdx.x == 0) out[0] = SeedItem{ok ? cnt : -1, 0, 0.0, 0, kItSkip};
  if (!ok) return;
  for (long long i = threadIdx.x; i < cnt; i += 256) out[1 + i] = items[i];
}

// phase 2: compose every rank's program in rank order from 0 (one wave; a
// rank's items staged in LDS, then walked in scalar registers)
__global__ __launch_bounds__(64) void shard_compose_kernel(const SeedItem* __restrict__ progs,
                                                           int nranks, int rank,
                                                           double* __restrict__ sc) {
  __shared__ SeedItem sit[kShardProgCap];
  const int lane = threadIdx.x;
  double c = 0.0, mine = 0.0, after = 0.0;
  bool ok = sc[kSsFail] == 0.0;
  for (int r = 0; r < nranks && ok; ++r) {
    const SeedItem* P = progs + (size_t)r * kShardProgCap;
    const long long cnt = sgpr64(P[0].d0);
    if (cnt < 0) {
      ok = false;
      break;
    }
    __syncthreads();
    for (long long i = lane; i < cnt; i += 64) sit[i] = P[1 + i];
    __syncthreads();
    if (r == rank) mine = c;
    for (long long i = 0; i < cnt; ++i) {
      SeedItem it;
      it.kind = __builtin_amdgcn_readfirstlane(sit[i].kind);
      if (it.kind == kItEnd) break;
      it.e = __builtin_amdgcn_readfirstlane(sit[i].e);
      it.d0 = sgpr64(sit[i].d0);
      it.d1 = sgpr64(sit[i].d1);
      it.p = __builtin_bit_cast(double, sgpr64(__builtin_bit_cast(long long, sit[i].p)));
      if (!item_apply(it, c)) {
        ok = false;
        break;
      }
    }
    if (r == rank) after = c;
  }
  if (lane == 0) {
    sc[kSsMine] = mine;
    sc[kSsAfter] = after;
    sc[kSsLast] = c;
    if (!ok) sc[kSsFail] = 1.0;
  }
}

// phase 2 end: this rank's part of the SUM all-reduce — the picked row, its
// global index + 1 and the flags (own program vs the composition, a failed
// composition, a bad total) when it holds the pick or sees a problem
__global__ __launch_bounds__(64) void shard_red_kernel(const float* __restrict__ x32,
                                                       const double* __restrict__ x64,
                                                       const int64_t* __restrict__ hit, int d,
                                                       int64_t n_pad, int64_t row_begin,
                                                       const double* __restrict__ res,
                                                       const double* __restrict__ bad,
                                                       const double* __restrict__ sc, int rank,
                                                       const double* __restrict__ u,
                                                       double* __restrict__ red) {
  // the shard's search gives its first element whose running value exceeds
  // u c_last; when that is its first element, the pick belongs to this shard
  // only if the running value before it (the shard start) does not already
  // exceed it — else an earlier shard holds the pick (searchsorted 'right')
  int64_t i = hit[0];
  if (i == 0 && u && sc[kSsMine] / sc[kSsLast] > u[0]) i = -1;
  for (int f = threadIdx.x; f < d; f += 64)
    red[f] = i < 0 ? 0.0 : x32 ? (double)x32[xidx(x32, f, i, n_pad)] : x64[xidx(x64, f, i, n_pad)];
  if (threadIdx.x == 0) {
    red[d] = i < 0 ? 0.0 : (double)(row_begin + i + 1);
    // own program run from the composed start must end where the composition did
    const bool mism = res[1] == 0.0 || res[0] != sc[kSsAfter];
    red[d + 1] = (sc[kSsFail] != 0.0 || mism) ? 1.0 : 0.0;
    red[d + 2] = (rank == 0 && bad[0] != 0.0) ? 1.0 : 0.0;
    red[d + 3] = 0.0;
  }
}

static void ss_require(const Ctx& c) {
  if (!c.ss_on) CDR_FAIL(CDR_ERR_STATE, "cdr_seed_shard_begin first");
}
static double* ss_sc(Ctx& c) {
  return c.ss_buf.as<double>() + (c.ss_k - 1) + c.ss_k;
}

// Sizes of the exchanged buffers (in bytes per rank): block sums, programs,
// the all-reduced record.
static void ss_sizes(const Ctx& c, int64_t* sizes) {
  sizes[0] = (int64_t)sizeof(double) * c.ss_nbmax;
  sizes[1] = (int64_t)sizeof(SeedItem) * kShardProgCap;
  sizes[2] = (int64_t)sizeof(double) * (c.d + kShardRed);
}

void seed_shard_begin(Ctx& c, int64_t row_begin, int64_t n_total, int nranks, int rank,
                      int64_t first, int k, const double* u, double* red_out, int64_t* sizes) {
  check_points(c);
  if (k < 1 || nranks < 1 || rank < 0 || rank >= nranks) CDR_FAIL(CDR_ERR_ARG, "bad k / ranks");
  if (first < 0 || first >= n_total) CDR_FAIL(CDR_ERR_ARG, "first row out of range");
  if (row_begin % kSeedBlock != 0 && c.n > 0)
    CDR_FAIL(CDR_ERR_ARG, "shards must start on an 8192-row block");
  c.ss_row_begin = row_begin;
  c.ss_n_total = n_total;
  c.ss_nranks = nranks;
  c.ss_rank = rank;
  c.ss_k = k;
  c.ss_step = 1;
  // every shard but the last holds whole blocks: nbmax = the first shard's
  c.ss_nbmax = ceil_div(ceil_div(n_total, kSeedBlock), nranks);
  if (c.nblocks() > c.ss_nbmax) CDR_FAIL(CDR_ERR_ARG, "shard larger than n_total / nranks blocks");
  const size_t words = (size_t)(k - 1) + (size_t)k + kSsWords + 8;
  c.ss_buf.ensure(sizeof(double) * words);
  double* du = c.ss_buf.as<double>();
  if (k > 1)
    HIP_CHECK(hipMemcpyAsync(du, u, sizeof(double) * (k - 1), hipMemcpyHostToDevice, c.stream));
  double* sc = du + (k - 1) + k;
  HIP_CHECK(hipMemsetAsync(sc, 0, sizeof(double) * (kSsWords + 8), c.stream));
  seed_reset(c);
  c.seed_scalar.ensure(sizeof(double) * (2 * c.d + 8));
  c.cend.ensure(sizeof(double) * (c.nblocks() > 0 ? c.nblocks() : 1) * 2);
  c.seg_meta.ensure(sizeof(long long) * 8);
  c.ss_on = true;
  ss_sizes(c, sizes);
  // the first centre: its owner sends the row (the red buffer after the SUM)
  int64_t hit = first - row_begin;
  if (hit < 0 || hit >= c.n) hit = -1;
  c.seed_run_buf.ensure(sizeof(double) * 8);
  int64_t* dhit = reinterpret_cast<int64_t*>(c.seed_run_buf.as<double>());
  double* zres = c.seed_run_buf.as<double>() + 2;  // {c_after, ok}: no mismatch
  HIP_CHECK(hipMemcpyAsync(dhit, &hit, sizeof(hit), hipMemcpyHostToDevice, c.stream));
  const double zr[4] = {0.0, 1.0, 0.0, 0.0};
  HIP_CHECK(hipMemcpyAsync(zres, zr, sizeof(zr), hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(shard_red_kernel, dim3(1), dim3(64), 0, c.stream,
                     c.mode == CDR_MODE_F32X ? c.x32.as<float>() : nullptr,
                     c.mode == CDR_MODE_F64 ? c.x64.as<double>() : nullptr, dhit, c.d, c.n_pad,
                     row_begin, zres, zres + 2, sc, rank, nullptr, red_out);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipStreamSynchronize(c.stream));  // hit and zr live on this stack
}

// phase p of the current step (see above); in / out: device buffers
void seed_shard_phase(Ctx& c, int phase, const void* in, void* out) {
  ss_require(c);
  if (c.ss_step >= c.ss_k) CDR_FAIL(CDR_ERR_STATE, "seeding: every step done");
  const int d = c.d, rank = c.ss_rank;
  const int64_t nb = c.nblocks();
  double* du = c.ss_buf.as<double>();
  int64_t* dpick = reinterpret_cast<int64_t*>(du + (c.ss_k - 1));
  double* sc = ss_sc(c);
  if (phase == 0) {
    hipLaunchKernelGGL(shard_center_kernel, dim3(1), dim3(64), 0, c.stream,
                       static_cast<const double*>(in), d, c.seed_scalar.as<double>(),
                       dpick + (c.ss_step - 1), sc);
    HIP_CHECK(hipGetLastError());
    seed_update(c, nullptr);
    double* slot = static_cast<double*>(out) + (size_t)rank * c.ss_nbmax;
    if (nb > 0)
      hipLaunchKernelGGL(shard_bs_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(c.ss_nbmax, 256), 1024)),
                         dim3(256), 0, c.stream, c.blocksums.as<double>(), nb, c.ss_nbmax, slot);
    else
      HIP_CHECK(hipMemsetAsync(slot, 0, sizeof(double) * c.ss_nbmax, c.stream));
    HIP_CHECK(hipGetLastError());
  } else if (phase == 1) {
    const double* gbs = static_cast<const double*>(in);
    double* bad = sc + kSsWords;  // {bad total, no index}
    hipLaunchKernelGGL(seed_total_kernel, dim3(1), dim3(64), 0, c.stream, gbs,
                       (int64_t)c.ss_nranks * c.ss_nbmax, sc + kSsS, bad);
    hipLaunchKernelGGL(shard_guess_kernel, dim3(1), dim3(256), 0, c.stream, gbs,
                       (int64_t)rank * c.ss_nbmax, sc);
    HIP_CHECK(hipGetLastError());
    SeedItem* slot = static_cast<SeedItem*>(out) + (size_t)rank * kShardProgCap;
    if (nb > 0) {
      SeedDev dv;
      dv.S = sc + kSsS;
      dv.c_in = sc + kSsGuess;
      seed_scan_program(c, 1.0, 0.0, dv);
      hipLaunchKernelGGL(shard_pack_kernel, dim3(1), dim3(256), 0, c.stream,
                         c.seg_items.as<SeedItem>(), c.seg_meta.as<long long>(), slot);
    } else {  // an empty shard: the identity program
      const SeedItem hdr[2] = {SeedItem{1, 0, 0.0, 0, kItSkip}, SeedItem{0, 0, 0.0, 0, kItEnd}};
      HIP_CHECK(hipMemcpyAsync(slot, hdr, sizeof(hdr), hipMemcpyHostToDevice, c.stream));
      HIP_CHECK(hipStreamSynchronize(c.stream));
    }
    HIP_CHECK(hipGetLastError());
  } else if (phase == 2) {
    hipLaunchKernelGGL(shard_compose_kernel, dim3(1), dim3(64), 0, c.stream,
                       static_cast<const SeedItem*>(in), c.ss_nranks, rank, sc);
    HIP_CHECK(hipGetLastError());
    double* res = seed_res(c);
    c.seed_run_buf.ensure(sizeof(double) * 8);
    int64_t* dhit = reinterpret_cast<int64_t*>(c.seed_run_buf.as<double>());
    if (nb > 0) {
      SeedDev dv;
      dv.S = sc + kSsS;
      dv.c_in = sc + kSsMine;
      seed_scan_finish(c, 0.0, nullptr, dv);
      SeedDev ds;
      ds.S = sc + kSsS;
      ds.c_last = sc + kSsLast;
      ds.u = du + (c.ss_step - 1);
      ds.c_in = sc + kSsMine;
      hipLaunchKernelGGL(search_kernel, dim3(1), dim3(64), 0, c.stream, c.dmin.as<double>(), c.n,
                         1.0, c.cend.as<double>(), nb, 0.0, 1.0, 0.5, dhit, ds);
    } else {
      const int64_t none = -1;
      HIP_CHECK(hipMemcpyAsync(dhit, &none, sizeof(none), hipMemcpyHostToDevice, c.stream));
      // (no own program: the composition's "after" is the start itself)
      HIP_CHECK(hipMemcpyAsync(res, sc + kSsAfter, sizeof(double), hipMemcpyDeviceToDevice,
                               c.stream));
      const double one = 1.0;
      HIP_CHECK(hipMemcpyAsync(res + 1, &one, sizeof(one), hipMemcpyHostToDevice, c.stream));
      HIP_CHECK(hipStreamSynchronize(c.stream));
    }
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(shard_red_kernel, dim3(1), dim3(64), 0, c.stream,
                       c.mode == CDR_MODE_F32X ? c.x32.as<float>() : nullptr,
                       c.mode == CDR_MODE_F64 ? c.x64.as<double>() : nullptr, dhit, d, c.n_pad,
                       c.ss_row_begin, res, sc + kSsWords, sc, rank, du + (c.ss_step - 1),
                       static_cast<double*>(out));
    HIP_CHECK(hipGetLastError());
    c.ss_step += 1;
  } else {
    CDR_FAIL(CDR_ERR_ARG, "phase 0, 1 or 2");
  }
}

// The last step's pick from the final all-reduced buffer; picks (k global row
// indices) and the status: 0 ok, 1 the host protocol must redo the seeding
// (a program could not be composed or disagreed with its scan), 2 a total
// was not finite and positive (Probabilities contain NaN).
void seed_shard_end(Ctx& c, const double* red, int64_t* picks, double* cents, int32_t* status) {
  ss_require(c);
  if (c.ss_step != c.ss_k) CDR_FAIL(CDR_ERR_STATE, "seeding: steps left");
  double* du = c.ss_buf.as<double>();
  int64_t* dpick = reinterpret_cast<int64_t*>(du + (c.ss_k - 1));
  double* sc = ss_sc(c);
  hipLaunchKernelGGL(shard_center_kernel, dim3(1), dim3(64), 0, c.stream, red, c.d,
                     c.seed_scalar.as<double>(), dpick + (c.ss_k - 1), sc);
  HIP_CHECK(hipGetLastError());
  double flags[kSsWords];
  HIP_CHECK(hipMemcpyAsync(picks, dpick, sizeof(int64_t) * c.ss_k, hipMemcpyDeviceToHost, c.stream));
  // the centres: the k - 1 the updates used (seed_track's list, in order) and
  // the last pick's row (just written to seed_scalar)
  const size_t d = (size_t)c.d;
  if (c.ss_k > 1)
    HIP_CHECK(hipMemcpyAsync(cents, c.seed_cents.p, sizeof(double) * d * (c.ss_k - 1),
                             hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(cents + d * (c.ss_k - 1), c.seed_scalar.p, sizeof(double) * d,
                           hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(flags, sc, sizeof(flags), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.ss_on = false;
  c.seed_scanned = false;
  c.seed_prog_ready = false;
  *status = flags[kSsFail] != 0.0 ? 1 : flags[kSsNan] != 0.0 ? 2 : flags[kSsNoHit] != 0.0 ? 1 : 0;
}

// Every step with the context's communicator (csrc/comm.hip): the same phases,
// the collectives enqueued from C between them.
void seed_run_sharded(Ctx& c, int64_t row_begin, int64_t n_total, int64_t first, int k,
                      const double* u, int64_t* picks, double* cents, int32_t* status) {
  if (!c.comm) CDR_FAIL(CDR_ERR_STATE, "no communicator (cdr_comm_init)");
  int64_t sizes[3];
  DevBuf bufs;
  // (sizes depend on the shard layout: computed by begin, buffers after it)
  c.ss_nbmax = ceil_div(ceil_div(n_total, kSeedBlock), c.comm_ranks);
  const size_t bs_b = sizeof(double) * c.ss_nbmax, pg_b = sizeof(SeedItem) * kShardProgCap,
               rd_b = sizeof(double) * (c.d + kShardRed);
  const size_t R = (size_t)c.comm_ranks;
  bufs.ensure(R * bs_b + R * pg_b + rd_b);
  unsigned char* base = static_cast<unsigned char*>(bufs.p);
  double* gbs = reinterpret_cast<double*>(base);
  SeedItem* progs = reinterpret_cast<SeedItem*>(base + R * bs_b);
  double* red = reinterpret_cast<double*>(base + R * bs_b + R * pg_b);
  try {
    seed_shard_begin(c, row_begin, n_total, c.comm_ranks, c.comm_rank, first, k, u, red, sizes);
    comm_allreduce_f64(c, red, c.d + kShardRed);
    for (int i = 1; i < k; ++i) {
      seed_shard_phase(c, 0, red, gbs);
      comm_allgather(c, gbs, bs_b);
      seed_shard_phase(c, 1, gbs, progs);
      comm_allgather(c, progs, pg_b);
      seed_shard_phase(c, 2, progs, red);
      comm_allreduce_f64(c, red, c.d + kShardRed);
    }
    seed_shard_end(c, red, picks, cents, status);
  } catch (...) {
    (void)hipStreamSynchronize(c.stream);
    bufs.release();
    c.ss_on = false;
    throw;
  }
  bufs.release();
}

}  // namespace cdr

using namespace cdr;

namespace cdr {

// ---------------------------------------------------------------------------
// The reference's float32 runs (X float32 keeps its dtype:
// src/kmeans_plusplus.py:6): dist_sq, its sum and the probabilities are
// float32 arrays there.
//   t       = np.linalg.norm(X - c, axis=2)   fp32 NumPy order, one rounded sqrt (:15)
//   dist_sq = min(dist_sq, t ** 2)            fp32 square; np.min keeps NaN (:14)
//   total   = dist_sq.sum()                   fp32: 8192-element chunks pairwise,
//                                             chunks added left to right (:18)
//   probs   = dist_sq / total                 fp32 (:18)
// and Generator.choice converts p to float64 before its cumsum (:19), so the
// exact cumsum scan (seed_scan) runs unchanged on p as doubles with S = 1.
// ---------------------------------------------------------------------------
template <typename S, int D>
__global__ __launch_bounds__(256) void f32r_min_kernel(const S* __restrict__ X, int64_t n,
                                                       int64_t n_pad, int d,
                                                       const float* __restrict__ cen,
                                                       float* __restrict__ dmin32,
                                                       int* __restrict__ infflag) {
  const int dd = D ? D : d;
  bool inf = false;
  for (int64_t pt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; pt < n;
       pt += (int64_t)gridDim.x * blockDim.x) {
    auto xv = [&](int f) { return (float)X[xidx(X, f, pt, n_pad)]; };  // exact: fp32 values
    auto cv = [&](int f) { return cen[f]; };
    const float R = np_sqdist<decltype(xv), decltype(cv), float>(xv, cv, dd);
    const float t = (float)sqrt((double)R);  // = the correctly rounded fp32 sqrt
    const float t2 = t * t;
    const float m = dmin32[pt];
    const float v = (m != m || t2 != t2) ? NAN : (t2 < m ? t2 : m);
    dmin32[pt] = v;
    inf = inf || isinf(v);
  }
  // (device-resident run: an infinite dist_sq makes probs inf / inf = NaN)
  if (infflag && __ballot(inf)) {
    if ((threadIdx.x & 63) == __ffsll((long long)__ballot(inf)) - 1) atomicOr(infflag, 1);
  }
}
__global__ void f32r_fill_kernel(float* __restrict__ p, int64_t n_pad, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = i < n ? INFINITY : 0.0f;
}
// fp32 pairwise sum of each 8192-element chunk: a full chunk is the perfect
// tree over 64 leaves of 128 (lane l: leaf l, combined left + right by
// shuffles); the partial last chunk runs the whole recursion on one lane.
__global__ __launch_bounds__(64) void f32r_block_kernel(const float* __restrict__ dmin32,
                                                        int64_t n, float* __restrict__ bs32) {
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t base = b * kSeedBlock;
  if (base + kSeedBlock <= n) {
    const float* src = dmin32 + base + lane * 128;
    auto leaf = [&](int i) { return src[i]; };
    float v = np_pw_leaf<decltype(leaf), float>(leaf, 128);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float r = __shfl_down(v, o);
      if ((lane & (2 * o - 1)) == 0) v = v + r;
    }
    if (lane == 0) bs32[b] = v;
  } else if (lane == 0) {
    auto all = [&](int64_t i) { return dmin32[base + i]; };
    bs32[b] = np_pairwise<decltype(all), float>(all, n - base);
  }
}
// p = fl32(dist_sq / total) as doubles (the scan's dmin, rows >= n zero) and
// each chunk's sum in any order (the scan's binade guesses only)
__global__ __launch_bounds__(256) void f32r_prob_kernel(const float* __restrict__ dmin32,
                                                        int64_t n, float total_v,
                                                        double* __restrict__ dmin,
                                                        double* __restrict__ bs,
                                                        const float* __restrict__ dtotal) {
  __shared__ double red[4];
  const int64_t b = blockIdx.x;
  const float total = dtotal ? dtotal[0] : total_v;
  double acc = 0.0;
  for (int i = threadIdx.x; i < kSeedBlock; i += 256) {
    const int64_t pt = b * kSeedBlock + i;
    // fp32 division via fp64: fl32(fl64(a / b)) = fl32(a / b) for fp32 a, b
    const double p = pt < n ? (double)(float)((double)dmin32[pt] / (double)total) : 0.0;
    dmin[pt] = p;
    acc += p;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) bs[b] = (red[0] + red[1]) + (red[2] + red[3]);
}

void f32r_seed_update(Ctx& c, const float* cen, int reset, float* total_out) {
  check_points(c);
  const int64_t nb = c.nblocks();
  c.dmin32.ensure(sizeof(float) * (size_t)(c.n_pad > 0 ? c.n_pad : 1));
  c.dmin.ensure(sizeof(double) * (size_t)(c.n_pad > 0 ? c.n_pad : 1));
  c.blocksums.ensure(sizeof(double) * (nb > 0 ? nb : 1));
  c.bs32.ensure(sizeof(float) * (nb > 0 ? nb : 1));
  c.seed_scalar.ensure(sizeof(double) * (2 * c.d + 8));
  if (reset) {
    hipLaunchKernelGGL(f32r_fill_kernel, dim3(2048), dim3(256), 0,
                       c.stream, c.dmin32.as<float>(), c.n_pad, c.n);
    HIP_CHECK(hipGetLastError());
  }
  float* dcen = reinterpret_cast<float*>(c.seed_scalar.p);
  HIP_CHECK(hipMemcpyAsync(dcen, cen, sizeof(float) * c.d, hipMemcpyHostToDevice, c.stream));
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(c.n, 256), 4096)));
  const int d = c.d;
#define INF_ ((int*)nullptr)
#define CDR_F32R_MIN(S_, X_)                                                                \
  switch (d) {                                                                             \
    case 2: hipLaunchKernelGGL((f32r_min_kernel<S_, 2>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dcen, c.dmin32.as<float>(), INF_); break; \
    case 5: hipLaunchKernelGGL((f32r_min_kernel<S_, 5>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dcen, c.dmin32.as<float>(), INF_); break; \
    case 8: hipLaunchKernelGGL((f32r_min_kernel<S_, 8>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dcen, c.dmin32.as<float>(), INF_); break; \
    case 16: hipLaunchKernelGGL((f32r_min_kernel<S_, 16>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dcen, c.dmin32.as<float>(), INF_); break; \
    default: hipLaunchKernelGGL((f32r_min_kernel<S_, 0>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dcen, c.dmin32.as<float>(), INF_); \
  }
  if (c.mode == CDR_MODE_F32X) {
    CDR_F32R_MIN(float, c.x32.as<float>())
  } else {
    CDR_F32R_MIN(double, c.x64.as<double>())
  }
#undef CDR_F32R_MIN
#undef INF_
  HIP_CHECK(hipGetLastError());
  float total = 0.0f;
  if (nb > 0) {
    hipLaunchKernelGGL(f32r_block_kernel, dim3((unsigned)nb), dim3(64), 0, c.stream,
                       c.dmin32.as<float>(), c.n, c.bs32.as<float>());
    HIP_CHECK(hipGetLastError());
    std::vector<float> bs((size_t)nb);
    HIP_CHECK(hipMemcpyAsync(bs.data(), c.bs32.p, sizeof(float) * nb, hipMemcpyDeviceToHost,
                             c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    for (float v : bs) total = total + v;  // NumPy: the chunks from 0, left to right (fp32)
  }
  *total_out = total;
  if (!(total > 0.0f) || std::isinf(total)) CDR_FAIL(CDR_ERR_NAN, "Probabilities contain NaN");
  if (nb > 0) {
    hipLaunchKernelGGL(f32r_prob_kernel, dim3((unsigned)nb), dim3(256), 0, c.stream,
                       c.dmin32.as<float>(), c.n, total, c.dmin.as<double>(),
                       c.blocksums.as<double>(), nullptr);
    HIP_CHECK(hipGetLastError());
  }
  c.seed_scanned = false;
  c.seed_prog_ready = false;
}

// ---- the reference's float32 seeding, every step on the device ----------
// The pick's row as the fp32 centre.
__global__ __launch_bounds__(64) void f32r_gather_kernel(const float* __restrict__ x32,
                                                         const double* __restrict__ x64,
                                                         const int64_t* __restrict__ pick, int d,
                                                         int64_t n_pad, float* __restrict__ cen) {
  // (a step after a bad total searches probabilities that may all be 0 and
  // find no row, -1: its pick is never used, the run raises; row 0 keeps the
  // gather in bounds)
  int64_t p = pick[0];
  if (p < 0 || p >= n_pad) p = 0;
  for (int f = threadIdx.x; f < d; f += 64)
    cen[f] = x32 ? x32[xidx(x32, f, p, n_pad)] : (float)x64[xidx(x64, f, p, n_pad)];
}
// dist_sq.sum() in fp32: the chunk sums from 0, left to right (one lane:
// the additions are sequential), and the step's verdict as Generator.choice
// gives it: a NaN, zero or infinite total with an infinite dist_sq
// (probs inf / inf) or a NaN is "Probabilities contain NaN" (code 1); an
// infinite total from finite dist_sq (overflow: probs all 0) is
// "probabilities do not sum to 1" (code 2).  The first bad step's code is
// kept; later steps run on total 1 (their picks are never used).
__global__ __launch_bounds__(64) void f32r_total_kernel(const float* __restrict__ bs32,
                                                        int64_t nb, int* __restrict__ infflag,
                                                        float* __restrict__ dtotal,
                                                        double* __restrict__ dbad) {
  float total = wave_seq_sum(bs32, nb);
  if (threadIdx.x != 0) return;
  if (!(total > 0.0f) || isinf(total)) {
    const double code = (isinf(total) && total > 0.0f && infflag[0] == 0) ? 2.0 : 1.0;
    if (dbad[0] == 0.0) dbad[0] = code;
    total = 1.0f;
  }
  infflag[0] = 0;
  dtotal[0] = total;
}

void f32r_seed_run(Ctx& c, int64_t first, int k, const double* u, int64_t* picks) {
  check_points(c);
  if (k < 1) CDR_FAIL(CDR_ERR_ARG, "k >= 1");
  if (first < 0 || first >= c.n) CDR_FAIL(CDR_ERR_ARG, "first row out of range");
  picks[0] = first;
  if (k == 1) return;
  const int64_t nb = c.nblocks();
  const int d = c.d;
  // [u: k-1][picks: k][bad x2][total f32 | inf flag][centre f32 x d]
  const size_t words = (size_t)(k - 1) + (size_t)k + 3 + (size_t)(d + 1) / 2 + 1;
  c.seed_run_buf.ensure(sizeof(double) * words);
  double* du = c.seed_run_buf.as<double>();
  int64_t* dpick = reinterpret_cast<int64_t*>(du + (k - 1));
  double* dbad = du + (k - 1) + k;
  float* dtotal = reinterpret_cast<float*>(dbad + 2);
  int* dinf = reinterpret_cast<int*>(dtotal + 1);
  float* dcen = reinterpret_cast<float*>(dbad + 3);
  HIP_CHECK(hipMemcpyAsync(du, u, sizeof(double) * (k - 1), hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipMemcpyAsync(dpick, &first, sizeof(int64_t), hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipMemsetAsync(dbad, 0, sizeof(double) * 3, c.stream));
  c.dmin32.ensure(sizeof(float) * (size_t)(c.n_pad > 0 ? c.n_pad : 1));
  c.dmin.ensure(sizeof(double) * (size_t)(c.n_pad > 0 ? c.n_pad : 1));
  c.blocksums.ensure(sizeof(double) * (nb > 0 ? nb : 1));
  c.bs32.ensure(sizeof(float) * (nb > 0 ? nb : 1));
  c.cend.ensure(sizeof(double) * nb * 2);
  c.seg_meta.ensure(sizeof(long long) * 8);
  hipLaunchKernelGGL(f32r_fill_kernel, dim3(2048), dim3(256), 0, c.stream, c.dmin32.as<float>(),
                     c.n_pad, c.n);
  HIP_CHECK(hipGetLastError());
  const float* x32 = c.mode == CDR_MODE_F32X ? c.x32.as<float>() : nullptr;
  const double* x64 = c.mode == CDR_MODE_F64 ? c.x64.as<double>() : nullptr;
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(c.n, 256), 4096)));
  for (int i = 1; i < k; ++i) {
    hipLaunchKernelGGL(f32r_gather_kernel, dim3(1), dim3(64), 0, c.stream, x32, x64,
                       dpick + (i - 1), d, c.n_pad, dcen);
#define CDR_F32R_MIN(S_, X_)                                                                  \
    switch (d) {                                                                             \
      case 2: hipLaunchKernelGGL((f32r_min_kernel<S_, 2>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dcen, c.dmin32.as<float>(), dinf); break; \
      case 5: hipLaunchKernelGGL((f32r_min_kernel<S_, 5>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dcen, c.dmin32.as<float>(), dinf); break; \
      case 8: hipLaunchKernelGGL((f32r_min_kernel<S_, 8>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dcen, c.dmin32.as<float>(), dinf); break; \
      case 16: hipLaunchKernelGGL((f32r_min_kernel<S_, 16>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dcen, c.dmin32.as<float>(), dinf); break; \
      default: hipLaunchKernelGGL((f32r_min_kernel<S_, 0>), grid, dim3(256), 0, c.stream, X_, c.n, c.n_pad, d, dcen, c.dmin32.as<float>(), dinf); \
    }
    if (x32) {
      CDR_F32R_MIN(float, x32)
    } else {
      CDR_F32R_MIN(double, x64)
    }
#undef CDR_F32R_MIN
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(f32r_block_kernel, dim3((unsigned)std::max<int64_t>(nb, 1)), dim3(64), 0,
                       c.stream, c.dmin32.as<float>(), c.n, c.bs32.as<float>());
    hipLaunchKernelGGL(f32r_total_kernel, dim3(1), dim3(64), 0, c.stream, c.bs32.as<float>(), nb,
                       dinf, dtotal, dbad);
    hipLaunchKernelGGL(f32r_prob_kernel, dim3((unsigned)std::max<int64_t>(nb, 1)), dim3(256), 0,
                       c.stream, c.dmin32.as<float>(), c.n, 1.0f, c.dmin.as<double>(),
                       c.blocksums.as<double>(), dtotal);
    HIP_CHECK(hipGetLastError());
    // Generator.choice on the float64 probabilities: the exact cumsum scan
    // (program, then the gated block walk) and the search, S = 1
    double* res = seed_res(c);
    SeedDev dv;
    seed_scan_program(c, 1.0, 0.0, dv);
    seed_scan_finish(c, 0.0, nullptr, dv);
    dv.gate = res + 1;  // the fallback runs only when the program failed
    seed_scan_walk(c, 1.0, 0.0, nullptr, dv, res);
    SeedDev ds;
    ds.c_last = res;
    ds.u = du + (i - 1);
    hipLaunchKernelGGL(search_kernel, dim3(1), dim3(64), 0, c.stream, c.dmin.as<double>(), c.n,
                       1.0, c.cend.as<double>(), nb, 0.0, 1.0, 0.5, dpick + i, ds);
    HIP_CHECK(hipGetLastError());
  }
  double bad[2];
  HIP_CHECK(hipMemcpyAsync(picks, dpick, sizeof(int64_t) * k, hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(bad, dbad, sizeof(bad), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.seed_scanned = false;
  c.seed_prog_ready = false;
  if (bad[0] == 2.0) CDR_FAIL(CDR_ERR_NAN, "probabilities do not sum to 1");
  if (bad[0] != 0.0) CDR_FAIL(CDR_ERR_NAN, "Probabilities contain NaN");
  if (bad[1] != 0.0) CDR_FAIL(CDR_ERR_STATE, "k-means++ sampler found no index");
}

}  // namespace cdr

extern "C" {

int cdr_f32r_seed_run(cdr_ctx* h, int64_t first, int32_t k, const double* u, int64_t* picks) {
  CDR_TRY
  if (!h || !picks || (k > 1 && !u)) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  f32r_seed_run(h->c, first, (int)k, u, picks);
  CDR_CATCH
}

int cdr_seed_reset(cdr_ctx* h) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_reset(h->c);
  CDR_CATCH
}

int cdr_f32r_seed_update(cdr_ctx* h, const float* c, int32_t reset, float* total) {
  CDR_TRY
  if (!h || !c || !total) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  f32r_seed_update(h->c, c, reset, total);
  CDR_CATCH
}

int cdr_seed_update(cdr_ctx* h, const double* c) {
  CDR_TRY
  if (!h || !c) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_update(h->c, c);
  CDR_CATCH
}

int cdr_seed_num_blocks(cdr_ctx* h, int64_t* nblocks) {
  CDR_TRY
  if (!h || !nblocks) CDR_FAIL(CDR_ERR_ARG, "null argument");
  *nblocks = h->c.nblocks();
  CDR_CATCH
}

int cdr_seed_block_sums(cdr_ctx* h, double* out) {
  CDR_TRY
  if (!h || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  const int64_t nb = c.nblocks();
  if (nb > 0) {
    HIP_CHECK(hipMemcpyAsync(out, c.blocksums.p, sizeof(double) * nb, hipMemcpyDeviceToHost,
                             c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
  }
  CDR_CATCH
}

int cdr_seed_scan(cdr_ctx* h, double total, double c_in, double* c_out) {
  CDR_TRY
  if (!h || !c_out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  if (!(total > 0.0) || std::isinf(total)) CDR_FAIL(CDR_ERR_NAN, "Probabilities contain NaN");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_scan(h->c, total, c_in, c_out);
  CDR_CATCH
}

int cdr_seed_scan_begin(cdr_ctx* h, double total, double c_guess, int64_t* n_items,
                        int64_t* n_fine) {
  CDR_TRY
  if (!h || !n_items || !n_fine) CDR_FAIL(CDR_ERR_ARG, "null argument");
  if (!(total > 0.0) || std::isinf(total)) CDR_FAIL(CDR_ERR_NAN, "Probabilities contain NaN");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_scan_begin(h->c, total, c_guess, n_items, n_fine);
  CDR_CATCH
}

int cdr_seed_scan_items(cdr_ctx* h, cdr_seed_item* out, int64_t cap, int64_t* n_items) {
  CDR_TRY
  if (!h || !n_items || (!out && cap > 0)) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_scan_items(h->c, out, cap, n_items);
  CDR_CATCH
}

int cdr_seed_scan_end(cdr_ctx* h, double c_in, double* c_out) {
  CDR_TRY
  if (!h || !c_out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_scan_end(h->c, c_in, c_out);
  CDR_CATCH
}

int cdr_seed_run(cdr_ctx* h, int64_t first, int32_t k, const double* u, int64_t* picks) {
  CDR_TRY
  if (!h || !picks || (k > 1 && !u)) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_run(h->c, first, (int)k, u, picks);
  CDR_CATCH
}

int cdr_seed_shard_begin(cdr_ctx* h, int64_t row_begin, int64_t n_total, int32_t nranks,
                         int32_t rank, int64_t first, int32_t k, const double* u, double* red,
                         int64_t* sizes) {
  CDR_TRY
  if (!h || !red || !sizes || (k > 1 && !u)) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_shard_begin(h->c, row_begin, n_total, nranks, rank, first, (int)k, u, red, sizes);
  CDR_CATCH
}

int cdr_seed_shard_phase(cdr_ctx* h, int32_t phase, const void* in, void* out) {
  CDR_TRY
  if (!h || !in || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_shard_phase(h->c, phase, in, out);
  CDR_CATCH
}

int cdr_seed_shard_end(cdr_ctx* h, const double* red, int64_t* picks, double* cents,
                       int32_t* status) {
  CDR_TRY
  if (!h || !red || !picks || !cents || !status) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_shard_end(h->c, red, picks, cents, status);
  CDR_CATCH
}

int cdr_seed_run_sharded(cdr_ctx* h, int64_t row_begin, int64_t n_total, int64_t first, int32_t k,
                         const double* u, int64_t* picks, double* cents, int32_t* status) {
  CDR_TRY
  if (!h || !picks || !cents || !status || (k > 1 && !u)) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_run_sharded(h->c, row_begin, n_total, first, (int)k, u, picks, cents, status);
  CDR_CATCH
}

int cdr_seed_stats(cdr_ctx* h, int64_t* out) {
  CDR_TRY
  if (!h || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  out[0] = h->c.seed_programs;
  out[1] = h->c.seed_fallbacks;
  CDR_CATCH
}

int cdr_seed_program_eval(const cdr_seed_item* items, int64_t n_items, double c_in,
                          double* c_out, int32_t* ok) {
  CDR_TRY
  if (!c_out || !ok || (!items && n_items > 0) || n_items < 0)
    CDR_FAIL(CDR_ERR_ARG, "bad argument");
  double c = c_in;
  int32_t good = 1;
  for (int64_t i = 0; i < n_items && good; ++i) {
    SeedItem it;
    std::memcpy(&it, items + i, sizeof(it));
    if (it.kind == kItEnd) break;
    if (it.kind == kItFine || !item_apply(it, c)) good = 0;
  }
  *c_out = c;
  *ok = good;
  CDR_CATCH
}

int cdr_seed_search(cdr_ctx* h, double c_last, double u, int64_t* idx) {
  CDR_TRY
  if (!h || !idx) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  seed_search(h->c, c_last, u, idx);
  CDR_CATCH
}

}  // extern "C"
