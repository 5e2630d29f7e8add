// screen_big.hip — Lloyd step for the large-k / large-d regime (BASELINE
// config 5: 50M x d=64, k=1024), reference src/kmeans_plusplus.py:33-41.
//
// At k*d this large the distance computation is a dense contraction
// (2nkd = 6.6 TFLOP per step) and belongs on the matrix cores; the update
// table k x (d+1) (520 KB) no longer fits a workgroup's LDS, so assign and
// update are separate passes:
//
//  L1  screen_big<DQ, 1>: every point, ONE fp16 MFMA product per 32x32 block,
//      S_j = fl32(C_j - 2 chi_j . xhi) with C_j = ||chat_j||^2 + D (the MFMA C
//      operand), xhat = (x - mu) 2^sigma the exact pre-centred copy.  The
//      fp16 A fragments of all k centroids (128 KB at k = 1024, d = 64) and
//      the C operand rows sit in LDS for the whole persistent launch; a wave
//      takes 64 points (two 32-point B tiles sharing every A fragment read).
//      Per 32-centroid block each lane reduces its 16 values to a keyed
//      top-2 (v_min3/v_med3 on (bits & ~15) | reg), then merges that into a
//      full-precision running (best, index, runner-up).  A point is certified
//      when runner > best (1 + 2^-18) + T1 (T1 = twice the rigorous bound on
//      |S_j - exact shifted distance| + the reference's rounding slack);
//      the rest go to per-wave regions.
//  L2  cand_big<DQ>: the L1 leftovers, 64 per wave (chunks of L1's regions
//      numbered through an LDS prefix): the same one-product screen is
//      recomputed and every centroid with S_j <= best (1 + 2^-18) + T1 is a
//      candidate (the exact argmin is among them); each lane then takes one
//      point and evaluates its few candidates in exact fp64 NumPy order.
//  L3  exact_big: points with more than kMaxCand candidates, one wave per
//      point in exact fp64 NumPy order over all k (8 lanes per centroid = the
//      8 pairwise accumulators, combined in NumPy's tree by shfl_xor 1, 2, 4),
//      correctly rounded sqrt, first minimum of the roots (np.argmin of
//      np.linalg.norm).
//  U   update_big<FG>: sums per (cluster, feature) from the labels, in passes
//      of FG features: one workgroup per CU holds an LDS table [FG][k] of
//      fp64 sums (exact: grid values) fed by ds_add_f64, then adds its table
//      as exact int64 fixed point into the (k, d+1) output with atomics.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cdr_internal.h"
#include "exact_math.h"

namespace cdr {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

struct BigArgs {
  const float* XT;      // pre-centred points [Q][n_pad][4]
  int64_t n, n_pad;
  int d, k, Q, KB;      // Q = stored feature quads, KB = ceil(k / 32)
  const h8* frag;       // NPROD 1: [KB][DQ][64]; NPROD 3: [KB][2][DQ][64]
  const float* cinit;   // [KB * 32] C operand per centroid row (1e30 past k)
  float thr0, thr_rel;
  int32_t* labels;
  // GATHER input: per-region point lists of the previous level
  const int32_t* in_list;
  const int32_t* in_count;
  int in_cap, in_regions;
  // uncertified output: one region of out_cap entries per wave
  int32_t* out_list;
  float* out_best;     // L1: the point's best screen value (truncated key), same slots
  int32_t* out_count;  // [nwaves + 1]: per-wave counts, then the total
  int out_cap;
};

__device__ __forceinline__ unsigned pack_h2(float a, float b) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  h2 h = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(unsigned, h);
}

__device__ __forceinline__ void swap32(unsigned& x, unsigned& y) {
  auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}

}  // namespace

// DQ: 16-feature K chunks (d <= 16 DQ).  NPROD: 1 (A = -2 chi, B = xhi) or 3
// (A1 = -2 chi, A3 = -2 clo; A1 xhi + A1 xlo + A3 xhi).  GATHER: points come
// from the previous level's regions (a.in_*) instead of a dense sweep.
// ALDS: A fragments staged in LDS (L1) or read from global (L2).
constexpr int kBigThreads = 1024;  // L1: one workgroup per CU, 4 waves per SIMD

template <int DQ, int NPROD, bool GATHER, bool ALDS>
__global__ __launch_bounds__(kBigThreads) void screen_big(BigArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NA = NPROD == 1 ? 1 : 2;
  float* scin = reinterpret_cast<float*>(smem);                       // [KB * 32]
  h8* sfrag = reinterpret_cast<h8*>(smem + (size_t)a.KB * 32 * 4);    // [KB][NA][DQ][64]
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int p = lane & 31;
  for (int i = threadIdx.x; i < a.KB * 32; i += blockDim.x) scin[i] = a.cinit[i];
  if constexpr (ALDS) {
    const int nf = a.KB * NA * DQ * 64;
    for (int i = threadIdx.x; i < nf; i += blockDim.x) sfrag[i] = a.frag[i];
  }
  __syncthreads();
  const h8* frag = ALDS ? sfrag : a.frag;

  const int wpb = blockDim.x >> 6;
  const int wave_id = blockIdx.x * wpb + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * wpb;
  int32_t* region = a.out_list + (size_t)wave_id * a.out_cap;
  int used = 0;
  int cur_region = 0;  // GATHER: the input region being worked
  const f4* X4 = reinterpret_cast<const f4*>(a.XT);

  // work items: dense groups of 64 points, or (region, 64-point chunk) pairs
  int64_t items;
  if constexpr (GATHER) {
    items = 0;  // walk regions below
  } else {
    items = (a.n + 63) >> 6;
  }
  auto run_group = [&](const int64_t (&pt)[2], const bool (&real)[2]) {
    // B fragments: tile t, chunk c: features 16c + 8h .. + 8 of point pt[t]
    h8 BH[2][DQ], BL[2][DQ];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int c = 0; c < DQ; ++c) {
        const int q0 = 4 * c + 2 * h;
        f4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
        if (real[t] && q0 < a.Q) v0 = X4[(int64_t)q0 * a.n_pad + pt[t]];
        if (real[t] && q0 + 1 < a.Q) v1 = X4[(int64_t)(q0 + 1) * a.n_pad + pt[t]];
        u4v H = {pack_h2(v0[0], v0[1]), pack_h2(v0[2], v0[3]), pack_h2(v1[0], v1[1]),
                 pack_h2(v1[2], v1[3])};
        BH[t][c] = __builtin_bit_cast(h8, H);
        if constexpr (NPROD == 3) {
          const h8 hh = BH[t][c];
          u4v L = {pack_h2(v0[0] - (float)hh[0], v0[1] - (float)hh[1]),
                   pack_h2(v0[2] - (float)hh[2], v0[3] - (float)hh[3]),
                   pack_h2(v1[0] - (float)hh[4], v1[1] - (float)hh[5]),
                   pack_h2(v1[2] - (float)hh[6], v1[3] - (float)hh[7])};
          BL[t][c] = __builtin_bit_cast(h8, L);
        }
      }
    float bv[2] = {INFINITY, INFINITY}, sv[2] = {INFINITY, INFINITY};
    int bi[2] = {0, 0};
    for (int b = 0; b < a.KB; ++b) {
      f16v acc[2];
      {
        const f4* cr = reinterpret_cast<const f4*>(scin + 32 * b + 4 * h);
        f16v ci;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 v = cr[2 * q];  // rows 8q + 4h .. + 4
#pragma unroll
          for (int i = 0; i < 4; ++i) ci[4 * q + i] = v[i];
        }
        acc[0] = ci;
        acc[1] = ci;
      }
#pragma unroll
      for (int c = 0; c < DQ; ++c) {
        const h8 A1 = frag[((size_t)(b * NA + 0) * DQ + c) * 64 + lane];
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, BH[0][c], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, BH[1][c], acc[1], 0, 0, 0);
        if constexpr (NPROD == 3) {
          const h8 A3 = frag[((size_t)(b * NA + 1) * DQ + c) * 64 + lane];
          acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, BL[0][c], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, BL[1][c], acc[1], 0, 0, 0);
          acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A3, BH[0][c], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A3, BH[1][c], acc[1], 0, 0, 0);
        }
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        // keyed top-2 of the lane's 16 values (every value >= 0: bits order)
        auto key = [&](int i) { return (__float_as_uint(acc[t][i]) & ~15u) | (unsigned)i; };
        unsigned kb = min(key(0), key(1)), ks = max(key(0), key(1));
#pragma unroll
        for (int i = 2; i < 16; i += 2) {
          const unsigned x = key(i), y = key(i + 1);
          unsigned m;
          asm("v_med3_u32 %0, %1, %2, %3" : "=v"(m) : "v"(kb), "v"(x), "v"(y));
          asm("v_min3_u32 %0, %1, %2, %3" : "=v"(kb) : "v"(kb), "v"(x), "v"(y));
          ks = min(ks, m);
        }
        const int ib = (int)(kb & 15u);
        const float vb = __uint_as_float(kb & ~15u);
        const float vs = __uint_as_float(ks & ~15u);
        const int jb = 32 * b + 8 * (ib >> 2) + 4 * h + (ib & 3);
        const bool tk = vb < bv[t];
        sv[t] = fminf(fminf(sv[t], vs), tk ? bv[t] : vb);
        bi[t] = tk ? jb : bi[t];
        bv[t] = tk ? vb : bv[t];
      }
    }
    // merge the two row halves: lanes < 32 end with tile 0's point p,
    // lanes >= 32 with tile 1's point p
    unsigned b0 = __float_as_uint(bv[0]), b1 = __float_as_uint(bv[1]);
    unsigned s0 = __float_as_uint(sv[0]), s1 = __float_as_uint(sv[1]);
    unsigned i0 = (unsigned)bi[0], i1 = (unsigned)bi[1];
    swap32(b0, b1);
    swap32(s0, s1);
    swap32(i0, i1);
    const float fb0 = __uint_as_float(b0), fb1 = __uint_as_float(b1);
    const float fs0 = __uint_as_float(s0), fs1 = __uint_as_float(s1);
    const bool t1 = fb1 < fb0 || (fb1 == fb0 && (int)i1 < (int)i0);
    const float best = t1 ? fb1 : fb0;
    const int label = (int)(t1 ? i1 : i0);
    const float run = fminf(fminf(fs0, fs1), t1 ? fb0 : fb1);
    const int64_t mypt = h == 0 ? pt[0] : pt[1];
    const bool myreal = h == 0 ? real[0] : real[1];
    // rows past k carry C = 1e30: never best, never a close runner-up
    const bool cert = run > fmaf(best, a.thr_rel, a.thr0);  // NaN: never
    if (myreal && cert) a.labels[mypt] = label;
    const unsigned long long need = __ballot(myreal && !cert);
    if (need) {
      const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(need >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((unsigned)need, 0u));
      const int cntn = __popcll(need);
      int base;
      int32_t* reg;
      if constexpr (GATHER) {
        // leftovers go to the input region's slot range (capacity in_cap)
        int b0 = 0;
        if (lane == 0) {
          b0 = atomicAdd(a.out_count + cur_region, cntn);
          atomicAdd(a.out_count + a.in_regions, cntn);
        }
        base = __shfl(b0, 0);
        reg = a.out_list + (size_t)cur_region * a.out_cap;
      } else {
        base = used;
        reg = region;
        used += cntn;
      }
      if (myreal && !cert) {
        reg[base + rank] = (int32_t)mypt;
        if constexpr (!GATHER) a.out_best[(size_t)wave_id * a.out_cap + base + rank] = best;
      }
    }
  };

  if constexpr (!GATHER) {
    for (int64_t g = wave_id; g < items; g += nwaves) {
      const int64_t base = g << 6;
      const int64_t pt[2] = {base + p, base + 32 + p};
      const bool real[2] = {pt[0] < a.n, pt[1] < a.n};
      run_group(pt, real);
    }
  } else {
    // regions of the previous level, 64 points at a time
    for (int r = 0; r < a.in_regions; ++r) {
      const int cnt = a.in_count[r];
      cur_region = r;
      const int32_t* src = a.in_list + (size_t)r * a.in_cap;
      for (int e0 = 0; e0 < cnt; e0 += 64) {
        if (((r * 7919 + e0 / 64) % nwaves) != wave_id) continue;  // spread the chunks
        const int e_a = e0 + p, e_b = e0 + 32 + p;
        const bool real[2] = {e_a < cnt, e_b < cnt};
        const int64_t pt[2] = {real[0] ? (int64_t)src[e_a] : 0, real[1] ? (int64_t)src[e_b] : 0};
        run_group(pt, real);
      }
    }
  }
  if constexpr (!GATHER) {
    if (lane == 0) {
      a.out_count[wave_id] = used;
      if (used) atomicAdd(a.out_count + nwaves, used);
    }
  }
}

// dst[i] = src[i] for 16-byte words; src is mapped pinned host memory.
__global__ __launch_bounds__(256) void pull_host_big(const uint4* __restrict__ src,
                                                     uint4* __restrict__ dst, int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) dst[i] = src[i];
}

// L2: the points L1 could not certify, 64 per wave (chunks of L1's regions).
// The one-product screen is recomputed (bit-identical to L1's) and every
// centroid with S_j <= best_L1 (1 + 2^-18) + T1 is a candidate: the exact
// argmin is among them (|S_j - T_j| <= E for every j, T1 >= 2E + the
// reference's rounding slack).  Candidates go to a per-point LDS list; then
// each lane takes one point and evaluates its candidates in exact fp64 NumPy
// order (np_sqdist, correctly rounded sqrt, first minimum by (root, index)).
// A point with more than kMaxCand candidates goes to the flat overflow list
// for exact_big (all k centroids).
constexpr int kMaxCand = 16;
constexpr int kMaxRegions = 8192;  // L1 waves (regions) the candidate level can index

template <int DQ>
__global__ __launch_bounds__(256) void cand_big(BigArgs a, const float* __restrict__ X0,
                                                const double* __restrict__ C64,
                                                int32_t* __restrict__ ovf,
                                                int32_t* __restrict__ ovf_count, int abl) {
  __shared__ int scnt[4][64];
  __shared__ int scand[4][64 * kMaxCand];
  __shared__ int schunk[kMaxRegions + 1];  // exclusive prefix of 64-point chunks per region
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int h = lane >> 5;
  const int p = lane & 31;
  const int wave_id = blockIdx.x * 4 + w;
  const int nwaves = gridDim.x * 4;
  const f4* X4 = reinterpret_cast<const f4*>(a.XT);
  // chunk numbering: region r owns chunks [schunk[r], schunk[r + 1])
  const int R = a.in_regions;
  for (int r = threadIdx.x; r < R; r += blockDim.x) schunk[r + 1] = (a.in_count[r] + 63) >> 6;
  if (threadIdx.x == 0) schunk[0] = 0;
  __syncthreads();
  if (w == 0) {  // one wave scans: lane l sums a contiguous slice, then a wave scan
    const int per = (R + 63) / 64;
    const int lo = 1 + lane * per, hi = min(R + 1, lo + per);
    int sum = 0;
    for (int i = lo; i < hi; ++i) sum += schunk[i];
    int incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    int run = incl - sum;
    for (int i = lo; i < hi; ++i) {
      run += schunk[i];
      schunk[i] = run;
    }
  }
  __syncthreads();
  const int nchunks = (abl & 1) ? 0 : schunk[R];
  for (int ch = wave_id; ch < nchunks; ch += nwaves) {
    int lo = 0, hi = R;  // last r with schunk[r] <= ch
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (schunk[mid] <= ch) lo = mid; else hi = mid;
    }
    const int r = lo;
    const int cnt = a.in_count[r];
    const int e0 = (ch - schunk[r]) * 64;
    const int32_t* src = a.in_list + (size_t)r * a.in_cap;
    const float* srcb = a.out_best + (size_t)r * a.in_cap;
    {
      int64_t pt[2];
      bool real[2];
      float lim[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int e = e0 + 32 * t + p;
        real[t] = e < cnt;
        pt[t] = real[t] ? (int64_t)src[e] : 0;
        lim[t] = real[t] ? fmaf(srcb[e], a.thr_rel, a.thr0) : -1.0f;
      }
      scnt[w][lane] = 0;
      h8 BH[2][DQ];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < DQ; ++c) {
          const int q0 = 4 * c + 2 * h;
          f4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
          if (real[t] && q0 < a.Q) v0 = X4[(int64_t)q0 * a.n_pad + pt[t]];
          if (real[t] && q0 + 1 < a.Q) v1 = X4[(int64_t)(q0 + 1) * a.n_pad + pt[t]];
          u4v H = {pack_h2(v0[0], v0[1]), pack_h2(v0[2], v0[3]), pack_h2(v1[0], v1[1]),
                   pack_h2(v1[2], v1[3])};
          BH[t][c] = __builtin_bit_cast(h8, H);
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int b = 0; b < ((abl & 2) ? 0 : a.KB); ++b) {
        f16v acc[2];
        {
          const f4* cr = reinterpret_cast<const f4*>(a.cinit + 32 * b + 4 * h);
          f16v ci;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f4 v = cr[2 * q];
#pragma unroll
            for (int i = 0; i < 4; ++i) ci[4 * q + i] = v[i];
          }
          acc[0] = ci;
          acc[1] = ci;
        }
#pragma unroll
        for (int c = 0; c < DQ; ++c) {
          const h8 A1 = a.frag[((size_t)b * DQ + c) * 64 + lane];
          acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, BH[0][c], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, BH[1][c], acc[1], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (acc[t][i] <= lim[t]) {
              const int j = 32 * b + 8 * (i >> 2) + 4 * h + (i & 3);
              const int slot = atomicAdd(&scnt[w][32 * t + p], 1);
              if (slot < kMaxCand) scand[w][(32 * t + p) * kMaxCand + slot] = j;
            }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // lane l: point l of the chunk (tile l / 32, column l % 32)
      const int e = e0 + lane;
      if (e < cnt) {
        const int64_t mypt = (int64_t)src[e];
        const int nc = scnt[w][lane];
        if (abl & 4) {
        } else if (nc > kMaxCand || nc == 0) {
          ovf[atomicAdd(ovf_count, 1)] = (int32_t)mypt;
        } else {
          double rb = INFINITY;
          int jb = 0x7fffffff;
          for (int s2 = 0; s2 < nc; ++s2) {
            const int j = scand[w][lane * kMaxCand + s2];
            const double* cj = C64 + (size_t)j * a.d;
            const double R = np_sqdist([&](int f) { return (double)X0[xidx(f, mypt, a.n_pad)]; },
                                       [&](int f) { return cj[f]; }, a.d);
            const double root = sqrt(R);
            if (root < rb || (root == rb && j < jb)) {
              rb = root;
              jb = j;
            }
          }
          a.labels[mypt] = jb;
        }
      }
    }
  }
}

// L3: exact fp64 assignment of the overflow list (flat, count at *count):
// one wave per point.  Lane (c, r) = (lane >> 3, lane & 7) takes centroids
// c, c + 8, ... and NumPy's pairwise accumulator r (features r, r + 8, ...,
// summed sequentially), shfl_xor 1, 2, 4 combine ((r0+r1)+(r2+r3))+
// ((r4+r5)+(r6+r7)), the d % 8 tail is added in order; sqrt is correctly
// rounded; first minimum of the roots (src/kmeans_plusplus.py:33-34).
// d >= 8 here (the large regime); the point sits in LDS.
__global__ __launch_bounds__(64) void exact_big(const float* __restrict__ X, int64_t n_pad,
                                                int d, const double* __restrict__ C, int k,
                                                const int32_t* __restrict__ list,
                                                const int32_t* __restrict__ count,
                                                int32_t* __restrict__ labels) {
  __shared__ double sx[128];
  const int lane = threadIdx.x;
  const int c8 = lane >> 3, r = lane & 7;
  const int dd = d - (d & 7);
  const int total = *count;
  for (int e = blockIdx.x; e < total; e += gridDim.x) {
    const int64_t pt = list[e];
    __syncthreads();
    for (int f = lane; f < d; f += 64) sx[f] = (double)X[xidx(f, pt, n_pad)];
    __syncthreads();
    double rb = INFINITY;
    int jmin = 0x7fffffff;
    for (int j0 = 0; j0 < k; j0 += 8) {
      const int j = j0 + c8;
      const double* cj = C + (size_t)(j < k ? j : 0) * d;
      double acc;
      {
        const double t = sx[r] - cj[r];
        acc = t * t;
      }
      for (int f = 8 + r; f < dd; f += 8) {
        const double t = sx[f] - cj[f];
        acc = acc + t * t;
      }
      acc = acc + __shfl_xor(acc, 1);
      acc = acc + __shfl_xor(acc, 2);
      acc = acc + __shfl_xor(acc, 4);
      for (int f = dd; f < d; ++f) {
        const double t = sx[f] - cj[f];
        acc = acc + t * t;
      }
      const double root = sqrt(acc);
      if (j < k && root < rb) {  // strict: first index on ties
        rb = root;
        jmin = j;
      }
    }
    for (int o = 8; o < 64; o <<= 1) {
      const double ro = __shfl_xor(rb, o);
      const int jo = __shfl_xor(jmin, o);
      if (ro < rb || (ro == rb && jo < jmin)) {
        rb = ro;
        jmin = jo;
      }
    }
    if (lane == 0) labels[pt] = jmin < k ? jmin : 0;
  }
}

// Sums per (cluster, feature) of features [FG g, FG g + FG) from the labels,
// blockIdx.y = g; each workgroup takes a contiguous point range.  The LDS
// table [FG][k] is exact (fp64 of grid values, |sum| < 2^53 grid units);
// it is added to out (k, d+1) int64 as x 2^S with atomics; g = 0 also counts.
template <int FG>
__global__ __launch_bounds__(1024) void update_big(const float* __restrict__ X, int64_t n,
                                                   int64_t n_pad, int d, int k,
                                                   const int32_t* __restrict__ labels,
                                                   double fx, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* tsum = reinterpret_cast<double*>(smem);        // [FG][k]
  int* tcnt = reinterpret_cast<int*>(tsum + (size_t)FG * k);  // [k]
  const int g = blockIdx.y;
  const int f0 = FG * g;
  for (int i = threadIdx.x; i < FG * k; i += blockDim.x) tsum[i] = 0.0;
  for (int i = threadIdx.x; i < k; i += blockDim.x) tcnt[i] = 0;
  __syncthreads();
  const int64_t per = ((n + gridDim.x - 1) / gridDim.x + 63) & ~63ll;
  const int64_t i0 = (int64_t)blockIdx.x * per;
  const int64_t i1 = (i0 + per) < n ? (i0 + per) : n;
  const f4* X4 = reinterpret_cast<const f4*>(X);
  constexpr int FQ = FG / 4;
  const int Q = d4_of(d) / 4;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const int l = labels[i];
    f4 v[FQ];
#pragma unroll
    for (int q = 0; q < FQ; ++q) {
      const int qq = f0 / 4 + q;
      v[q] = qq < Q ? X4[(int64_t)qq * n_pad + i] : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < FQ; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (f0 + 4 * q + c < d) atomicAdd(&tsum[(4 * q + c) * k + l], (double)v[q][c]);
    if (g == 0) atomicAdd(&tcnt[l], 1);
  }
  __syncthreads();
  const int d1 = d + 1;
  for (int i = threadIdx.x; i < FG * k; i += blockDim.x) {
    const int f = f0 + i / k, j = i % k;
    const double s = tsum[i];
    if (f < d && s != 0.0)
      atomicAdd(&out[(size_t)j * d1 + f], (unsigned long long)__double2ll_rn(s * fx));
  }
  if (g == 0)
    for (int j = threadIdx.x; j < k; j += blockDim.x)
      if (tcnt[j]) atomicAdd(&out[(size_t)j * d1 + d], (unsigned long long)(long long)tcnt[j]);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
extern int lloyd_num_cus(int device);
void ensure_precentered(Ctx& c);

static int big_dq(int d) { return (d + 15) / 16; }
static size_t big_l1_lds(int k, int d) {
  const int KB = (k + 31) / 32;
  return (size_t)KB * 32 * 4 + (size_t)KB * big_dq(d) * 64 * 16;
}
static int big_fg(int k) {
  const size_t lim = 150 * 1024;
  if ((size_t)k * (16 * 8 + 4) <= lim) return 16;
  if ((size_t)k * (8 * 8 + 4) <= lim) return 8;
  if ((size_t)k * (4 * 8 + 4) <= lim) return 4;
  return 0;
}

bool big_supported(const Ctx& c, int k) {
  return c.mode == CDR_MODE_F32X && c.pre_ok && c.d >= 8 && c.d <= 64 && k >= 1 &&
         big_l1_lds(k, c.d) <= 150 * 1024 && big_fg(k) > 0;
}

struct PlanBig {
  std::vector<h8> frag1, frag3;
  std::vector<float> cinit;
  float thr1, thr3, thr_rel;
};

// Rigorous screen error bounds (see the file header); mirrors build_plan32's
// terms with N = fp32 additions in the MFMA chain.
static void build_plan_big(const Ctx& c, const double* C, int k, PlanBig& pl) {
  const int d = c.d, DQ = big_dq(d), KB = (k + 31) / 32;
  const double sc = std::ldexp(1.0, c.sigma);
  std::vector<double> ch((size_t)k * d), cc(k, 0.0);
  double ccmax = 0.0, l1c = 0.0;
  for (int j = 0; j < k; ++j) {
    double s = 0.0, l1 = 0.0;
    for (int f = 0; f < d; ++f) {
      const double v = (C[(size_t)j * d + f] - (double)c.mu[f]) * sc;
      ch[(size_t)j * d + f] = v;
      s += v * v;
      l1 += std::fabs(v);
    }
    cc[j] = s;
    ccmax = std::fmax(ccmax, s);
    l1c = std::fmax(l1c, l1);
  }
  double xxmax = 0.0, l1x = 0.0;
  for (int f = 0; f < d; ++f) {
    const double dev =
        std::fmax(c.fmax[f] - (double)c.mu[f], (double)c.mu[f] - c.fmin[f]) * sc;
    xxmax += dev * dev;
    l1x += dev;
  }
  xxmax *= 1.0 + 1e-6;
  const double u = std::ldexp(1.0, -24);
  const double eps = std::ldexp(1.0, -11), eta = std::ldexp(1.0, -25);
  const double cx = std::sqrt(ccmax * xxmax);
  // one product: |c.x - chi.xhi| <= 2 eps (1 + eps) ||c|| ||x|| + eta (l1x + (1 + eps) l1c)
  const double P1 = 2.0 * eps * (1.0 + eps) * cx + eta * (l1x + (1.0 + eps) * l1c);
  const double N1 = 16.0 * DQ + 1.0, N3 = 3.0 * 16.0 * DQ + 1.0;
  const double g1 = 2.0 * u * N1 / (1.0 - 2.0 * u * N1);
  const double g3 = 2.0 * u * N3 / (1.0 - 2.0 * u * N3);
  const double E1a = 2.0 * P1 + g1 * (ccmax + 2.0 * xxmax + 4.0 * cx + 4.0) + u * (ccmax + 2.0 * xxmax + 4.0);
  // D >= max ||xhat||^2 + margin keeps every screen value >= 0
  const double D = xxmax + 4.0 * E1a + std::ldexp(1.0, -20);
  const double sum1 = (ccmax + D) * (1.0 + u) + 2.0 * (1.0 + eps) * (1.0 + eps) * cx;
  const double E1 = 2.0 * P1 + g1 * sum1 + u * (ccmax + D) + std::ldexp(1.0, -46) * (ccmax + D);
  // three products: the split leaves |c.x - (chi xhi + chi xlo + clo xhi)| <=
  // 2.4 2^-22 ||c|| ||x|| + 2^-24 (l1c + l1x)
  const double P3 = 2.4 * std::ldexp(1.0, -22) * cx + std::ldexp(1.0, -24) * (l1c + l1x);
  const double sum3 = (ccmax + D) * (1.0 + u) + 2.0 * (1.0 + std::ldexp(1.0, -9)) * cx;
  const double E3 = 2.0 * P3 + g3 * sum3 + u * (ccmax + D) + std::ldexp(1.0, -46) * (ccmax + D);
  // reference slack: the fp64 distances and roots must not tie or flip
  const double Wmax = (std::sqrt(ccmax) + std::sqrt(xxmax)) * (std::sqrt(ccmax) + std::sqrt(xxmax));
  const double slack = std::ldexp(Wmax + 1.0, -38);
  pl.thr1 = (float)((2.0 * E1 + slack) * 1.001);
  pl.thr3 = (float)((2.0 * E3 + slack) * 1.001);
  pl.thr_rel = 1.0f + std::ldexp(1.0f, -18);  // the 16-ulp key truncation
  pl.cinit.assign((size_t)KB * 32, 1.0e30f);
  for (int j = 0; j < k; ++j) pl.cinit[j] = (float)(cc[j] + D);
  pl.frag1.assign((size_t)KB * DQ * 64, h8{});
  pl.frag3.assign((size_t)KB * 2 * DQ * 64, h8{});
  for (int b = 0; b < KB; ++b)
    for (int cq = 0; cq < DQ; ++cq)
      for (int lane = 0; lane < 64; ++lane) {
        const int j = 32 * b + (lane & 31);
        const int hh = lane >> 5;
        h8 A1 = {}, A3 = {};
        for (int i = 0; i < 8; ++i) {
          const int f = 16 * cq + 8 * hh + i;
          if (j >= k || f >= d) continue;
          const double v = ch[(size_t)j * d + f];
          const _Float16 hi = (_Float16)v;
          const _Float16 lo = (_Float16)(v - (double)hi);
          A1[i] = (_Float16)(-2.0 * (double)hi);
          A3[i] = (_Float16)(-2.0 * (double)lo);
        }
        pl.frag1[((size_t)b * DQ + cq) * 64 + lane] = A1;
        pl.frag3[((size_t)(b * 2 + 0) * DQ + cq) * 64 + lane] = A1;
        pl.frag3[((size_t)(b * 2 + 1) * DQ + cq) * 64 + lane] = A3;
      }
}

template <int DQ>
static void launch_big_levels(Ctx& c, const BigArgs& a1, const BigArgs& a2, dim3 g1, dim3 g2,
                              size_t lds1, const double* dC, int32_t* ovf, int32_t* ovf_count,
                              bool prof) {
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&screen_big<DQ, 1, false, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((screen_big<DQ, 1, false, true>), g1, dim3(kBigThreads), lds1, c.stream, a1);
  HIP_CHECK(hipGetLastError());
  if (prof) prof_mark(c, 1);  // the L1 screen alone
#ifdef CDR_EXPERIMENTS
  static const int abl = std::getenv("CDR_BIG_ABL") ? std::atoi(std::getenv("CDR_BIG_ABL")) : 0;
#else
  constexpr int abl = 0;
#endif
  hipLaunchKernelGGL((cand_big<DQ>), g2, dim3(256), 0, c.stream, a2, c.x32.as<float>(), dC, ovf,
                     ovf_count, abl);
  HIP_CHECK(hipGetLastError());
}

// One F32X Lloyd step in the large regime: labels for every point and the
// exact int64 (k, d+1) sums/counts in dout (device).  Returns false when the
// shape is not covered (nothing launched).
bool big_step(Ctx& c, const double* C, int k, long long* dout, bool prof) {
  if (!big_supported(c, k)) return false;
  ensure_precentered(c);
  PlanBig pl;
  build_plan_big(c, C, k, pl);
  const int d = c.d, DQ = big_dq(d), KB = (k + 31) / 32, Q = d4_of(d) / 4;
  const int cus = lloyd_num_cus(c.device);
  // one upload: frag1 | cinit | C (fp64)
  const size_t b1 = pl.frag1.size() * sizeof(h8), b3 = 0;
  const size_t bc = pl.cinit.size() * sizeof(float), bC = sizeof(double) * (size_t)k * d;
  const size_t ball = b1 + b3 + bc + bC;
  if (c.up_pending) HIP_CHECK(hipEventSynchronize(c.up_event));
  c.h_up.ensure((ball + 15) / 16 * 16);
  char* hp = static_cast<char*>(c.h_up.p);
  memcpy(hp, pl.frag1.data(), b1);
  memcpy(hp + b1 + b3, pl.cinit.data(), bc);
  memcpy(hp + b1 + b3 + bc, C, bC);
  c.frag.ensure((ball + 15) / 16 * 16);
  {
    void* hdev = nullptr;
    HIP_CHECK(hipHostGetDevicePointer(&hdev, c.h_up.p, 0));
    const int64_t n16 = (int64_t)((ball + 15) / 16);
    hipLaunchKernelGGL(pull_host_big, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0,
                       c.stream, static_cast<const uint4*>(hdev), static_cast<uint4*>(c.frag.p),
                       n16);
    HIP_CHECK(hipGetLastError());
  }
  if (!c.up_event) HIP_CHECK(hipEventCreateWithFlags(&c.up_event, hipEventDisableTiming));
  HIP_CHECK(hipEventRecord(c.up_event, c.stream));
  c.up_pending = true;
  char* dp = static_cast<char*>(c.frag.p);
  const h8* dfrag1 = reinterpret_cast<const h8*>(dp);
  const float* dcin = reinterpret_cast<const float*>(dp + b1 + b3);
  const double* dC = reinterpret_cast<const double*>(dp + b1 + b3 + bc);

  // level 1: persistent, one kBigThreads workgroup per CU (LDS-bound)
  const size_t lds1 = big_l1_lds(k, d);
  const int64_t groups = (c.n + 63) / 64;
  const int wpb1 = kBigThreads / 64;
  const int nwg1 = (int)std::max<int64_t>(1, std::min<int64_t>(cus, (groups + wpb1 - 1) / wpb1));
  const int nw1 = nwg1 * wpb1;
  if (nw1 > kMaxRegions) return false;
  const int cap1 = (int)(((groups + nw1 - 1) / nw1) * 64);
  // L1 regions (point, best screen value); L2 overflow list (flat)
  const int nwg2 = cus * 2;
  const size_t slots = (size_t)nw1 * cap1;
  c.fb_list.ensure(sizeof(int32_t) * 3 * slots);
  c.fb_count.ensure(sizeof(int32_t) * (size_t)(nw1 + 2));
  HIP_CHECK(hipMemsetAsync(c.fb_count.p, 0, sizeof(int32_t) * (size_t)(nw1 + 2), c.stream));
  int32_t* list1 = c.fb_list.as<int32_t>();
  float* best1 = reinterpret_cast<float*>(list1 + slots);
  int32_t* ovf = list1 + 2 * slots;
  int32_t* cnt1 = c.fb_count.as<int32_t>();
  int32_t* ovf_count = cnt1 + nw1 + 1;
  c.fb_regions = nw1;
  c.fb_total_slot = nw1;  // L1 leftovers: the "fallback" statistic
  c.fb_layout = -1;       // screen32 must re-zero its counter layout
  BigArgs a;
  a.XT = c.xt32.as<float>();
  a.n = c.n;
  a.n_pad = c.n_pad;
  a.d = d;
  a.k = k;
  a.Q = Q;
  a.KB = KB;
  a.frag = dfrag1;
  a.cinit = dcin;
  a.thr0 = pl.thr1;
  a.thr_rel = pl.thr_rel;
  a.labels = c.labels.as<int32_t>();
  a.in_list = nullptr;
  a.in_count = nullptr;
  a.in_cap = 0;
  a.in_regions = 0;
  a.out_list = list1;
  a.out_best = best1;
  a.out_count = cnt1;
  a.out_cap = cap1;
  BigArgs a2 = a;  // L2 reads L1's regions and the same fragments / thresholds
  a2.in_list = list1;
  a2.in_count = cnt1;
  a2.in_cap = cap1;
  a2.in_regions = nw1;
  snprintf(c.prof_kernel, sizeof(c.prof_kernel), "screen_big<%d,1,false,true>", DQ);
  if (prof) prof_mark(c, 0);
  switch (DQ) {
    case 1: launch_big_levels<1>(c, a, a2, dim3(nwg1), dim3(nwg2), lds1, dC, ovf, ovf_count, prof); break;
    case 2: launch_big_levels<2>(c, a, a2, dim3(nwg1), dim3(nwg2), lds1, dC, ovf, ovf_count, prof); break;
    case 3: launch_big_levels<3>(c, a, a2, dim3(nwg1), dim3(nwg2), lds1, dC, ovf, ovf_count, prof); break;
    default: launch_big_levels<4>(c, a, a2, dim3(nwg1), dim3(nwg2), lds1, dC, ovf, ovf_count, prof); break;
  }
  hipLaunchKernelGGL(exact_big, dim3(cus * 4), dim3(64), 0, c.stream, c.x32.as<float>(), c.n_pad,
                     d, dC, k, ovf, ovf_count, c.labels.as<int32_t>());
  HIP_CHECK(hipGetLastError());
  // update from the labels
  const int len = k * (d + 1);
  HIP_CHECK(hipMemsetAsync(dout, 0, sizeof(long long) * len, c.stream));
  const int FG = big_fg(k);
  const int ngrp = (d + FG - 1) / FG;
  const size_t ldsu = (size_t)FG * k * 8 + (size_t)k * 4;
  const dim3 gu(cus, ngrp);
  static bool uattr = false;
  if (!uattr) {
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&update_big<16>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&update_big<8>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&update_big<4>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    uattr = true;
  }
  const double fx = std::ldexp(1.0, c.scale_bits);
  unsigned long long* uo = reinterpret_cast<unsigned long long*>(dout);
  if (FG == 16)
    hipLaunchKernelGGL(update_big<16>, gu, dim3(1024), ldsu, c.stream, c.x32.as<float>(), c.n,
                       c.n_pad, d, k, c.labels.as<int32_t>(), fx, uo);
  else if (FG == 8)
    hipLaunchKernelGGL(update_big<8>, gu, dim3(1024), ldsu, c.stream, c.x32.as<float>(), c.n,
                       c.n_pad, d, k, c.labels.as<int32_t>(), fx, uo);
  else
    hipLaunchKernelGGL(update_big<4>, gu, dim3(1024), ldsu, c.stream, c.x32.as<float>(), c.n,
                       c.n_pad, d, k, c.labels.as<int32_t>(), fx, uo);
  HIP_CHECK(hipGetLastError());
  c.run_valid = false;
  return true;
}

}  // namespace cdr
