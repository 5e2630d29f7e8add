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
  const h8* XB;         // screen_big_sp: fp16 B fragments per 64-point group (big_frag_copy)
  int64_t n, n_pad;
  int d, k, Q, KB;      // Q = stored feature quads, KB = ceil(k / 32)
  const h8* frag;       // NPROD 1: [KB][DQ][64]; NPROD 3: [KB][2][DQ][64]
  const float* cinit;   // [KB * 32] C operand per centroid row (1e30 past k)
  float thr0, thr_rel;
  const float* thr_dev;   // device plan: {thr0, thr_rel} in device memory (else the values above)
  const long long* gate;  // device loop state: nothing runs once gate[0] == 0
  unsigned jkeep;       // screen_big_sp: bits of a keyed value kept when its block is merged
  // DELTA steps (labels of the previous large-k step in place): a label is
  // written only when it changes, and the change {pt, old << 16 | new} goes
  // to L1's per-wave regions (mv1, same capacity as out_list) or, from L2 /
  // L3, to the flat list mv2 (count at mv2_count)
  int delta;
  int2* mv1;
  int32_t* mv1_count;
  int2* mv2;
  int32_t* mv2_count;
  const float* XA;      // the points row-major [n_pad][d4] (ensure_rowmajor)
  int d4;
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

// Centroid order inside a 32-row block: MFMA row r (the A-operand row of lane
// r and r + 32) holds centroid 32 b + big_row(r), chosen so that output value
// i of lane half h (row 8 (i >> 2) + 4 h + (i & 3)) is centroid 32 b + 16 h + i:
// a lane's keyed top-2 then carries the centroid's low bits directly.
__host__ __device__ inline int big_row(int r) { return 16 * ((r >> 2) & 1) + 4 * (r >> 3) + (r & 3); }

// DQ: 16-feature K chunks (d <= 16 DQ).  NPROD: 1 (A = -2 chi, B = xhi) or 3
// (A1 = -2 chi, A3 = -2 clo; A1 xhi + A1 xlo + A3 xhi).  GATHER: points come
// from the previous level's regions (a.in_*) instead of a dense sweep.
// ALDS: A fragments staged in LDS (L1) or read from global (L2).
constexpr int kBigThreads = 1024;  // L1: one workgroup per CU, 4 waves per SIMD

template <int DQ, int NPROD, bool GATHER, bool ALDS>
__global__ __launch_bounds__(kBigThreads) void screen_big(BigArgs a) {
  if (a.gate && a.gate[0] == 0) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const float thr0 = a.thr_dev ? a.thr_dev[0] : a.thr0;
  const float thr_rel = a.thr_dev ? a.thr_dev[1] : a.thr_rel;
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
        const int jb = 32 * b + 16 * h + ib;
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
    const bool cert = run > fmaf(best, thr_rel, thr0);  // NaN: never
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

// The L1 B fragments of every 64-point group, built once per point set from
// the pre-centred copy with the same fp16 conversion run_group applies
// (pack_h2): [g][t][c][lane] h8, lane (h, p) = features 16 c + 8 h .. + 8 of
// point 64 g + 32 t + p.  Half the bytes of the fp32 copy, and a wave's
// fragment loads are 1 KiB contiguous.
__global__ void big_frag_copy(const float* __restrict__ XT, int64_t n, int64_t n_pad, int Q,
                              int DQ, uint4* __restrict__ xb) {
  const f4* X4 = reinterpret_cast<const f4*>(XT);
  const int64_t total = (n_pad >> 6) * 2 * DQ * 64;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(e & 63);
    const int64_t r = e >> 6;
    const int c = (int)(r % DQ);
    const int64_t gt = r / DQ;
    const int t = (int)(gt & 1);
    const int64_t g = gt >> 1;
    const int h = lane >> 5, p = lane & 31;
    const int64_t pt = g * 64 + 32 * t + p;
    const int q0 = 4 * c + 2 * h;
    f4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
    if (pt < n && q0 < Q) v0 = X4[(int64_t)q0 * n_pad + pt];
    if (pt < n && q0 + 1 < Q) v1 = X4[(int64_t)(q0 + 1) * n_pad + pt];
    xb[e] = uint4{pack_h2(v0[0], v0[1]), pack_h2(v0[2], v0[3]), pack_h2(v1[0], v1[1]),
                  pack_h2(v1[2], v1[3])};
  }
}

// L1, software-pipelined (the product L1; screen_big<DQ, 1, false, true> is
// kept for comparisons, CDR_BIG_L1=0).  Per 32-centroid block a wave issues
// the block's MFMAs into one accumulator pair while it reduces the previous
// block's values from the other pair, so its own VALU runs beside its
// matrix work (PMC of the unpipelined kernel: MFMA busy 0.45 + VALU 0.38 of
// the cycles, i.e. serialised).  Keys: the local top-2 keys value i as
// (bits & ~15) | i (inline constants); with the row order of big_row, i is
// centroid 32 b + 16 h + i, so the block merge is one v_and_or that writes
// (b, h) above i, and the running (best, runner-up) keys carry the centroid
// index in their low JB bits (no separate index or float compare).
// NT threads per workgroup (one workgroup per CU): 768 = 3 waves per SIMD
// (<= 168 VGPRs), 512 = 2 waves per SIMD (<= 256 VGPRs, no spills at DQ = 4)
template <int DQ, int NT>
__global__ __launch_bounds__(NT) void screen_big_sp(BigArgs a) {
  if (a.gate && a.gate[0] == 0) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const float thr0 = a.thr_dev ? a.thr_dev[0] : a.thr0;
  const float thr_rel = a.thr_dev ? a.thr_dev[1] : a.thr_rel;
  float* scin = reinterpret_cast<float*>(smem);                     // [KB * 32]
  h8* sfrag = reinterpret_cast<h8*>(smem + (size_t)a.KB * 32 * 4);  // [KB][DQ][64]
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int p = lane & 31;
  for (int i = threadIdx.x; i < a.KB * 32; i += blockDim.x) scin[i] = a.cinit[i];
  {
    const int nf = a.KB * DQ * 64;
    for (int i = threadIdx.x; i < nf; i += blockDim.x) sfrag[i] = a.frag[i];
  }
  __syncthreads();
  const int wpb = blockDim.x >> 6;
  const int wave_id = blockIdx.x * wpb + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * wpb;
  int32_t* region = a.out_list + (size_t)wave_id * a.out_cap;
  float* region_best = a.out_best + (size_t)wave_id * a.out_cap;
  int used = 0;
  const h8* XB = a.XB;
  const unsigned jkeep = a.jkeep;
  const int KB = a.KB;
  const int64_t items = (a.n + 63) >> 6;
  // the group's B fragments: 2 DQ coalesced 16-byte loads per lane, the next
  // group's issued before this group's blocks (one group of prefetch)
  h8 BN[2][DQ];
  auto fetch = [&](int64_t gg) {
    if (gg < items) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < DQ; ++c) BN[t][c] = XB[((gg * 2 + t) * DQ + c) * 64 + lane];
    }
  };
  fetch(wave_id);
  int2* mv_region = a.delta ? a.mv1 + (size_t)wave_id * a.out_cap : nullptr;
  int mv_used = 0;
  for (int64_t g = wave_id; g < items; g += nwaves) {
    const int64_t base = g << 6;
    const int64_t pt[2] = {base + p, base + 32 + p};
    const bool real[2] = {pt[0] < a.n, pt[1] < a.n};
    // DELTA: the previous label of this lane's point (after the swap below:
    // lanes < 32 tile 0's point, lanes >= 32 tile 1's), loaded now
    const int64_t lpt = base + lane;
    const int oldl = a.delta && lpt < a.n ? a.labels[lpt] : -1;
    h8 BH[2][DQ];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int c = 0; c < DQ; ++c) BH[t][c] = BN[t][c];
    fetch(g + nwaves);
    unsigned RB[2] = {~0u, ~0u}, RS[2] = {~0u, ~0u};
    // the block's MFMAs: C operand rows from LDS, A fragments from LDS
    auto mm = [&](int b, f16v (&acc)[2]) {
      const f4* cr = reinterpret_cast<const f4*>(scin + 32 * b + 4 * h);
      f16v ci;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f4 v = cr[2 * q];  // rows 8q + 4h .. + 4
#pragma unroll
        for (int i = 0; i < 4; ++i) ci[4 * q + i] = v[i];
      }
      h8 A[DQ];
#pragma unroll
      for (int c = 0; c < DQ; ++c) A[c] = sfrag[((size_t)b * DQ + c) * 64 + lane];
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[0], BH[0][0], ci, 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[0], BH[1][0], ci, 0, 0, 0);
#pragma unroll
      for (int c = 1; c < DQ; ++c) {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[c], BH[0][c], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[c], BH[1][c], acc[1], 0, 0, 0);
      }
    };
    // keyed top-2 of each tile's 16 values (all >= 0: bits order), merged
    // into the running keys with the block and lane half written above i
    auto red = [&](int b, const f16v (&acc)[2]) {
      const unsigned bo = ((unsigned)b << 5) | ((unsigned)h << 4);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
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
        const unsigned kj = (kb & jkeep) | bo;
        unsigned ms;
        asm("v_min3_u32 %0, %1, %2, %3" : "=v"(ms) : "v"(max(RB[t], kj)), "v"(RS[t]), "v"(ks));
        RS[t] = ms;
        RB[t] = min(RB[t], kj);
      }
    };
    f16v accA[2], accB[2];
    mm(0, accA);
    int b = 1;
    for (; b + 1 < KB; b += 2) {
      mm(b, accB);
      red(b - 1, accA);
      mm(b + 1, accA);
      red(b, accB);
    }
    if (b < KB) {
      mm(b, accB);
      red(b - 1, accA);
      red(b, accB);
    } else {
      red(b - 1, accA);
    }
    // lanes < 32 end with tile 0's point p (both halves), lanes >= 32 with
    // tile 1's
    unsigned b0 = RB[0], b1 = RB[1], s0 = RS[0], s1 = RS[1];
    swap32(b0, b1);
    swap32(s0, s1);
    const unsigned kbest = min(b0, b1);
    unsigned krun;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(krun) : "v"(max(b0, b1)), "v"(s0), "v"(s1));
    const float best = __uint_as_float(kbest);
    const int label = (int)(kbest & ~jkeep) | (int)(kbest & 15u);
    const int64_t mypt = h == 0 ? pt[0] : pt[1];
    const bool myreal = h == 0 ? real[0] : real[1];
    // rows past k carry C = 1e30: never best, never a close runner-up
    const bool cert = __uint_as_float(krun) > fmaf(best, thr_rel, thr0);
    if (!a.delta) {
      if (myreal && cert) a.labels[mypt] = label;
    } else {
      const bool moved = myreal && cert && label != oldl;
      if (moved) a.labels[mypt] = label;
      const unsigned long long mvb = __ballot(moved);
      if (mvb) {
        const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(mvb >> 32),
                                                __builtin_amdgcn_mbcnt_lo((unsigned)mvb, 0u));
        if (moved) mv_region[mv_used + r] = int2{(int)mypt, (oldl << 16) | label};
        mv_used += __popcll(mvb);
      }
    }
    const unsigned long long need = __ballot(myreal && !cert);
    if (need) {
      const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(need >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((unsigned)need, 0u));
      if (myreal && !cert) {
        region[used + rank] = (int32_t)mypt;
        region_best[used + rank] = best;
      }
      used += __popcll(need);
    }
  }
  if (lane == 0) {
    a.out_count[wave_id] = used;
    if (used) atomicAdd(a.out_count + nwaves, used);
    if (a.delta) a.mv1_count[wave_id] = mv_used;
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
// np_sqdist (exact_math.h) for d >= 8 with the point's features in
// registers (DMAX >= d, a compile-time bound so every index is static)
template <int DMAX>
__device__ __forceinline__ double np_sqdist_reg(const float (&x)[DMAX],
                                                const double* __restrict__ cj, int d) {
  double r[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const double t = (double)x[i] - cj[i];
    r[i] = t * t;
  }
  const int dd = d - (d & 7);
#pragma unroll
  for (int f = 8; f < DMAX; f += 8) {
    if (f < dd) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const double t = (double)x[f + i] - cj[f + i];
        r[i] = r[i] + t * t;
      }
    }
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
  for (int f = 8; f < DMAX; ++f) {
    if (f >= dd && f < d) {
      const double t = (double)x[f] - cj[f];
      res = res + t * t;
    }
  }
  return res;
}

constexpr int kMaxCand = 16;
constexpr int kMaxRegions = 8192;  // L1 waves (regions) the candidate level can index

template <int DQ>
__global__ __launch_bounds__(256) void cand_big(BigArgs a, const float* __restrict__ X0,
                                                const double* __restrict__ C64,
                                                int32_t* __restrict__ ovf,
                                                int32_t* __restrict__ ovf_count, int abl) {
  if (a.gate && a.gate[0] == 0) return;
  const float thr0 = a.thr_dev ? a.thr_dev[0] : a.thr0;
  const float thr_rel = a.thr_dev ? a.thr_dev[1] : a.thr_rel;
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
        lim[t] = real[t] ? fmaf(srcb[e], thr_rel, thr0) : -1.0f;
      }
      scnt[w][lane] = 0;
      h8 BH[2][DQ];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < DQ; ++c) {
          if (a.XB) {
            // the point's fragment in its group's block of the fp16 copy (one
            // 8 KB block per point, not DQ pages of the fp32 copy)
            const int64_t q = pt[t];
            const int64_t idx = (((q >> 6) * 2 + ((q >> 5) & 1)) * DQ + c) * 64 + h * 32 + (q & 31);
            BH[t][c] = real[t] ? a.XB[idx] : h8{};
          } else {
            const int q0 = 4 * c + 2 * h;
            f4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
            if (real[t] && q0 < a.Q) v0 = X4[(int64_t)q0 * a.n_pad + pt[t]];
            if (real[t] && q0 + 1 < a.Q) v1 = X4[(int64_t)(q0 + 1) * a.n_pad + pt[t]];
            u4v H = {pack_h2(v0[0], v0[1]), pack_h2(v0[2], v0[3]), pack_h2(v1[0], v1[1]),
                     pack_h2(v1[2], v1[3])};
            BH[t][c] = __builtin_bit_cast(h8, H);
          }
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
              const int j = 32 * b + 16 * h + i;
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
          // the point's features once (one batch of quad loads), then each
          // candidate's fp64 row (L2-resident) in NumPy's pairwise order
          float xv[16 * DQ];
          const f4* X04 = reinterpret_cast<const f4*>(X0);
          const f4* XA4 = reinterpret_cast<const f4*>(a.XA);
#pragma unroll
          for (int q = 0; q < 4 * DQ; ++q) {
            f4 v = {0.f, 0.f, 0.f, 0.f};
            if (q < a.Q) v = XA4 ? XA4[mypt * a.Q + q] : X04[(int64_t)q * a.n_pad + mypt];
#pragma unroll
            for (int i = 0; i < 4; ++i) xv[4 * q + i] = v[i];
          }
          double rb = INFINITY;
          int jb = 0x7fffffff;
          for (int s2 = 0; s2 < nc; ++s2) {
            const int j = scand[w][lane * kMaxCand + s2];
            const double R = np_sqdist_reg<16 * DQ>(xv, C64 + (size_t)j * a.d, a.d);
            const double root = sqrt(R);
            if (root < rb || (root == rb && j < jb)) {
              rb = root;
              jb = j;
            }
          }
          if (!a.delta) {
            a.labels[mypt] = jb;
          } else {
            const int oldl = a.labels[mypt];
            if (jb != oldl) {
              a.labels[mypt] = jb;
              a.mv2[atomicAdd(a.mv2_count, 1)] = int2{(int)mypt, (oldl << 16) | jb};
            }
          }
        }
      }
    }
  }
}

// L2 with the A fragments and C rows in LDS (the product L2 after
// screen_big_sp; cand_big reads them from global memory per chunk, 7x L1's
// cost per point).  One NT-thread workgroup per CU; the chunk numbering of
// L1's regions comes from big_chunk_prefix (global memory: the LDS holds the
// fragments).  Per chunk of 64 points: the same one-product screen as L1
// (bit-identical: same fragments, same B operands from xb16), candidates
// S_j <= best thr_rel + T1 into per-point LDS lists (u16), then the exact
// fp64 evaluation of each point's candidates as cand_big.
__global__ __launch_bounds__(1024) void big_chunk_prefix(const int32_t* __restrict__ cnt, int R,
                                                         int32_t* __restrict__ pre) {
  __shared__ int wsum[16];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int r0 = 0; r0 < R; r0 += 1024) {
    const int r = r0 + threadIdx.x;
    const int v = r < R ? (cnt[r] + 63) >> 6 : 0;
    int inc = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(inc, o);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int base = carry;
    for (int q = 0; q < w; ++q) base += wsum[q];
    if (r < R) pre[r] = base + inc - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = base + inc;
    __syncthreads();
  }
  if (threadIdx.x == 0) pre[R] = carry;
}

template <int DQ, int NT>
__global__ __launch_bounds__(NT) void cand_big_lds(BigArgs a, const double* __restrict__ C64,
                                                   const int32_t* __restrict__ chunk_pre,
                                                   int32_t* __restrict__ ovf,
                                                   int32_t* __restrict__ ovf_count) {
  if (a.gate && a.gate[0] == 0) return;
  constexpr int NW = NT / 64;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* scin = reinterpret_cast<float*>(smem);                     // [KB * 32]
  h8* sfrag = reinterpret_cast<h8*>(smem + (size_t)a.KB * 32 * 4);  // [KB][DQ][64]
  int* scnt = reinterpret_cast<int*>(sfrag + (size_t)a.KB * DQ * 64);  // [NW][64]
  unsigned short* scand = reinterpret_cast<unsigned short*>(scnt + NW * 64);  // [NW][64][kMaxCand]
  const float thr0 = a.thr_dev ? a.thr_dev[0] : a.thr0;
  const float thr_rel = a.thr_dev ? a.thr_dev[1] : a.thr_rel;
  const int R = a.in_regions;
  const int nchunks = chunk_pre[R];
  if (nchunks == 0) return;  // uniform over the grid
  for (int i = threadIdx.x; i < a.KB * 32; i += blockDim.x) scin[i] = a.cinit[i];
  for (int i = threadIdx.x; i < a.KB * DQ * 64; i += blockDim.x) sfrag[i] = a.frag[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int h = lane >> 5;
  const int p = lane & 31;
  const int wave_id = blockIdx.x * NW + w;
  const int nwaves = gridDim.x * NW;
  int* mycnt = scnt + w * 64;
  unsigned short* mycand = scand + (size_t)w * 64 * kMaxCand;
  const f4* XA4 = reinterpret_cast<const f4*>(a.XA);
  for (int ch = wave_id; ch < nchunks; ch += nwaves) {
    int lo = 0, hi = R;  // last r with chunk_pre[r] <= ch
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (chunk_pre[mid] <= ch) lo = mid; else hi = mid;
    }
    const int r = lo;
    const int cnt = a.in_count[r];
    const int e0 = (ch - chunk_pre[r]) * 64;
    const int32_t* src = a.in_list + (size_t)r * a.in_cap;
    const float* srcb = a.out_best + (size_t)r * a.in_cap;
    int64_t pt[2];
    bool real[2];
    float lim[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int e = e0 + 32 * t + p;
      real[t] = e < cnt;
      pt[t] = real[t] ? (int64_t)src[e] : 0;
      lim[t] = real[t] ? fmaf(srcb[e], thr_rel, thr0) : -1.0f;
    }
    mycnt[lane] = 0;
    h8 BH[2][DQ];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int c = 0; c < DQ; ++c) {
        const int64_t q = pt[t];
        const int64_t idx = (((q >> 6) * 2 + ((q >> 5) & 1)) * DQ + c) * 64 + h * 32 + (q & 31);
        BH[t][c] = real[t] ? a.XB[idx] : h8{};
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    auto mm = [&](int b, f16v (&acc)[2]) {
      const f4* cr = reinterpret_cast<const f4*>(scin + 32 * b + 4 * h);
      f16v ci;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f4 v = cr[2 * q];
#pragma unroll
        for (int i = 0; i < 4; ++i) ci[4 * q + i] = v[i];
      }
      h8 A[DQ];
#pragma unroll
      for (int c = 0; c < DQ; ++c) A[c] = sfrag[((size_t)b * DQ + c) * 64 + lane];
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[0], BH[0][0], ci, 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[0], BH[1][0], ci, 0, 0, 0);
#pragma unroll
      for (int c = 1; c < DQ; ++c) {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[c], BH[0][c], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[c], BH[1][c], acc[1], 0, 0, 0);
      }
    };
    auto take = [&](int b, const f16v (&acc)[2]) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (acc[t][i] <= lim[t]) {
            const int slot = atomicAdd(&mycnt[32 * t + p], 1);
            if (slot < kMaxCand)
              mycand[(32 * t + p) * kMaxCand + slot] = (unsigned short)(32 * b + 16 * h + i);
          }
    };
    f16v accA[2], accB[2];
    mm(0, accA);
    int b = 1;
    for (; b + 1 < a.KB; b += 2) {
      mm(b, accB);
      take(b - 1, accA);
      mm(b + 1, accA);
      take(b, accB);
    }
    if (b < a.KB) {
      mm(b, accB);
      take(b - 1, accA);
      take(b, accB);
    } else {
      take(b - 1, accA);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // lane l: point l of the chunk (tile l / 32, column l % 32)
    const int e = e0 + lane;
    if (e < cnt) {
      const int64_t mypt = (int64_t)src[e];
      const int nc = mycnt[lane];
      if (nc > kMaxCand || nc == 0) {
        ovf[atomicAdd(ovf_count, 1)] = (int32_t)mypt;
      } else {
        float xv[16 * DQ];
#pragma unroll
        for (int q = 0; q < 4 * DQ; ++q) {
          const f4 v = q < a.Q ? XA4[mypt * a.Q + q] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int i = 0; i < 4; ++i) xv[4 * q + i] = v[i];
        }
        double rb = INFINITY;
        int jb = 0x7fffffff;
        for (int s2 = 0; s2 < nc; ++s2) {
          const int j = mycand[lane * kMaxCand + s2];
          const double Rd = np_sqdist_reg<16 * DQ>(xv, C64 + (size_t)j * a.d, a.d);
          const double root = sqrt(Rd);
          if (root < rb || (root == rb && j < jb)) {
            rb = root;
            jb = j;
          }
        }
        if (!a.delta) {
          a.labels[mypt] = jb;
        } else {
          const int oldl = a.labels[mypt];
          if (jb != oldl) {
            a.labels[mypt] = jb;
            a.mv2[atomicAdd(a.mv2_count, 1)] = int2{(int)mypt, (oldl << 16) | jb};
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
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
                                                int32_t* __restrict__ labels,
                                                const long long* __restrict__ gate,
                                                int2* __restrict__ mv2,
                                                int32_t* __restrict__ mv2_count) {
  if (gate && gate[0] == 0) return;
  __shared__ double sx[128];
  const int lane = threadIdx.x;
  const int c8 = lane >> 3, r = lane & 7;
  const int dd = d - (d & 7);
  const int total = *count;
  for (int e = blockIdx.x; e < total; e += gridDim.x) {
    const int64_t pt = list[e];
    __syncthreads();
    for (int f = lane; f < d; f += 64) sx[f] = (double)X[xidx(X, f, pt, n_pad)];
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
    if (lane == 0) {
      const int jl = jmin < k ? jmin : 0;
      if (!mv2) {
        labels[pt] = jl;
      } else {  // DELTA step: record a change
        const int oldl = labels[pt];
        if (jl != oldl) {
          labels[pt] = jl;
          mv2[atomicAdd(mv2_count, 1)] = int2{(int)pt, (oldl << 16) | jl};
        }
      }
    }
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
                                                   double fx, unsigned long long* __restrict__ out,
                                                   const long long* __restrict__ gate) {
  if (gate && gate[0] == 0) return;
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

__global__ void zero_big_gated(long long* __restrict__ p, int64_t n,
                               const long long* __restrict__ gate) {
  if (gate && gate[0] == 0) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 0;
}

// DELTA update: the moves {pt, old << 16 | new} of L1's per-wave regions
// (mv1, counts cnt1) and of L2 / L3 (flat mv2, count *cnt2) applied to the
// running (k, d+1) int64 sums: +x into the new cluster, -x out of the old,
// x gathered from the row-major copy.  blockIdx.y = feature group (FG
// features), blockIdx.x = slice of the moves; an LDS table [FG][k] of fp64
// (exact: grid values) per workgroup, then its nonzero cells as exact int64
// fixed point with atomics.  Integer sums: equal to a full recompute.
constexpr int kFixSlices = 32;

template <int FG>
__global__ __launch_bounds__(1024) void fixup_big(const float* __restrict__ XA, int d4, int d,
                                                  int k, const int2* __restrict__ mv1,
                                                  const int32_t* __restrict__ cnt1, int nw1,
                                                  int cap1, const int2* __restrict__ mv2,
                                                  const int32_t* __restrict__ cnt2, double fx,
                                                  unsigned long long* __restrict__ out,
                                                  const long long* __restrict__ gate) {
  if (gate && gate[0] == 0) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* tsum = reinterpret_cast<double*>(smem);              // [FG][k]
  int* tcnt = reinterpret_cast<int*>(tsum + (size_t)FG * k);   // [k]
  const int g = blockIdx.y, f0 = FG * g;
  const int G = gridDim.x, sl = blockIdx.x;
  for (int i = threadIdx.x; i < FG * k; i += blockDim.x) tsum[i] = 0.0;
  for (int i = threadIdx.x; i < k; i += blockDim.x) tcnt[i] = 0;
  __syncthreads();
  auto apply = [&](const int2* list, int64_t cnt) {
    for (int64_t idx = threadIdx.x; idx < cnt * FG; idx += blockDim.x) {
      const int64_t e = idx / FG;
      const int ff = (int)(idx - e * FG);
      const int f = f0 + ff;
      const int2 m = list[e];
      const int oldl = (int)((unsigned)m.y >> 16), newl = m.y & 0xFFFF;
      if (f < d) {
        const double x = (double)XA[(int64_t)m.x * d4 + f];
        atomicAdd(&tsum[ff * k + newl], x);
        atomicAdd(&tsum[ff * k + oldl], -x);
      }
      if (ff == 0 && g == 0) {
        atomicAdd(&tcnt[newl], 1);
        atomicAdd(&tcnt[oldl], -1);
      }
    }
  };
  for (int r = sl; r < nw1; r += G) apply(mv1 + (size_t)r * cap1, cnt1[r]);
  {
    const int64_t n2 = *cnt2, per = (n2 + G - 1) / G;
    const int64_t e0 = (int64_t)sl * per, e1 = min(n2, e0 + per);
    if (e1 > e0) apply(mv2 + e0, e1 - e0);
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
void ensure_rowmajor(Ctx& c);

static int big_dq(int d) { return (d + 15) / 16; }
// L1 workgroup size: 3 waves per SIMD while the pipelined kernel fits 168
// VGPRs (DQ <= 2), else 2 (CDR_BIG_SP_NT=512|768 overrides, for comparisons)
static int big_sp_threads(int DQ) {
  static const int env = exp_env("CDR_BIG_SP_NT") ? std::atoi(exp_env("CDR_BIG_SP_NT")) : 0;
  if (env == 512 || env == 768) return env;
  return DQ <= 2 ? 768 : 512;
}
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
  int jbits;
};

// Rigorous screen error bounds (see the file header); mirrors build_plan32's
// terms with N = fp32 additions in the MFMA chain.  Shared by the host plan
// (build_plan_big) and the device plan (big_plan_kernel): the same fp64
// operations in the same order, so both give the same bits.
struct BigBounds {
  double D;
  float thr1, thr3, thr_rel;
  int jbits;
};

__host__ __device__ inline BigBounds big_bounds(double ccmax, double l1c, double xxmax,
                                                double l1x, int DQ, int KB) {
  BigBounds r;
  const double u = ldexp(1.0, -24);
  const double eps = ldexp(1.0, -11), eta = ldexp(1.0, -25);
  const double cx = sqrt(ccmax * xxmax);
  // one product: |c.x - chi.xhi| <= 2 eps (1 + eps) ||c|| ||x|| + eta (l1x + (1 + eps) l1c)
  const double P1 = 2.0 * eps * (1.0 + eps) * cx + eta * (l1x + (1.0 + eps) * l1c);
  const double N1 = 16.0 * DQ + 1.0, N3 = 3.0 * 16.0 * DQ + 1.0;
  const double g1 = 2.0 * u * N1 / (1.0 - 2.0 * u * N1);
  const double g3 = 2.0 * u * N3 / (1.0 - 2.0 * u * N3);
  const double E1a = 2.0 * P1 + g1 * (ccmax + 2.0 * xxmax + 4.0 * cx + 4.0) + u * (ccmax + 2.0 * xxmax + 4.0);
  // D >= max ||xhat||^2 + margin keeps every screen value >= 0
  const double D = xxmax + 4.0 * E1a + ldexp(1.0, -20);
  const double sum1 = (ccmax + D) * (1.0 + u) + 2.0 * (1.0 + eps) * (1.0 + eps) * cx;
  const double E1 = 2.0 * P1 + g1 * sum1 + u * (ccmax + D) + ldexp(1.0, -46) * (ccmax + D);
  // three products: the split leaves |c.x - (chi xhi + chi xlo + clo xhi)| <=
  // 2.4 2^-22 ||c|| ||x|| + 2^-24 (l1c + l1x)
  const double P3 = 2.4 * ldexp(1.0, -22) * cx + ldexp(1.0, -24) * (l1c + l1x);
  const double sum3 = (ccmax + D) * (1.0 + u) + 2.0 * (1.0 + ldexp(1.0, -9)) * cx;
  const double E3 = 2.0 * P3 + g3 * sum3 + u * (ccmax + D) + ldexp(1.0, -46) * (ccmax + D);
  // reference slack: the fp64 distances and roots must not tie or flip
  const double Wmax = (sqrt(ccmax) + sqrt(xxmax)) * (sqrt(ccmax) + sqrt(xxmax));
  const double slack = ldexp(Wmax + 1.0, -38);
  r.D = D;
  r.thr1 = (float)((2.0 * E1 + slack) * 1.001);
  r.thr3 = (float)((2.0 * E3 + slack) * 1.001);
  // keys keep the centroid index in their low JB bits (screen_big_sp): best
  // and runner-up are each within 2^JB ulps (2^(JB-23) relative) of their
  // screen values, covered by 1 + 4 * 2^(JB-23); >= the old kernel's 16-ulp need
  int JB = 5;
  while ((1 << (JB - 5)) < KB) ++JB;
  r.jbits = JB;
  r.thr_rel = 1.0f + ldexpf(1.0f, JB - 21);
  return r;
}

// The point side of the bounds: max ||xhat||^2 (with a 1e-6 margin) and max
// ||xhat||_1 over the data's bounding box.
static void big_point_side(const Ctx& c, double& xxmax, double& l1x) {
  const double sc = std::ldexp(1.0, c.sigma);
  xxmax = 0.0;
  l1x = 0.0;
  for (int f = 0; f < c.d; ++f) {
    const double dev =
        std::fmax(c.fmax[f] - (double)c.mu[f], (double)c.mu[f] - c.fmin[f]) * sc;
    xxmax += dev * dev;
    l1x += dev;
  }
  xxmax *= 1.0 + 1e-6;
}

// A1 fragment of one lane of centroid block b, feature chunk cq (the L1 / L2
// A operand: -2 chi, rows in big_row order).
__host__ __device__ inline h8 big_frag_lane(const double* C, const double* mu, double sc, int k,
                                            int d, int b, int cq, int lane) {
  const int j = 32 * b + big_row(lane & 31);
  const int hh = lane >> 5;
  h8 A1 = {};
  for (int i = 0; i < 8; ++i) {
    const int f = 16 * cq + 8 * hh + i;
    if (j >= k || f >= d) continue;
    const double v = (C[(size_t)j * d + f] - mu[f]) * sc;
    const _Float16 hi = f64_to_f16(v);
    A1[i] = f64_to_f16(-2.0 * (double)hi);
  }
  return A1;
}

static void build_plan_big(const Ctx& c, const double* C, int k, PlanBig& pl) {
  const int d = c.d, DQ = big_dq(d), KB = (k + 31) / 32;
  const double sc = std::ldexp(1.0, c.sigma);
  std::vector<double> mu(d), cc(k, 0.0);
  for (int f = 0; f < d; ++f) mu[f] = (double)c.mu[f];
  double ccmax = 0.0, l1c = 0.0;
  for (int j = 0; j < k; ++j) {
    double s = 0.0, l1 = 0.0;
    for (int f = 0; f < d; ++f) {
      const double v = (C[(size_t)j * d + f] - mu[f]) * sc;
      s += v * v;
      l1 += std::fabs(v);
    }
    cc[j] = s;
    ccmax = std::fmax(ccmax, s);
    l1c = std::fmax(l1c, l1);
  }
  double xxmax, l1x;
  big_point_side(c, xxmax, l1x);
  const BigBounds bb = big_bounds(ccmax, l1c, xxmax, l1x, DQ, KB);
  pl.thr1 = bb.thr1;
  pl.thr3 = bb.thr3;
  pl.thr_rel = bb.thr_rel;
  pl.jbits = bb.jbits;
  pl.cinit.assign((size_t)KB * 32, 1.0e30f);
  for (int r = 0; r < KB * 32; ++r) {
    const int j = 32 * (r / 32) + big_row(r % 32);
    if (j < k) pl.cinit[r] = (float)(cc[j] + bb.D);
  }
  pl.frag1.assign((size_t)KB * DQ * 64, h8{});
  for (int b = 0; b < KB; ++b)
    for (int cq = 0; cq < DQ; ++cq)
      for (int lane = 0; lane < 64; ++lane)
        pl.frag1[((size_t)b * DQ + cq) * 64 + lane] =
            big_frag_lane(C, mu.data(), sc, k, d, b, cq, lane);
}

// Device-resident loop (loop.hip): the same plan built on the device from the
// loop's centroids, into the layout big_step uploads (frag1 | cinit | C |
// {thr1, thr_rel}).  One 1024-thread workgroup; gated on the loop state.
struct BigPlanArgs {
  const double* C;
  const double* mu;  // double[d]
  double sc, xxmax, l1x;
  int k, d, DQ, KB;
  h8* frag1;
  float* cinit;
  double* C64;
  float* thr;
  const long long* gate;
};

__global__ __launch_bounds__(1024) void big_plan_kernel(BigPlanArgs a) {
  if (a.gate && a.gate[0] == 0) return;
  extern __shared__ double scc[];  // [k]
  __shared__ double rmax[2][16];
  __shared__ double sD;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int k = a.k, d = a.d;
  double m0 = 0.0, m1 = 0.0;
  for (int j = t; j < k; j += blockDim.x) {
    double s = 0.0, l1 = 0.0;
    for (int f = 0; f < d; ++f) {
      const double v = (a.C[(size_t)j * d + f] - a.mu[f]) * a.sc;
      s += v * v;
      l1 += fabs(v);
    }
    scc[j] = s;
    m0 = fmax(m0, s);
    m1 = fmax(m1, l1);
  }
  for (int o = 32; o > 0; o >>= 1) {
    m0 = fmax(m0, __shfl_xor(m0, o));
    m1 = fmax(m1, __shfl_xor(m1, o));
  }
  if (lane == 0) {
    rmax[0][w] = m0;
    rmax[1][w] = m1;
  }
  __syncthreads();
  if (t == 0) {
    double ccmax = 0.0, l1c = 0.0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      ccmax = fmax(ccmax, rmax[0][i]);
      l1c = fmax(l1c, rmax[1][i]);
    }
    const BigBounds bb = big_bounds(ccmax, l1c, a.xxmax, a.l1x, a.DQ, a.KB);
    sD = bb.D;
    a.thr[0] = bb.thr1;
    a.thr[1] = bb.thr_rel;
  }
  __syncthreads();
  const double D = sD;
  for (int r = t; r < a.KB * 32; r += blockDim.x) {
    const int j = 32 * (r / 32) + big_row(r % 32);
    a.cinit[r] = j < k ? (float)(scc[j] + D) : 1.0e30f;
  }
  for (int e = t; e < a.KB * a.DQ * 64; e += blockDim.x) {
    const int l = e & 63, bc = e >> 6;
    a.frag1[e] = big_frag_lane(a.C, a.mu, a.sc, k, d, bc / a.DQ, bc % a.DQ, l);
  }
  for (int e = t; e < k * d; e += blockDim.x) a.C64[e] = a.C[e];
}

template <int DQ>
static void launch_big_levels(Ctx& c, const BigArgs& a1, const BigArgs& a2, dim3 g1, dim3 g2,
                              size_t lds1, const double* dC, int32_t* ovf, int32_t* ovf_count,
                              bool prof, bool sp, int32_t* chunk_pre) {
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&screen_big<DQ, 1, false, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&screen_big_sp<DQ, 512>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&screen_big_sp<DQ, 768>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  if (sp && big_sp_threads(DQ) == 768)
    hipLaunchKernelGGL((screen_big_sp<DQ, 768>), g1, dim3(768), lds1, c.stream, a1);
  else if (sp)
    hipLaunchKernelGGL((screen_big_sp<DQ, 512>), g1, dim3(512), lds1, c.stream, a1);
  else
    hipLaunchKernelGGL((screen_big<DQ, 1, false, true>), g1, dim3(kBigThreads), lds1, c.stream,
                       a1);
  HIP_CHECK(hipGetLastError());
  if (prof) prof_mark(c, 1);  // the L1 screen alone
#ifdef CDR_EXPERIMENTS
  static const int abl = exp_env("CDR_BIG_ABL") ? std::atoi(exp_env("CDR_BIG_ABL")) : 0;
#else
  constexpr int abl = 0;
#endif
  const size_t lds2 = big_l1_lds(a2.k, a2.d) + (size_t)8 * 64 * 4 + (size_t)8 * 64 * kMaxCand * 2;
  if (sp && lds2 <= 160 * 1024) {
    // L2 on LDS-resident fragments: chunk numbering first (global), then
    // one workgroup per CU
    int32_t* pre = chunk_pre;
    hipLaunchKernelGGL(big_chunk_prefix, dim3(1), dim3(1024), 0, c.stream, a2.in_count,
                       a2.in_regions, pre);
    static bool lattr = false;
    if (!lattr) {
      HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&cand_big_lds<DQ, 512>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      lattr = true;
    }
    hipLaunchKernelGGL((cand_big_lds<DQ, 512>), dim3(lloyd_num_cus(c.device)), dim3(512), lds2,
                       c.stream, a2, dC, pre, ovf, ovf_count);
  } else {
    hipLaunchKernelGGL((cand_big<DQ>), g2, dim3(256), 0, c.stream, a2, c.x32.as<float>(), dC, ovf,
                       ovf_count, abl);
  }
  HIP_CHECK(hipGetLastError());
}

// One F32X Lloyd step in the large regime: labels for every point and the
// exact int64 (k, d+1) sums/counts in dout (device).  Returns false when the
// shape is not covered (nothing launched).
// Plan buffer layout (c.frag): frag1 | cinit | C (fp64) | {thr1, thr_rel}.
struct BigLayout {
  size_t b1, bc, bC, bt, all;
};
static BigLayout big_layout(int k, int d) {
  const int DQ = big_dq(d), KB = (k + 31) / 32;
  BigLayout l;
  l.b1 = (size_t)KB * DQ * 64 * sizeof(h8);
  l.bc = (size_t)KB * 32 * sizeof(float);
  l.bC = sizeof(double) * (size_t)k * d;
  l.bt = 16;
  l.all = (l.b1 + l.bc + l.bC + l.bt + 15) / 16 * 16;
  return l;
}

static bool big_launch(Ctx& c, int k, float thr1, float thr_rel, const float* thr_dev,
                       const long long* gate, long long* dout, bool prof);

bool big_step(Ctx& c, const double* C, int k, long long* dout, bool prof) {
  if (!big_supported(c, k)) return false;
  ensure_precentered(c);
  PlanBig pl;
  build_plan_big(c, C, k, pl);
  const int d = c.d;
  const BigLayout L = big_layout(k, d);
  // one upload: frag1 | cinit | C (fp64)
  if (c.up_pending) HIP_CHECK(hipEventSynchronize(c.up_event));
  c.h_up.ensure(L.all);
  char* hp = static_cast<char*>(c.h_up.p);
  memcpy(hp, pl.frag1.data(), L.b1);
  memcpy(hp + L.b1, pl.cinit.data(), L.bc);
  memcpy(hp + L.b1 + L.bc, C, L.bC);
  c.frag.ensure(L.all);
  {
    void* hdev = nullptr;
    HIP_CHECK(hipHostGetDevicePointer(&hdev, c.h_up.p, 0));
    const int64_t n16 = (int64_t)((L.b1 + L.bc + L.bC + 15) / 16);
    hipLaunchKernelGGL(pull_host_big, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0,
                       c.stream, static_cast<const uint4*>(hdev), static_cast<uint4*>(c.frag.p),
                       n16);
    HIP_CHECK(hipGetLastError());
  }
  if (!c.up_event) HIP_CHECK(hipEventCreateWithFlags(&c.up_event, hipEventDisableTiming));
  HIP_CHECK(hipEventRecord(c.up_event, c.stream));
  c.up_pending = true;
  return big_launch(c, k, pl.thr1, pl.thr_rel, nullptr, nullptr, dout, prof);
}

// The device-resident loop's plan (loop.hip): built on the device from the
// loop's centroids dC (fp64, k x d) into c.frag; gate = the loop state.
void big_plan_device(Ctx& c, int k, const double* dC, const double* dmu, const long long* gate) {
  const int d = c.d, DQ = big_dq(d), KB = (k + 31) / 32;
  const BigLayout L = big_layout(k, d);
  c.frag.ensure(L.all);
  char* dp = static_cast<char*>(c.frag.p);
  BigPlanArgs a;
  a.C = dC;
  a.mu = dmu;
  a.sc = std::ldexp(1.0, c.sigma);
  big_point_side(c, a.xxmax, a.l1x);
  a.k = k;
  a.d = d;
  a.DQ = DQ;
  a.KB = KB;
  a.frag1 = reinterpret_cast<h8*>(dp);
  a.cinit = reinterpret_cast<float*>(dp + L.b1);
  a.C64 = reinterpret_cast<double*>(dp + L.b1 + L.bc);
  a.thr = reinterpret_cast<float*>(dp + L.b1 + L.bc + L.bC);
  a.gate = gate;
  hipLaunchKernelGGL(big_plan_kernel, dim3(1), dim3(1024), sizeof(double) * (size_t)k, c.stream,
                     a);
  HIP_CHECK(hipGetLastError());
}

// One step on the device plan in c.frag (no host round trip); gate as above.
bool big_step_dev(Ctx& c, int k, long long* dout, bool prof, const long long* gate) {
  if (!big_supported(c, k)) return false;
  ensure_precentered(c);
  const BigLayout L = big_layout(k, c.d);
  const float* thr = reinterpret_cast<const float*>(static_cast<char*>(c.frag.p) + L.b1 + L.bc +
                                                    L.bC);
  return big_launch(c, k, 0.0f, 0.0f, thr, gate, dout, prof);
}

static bool big_launch(Ctx& c, int k, float thr1, float thr_rel, const float* thr_dev,
                       const long long* gate, long long* dout, bool prof) {
  const int d = c.d, DQ = big_dq(d), KB = (k + 31) / 32, Q = d4_of(d) / 4;
  const int cus = lloyd_num_cus(c.device);
  const BigLayout L = big_layout(k, d);
  char* dp = static_cast<char*>(c.frag.p);
  const h8* dfrag1 = reinterpret_cast<const h8*>(dp);
  const float* dcin = reinterpret_cast<const float*>(dp + L.b1);
  const double* dC = reinterpret_cast<const double*>(dp + L.b1 + L.bc);
  int JB = 5;
  while ((1 << (JB - 5)) < KB) ++JB;

  // level 1: persistent, one kBigThreads workgroup per CU (LDS-bound)
  const size_t lds1 = big_l1_lds(k, d);
  const int64_t groups = (c.n + 63) / 64;
  static const bool sp = !(exp_env("CDR_BIG_L1") && std::atoi(exp_env("CDR_BIG_L1")) == 0);
  const int wpb1 = (sp ? big_sp_threads(DQ) : kBigThreads) / 64;
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
  c.big_chunks.ensure(sizeof(int32_t) * (size_t)(nw1 + 1));
  int32_t* chunk_pre = c.big_chunks.as<int32_t>();
  c.fb_regions = nw1;
  c.fb_total_slot = nw1;  // L1 leftovers: the "fallback" statistic
  c.fb_layout = -1;       // screen32 must re-zero its counter layout
  BigArgs a;
  a.XT = c.xt32.as<float>();
  a.XB = nullptr;
  if (sp) {
    if (!c.xb_valid) {
      c.xb16.ensure((size_t)(c.n_pad >> 6) * 2 * DQ * 64 * 16);
      hipLaunchKernelGGL(big_frag_copy, dim3(4096), dim3(256), 0, c.stream, c.xt32.as<float>(),
                         c.n, c.n_pad, Q, DQ, c.xb16.as<uint4>());
      HIP_CHECK(hipGetLastError());
      c.xb_valid = true;
    }
    a.XB = c.xb16.as<h8>();
  }
  a.n = c.n;
  a.n_pad = c.n_pad;
  a.d = d;
  a.k = k;
  a.Q = Q;
  a.KB = KB;
  a.frag = dfrag1;
  a.cinit = dcin;
  a.thr0 = thr1;
  a.thr_rel = thr_rel;
  a.thr_dev = thr_dev;
  a.gate = gate;
  a.jkeep = ~((1u << JB) - 1u) | 15u;
  // DELTA: the running sums follow the labels of the previous large-k step
  // of this k (pipelined L1 only); moves go to c.mv_list, the sums are
  // updated by fixup_big instead of a pass over every point
  static const bool nodelta = exp_env("CDR_BIG_NODELTA") != nullptr;
  const bool delta = sp && !nodelta && c.big_valid && c.big_k == k;
  a.delta = delta ? 1 : 0;
  a.mv1 = nullptr;
  a.mv1_count = nullptr;
  a.mv2 = nullptr;
  a.mv2_count = nullptr;
  if (sp) ensure_rowmajor(c);
  a.XA = sp ? c.xa32.as<float>() : nullptr;
  a.d4 = d4_of(d);
  if (delta) {
    c.mv_list.ensure(sizeof(int2) * 2 * slots);
    c.mv_count.ensure(sizeof(int32_t) * (size_t)(nw1 + 2));
    HIP_CHECK(hipMemsetAsync(c.mv_count.p, 0, sizeof(int32_t) * (size_t)(nw1 + 2), c.stream));
    a.mv1 = c.mv_list.as<int2>();
    a.mv1_count = c.mv_count.as<int32_t>();
    a.mv2 = a.mv1 + slots;
    a.mv2_count = a.mv1_count + nw1;
  }
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
  if (sp)
    snprintf(c.prof_kernel, sizeof(c.prof_kernel), "screen_big_sp<%d,%d>", DQ, big_sp_threads(DQ));
  else
    snprintf(c.prof_kernel, sizeof(c.prof_kernel), "screen_big<%d,1,false,true>", DQ);
  if (prof) prof_mark(c, 0);
  switch (DQ) {
    case 1: launch_big_levels<1>(c, a, a2, dim3(nwg1), dim3(nwg2), lds1, dC, ovf, ovf_count, prof,
                                  sp, chunk_pre); break;
    case 2: launch_big_levels<2>(c, a, a2, dim3(nwg1), dim3(nwg2), lds1, dC, ovf, ovf_count, prof,
                                  sp, chunk_pre); break;
    case 3: launch_big_levels<3>(c, a, a2, dim3(nwg1), dim3(nwg2), lds1, dC, ovf, ovf_count, prof,
                                  sp, chunk_pre); break;
    default: launch_big_levels<4>(c, a, a2, dim3(nwg1), dim3(nwg2), lds1, dC, ovf, ovf_count, prof,
                                  sp, chunk_pre); break;
  }
  hipLaunchKernelGGL(exact_big, dim3(cus * 4), dim3(64), 0, c.stream, c.x32.as<float>(), c.n_pad,
                     d, dC, k, ovf, ovf_count, c.labels.as<int32_t>(), gate, a.mv2, a.mv2_count);
  HIP_CHECK(hipGetLastError());
  // the sums: a full pass over the points (first step) or the moves only
  const int len = k * (d + 1);
  c.big_sums.ensure(sizeof(long long) * len);
  unsigned long long* bs = c.big_sums.as<unsigned long long>();
  const int FG = big_fg(k);
  const int ngrp = (d + FG - 1) / FG;
  const size_t ldsu = (size_t)FG * k * 8 + (size_t)k * 4;
  static bool uattr = false;
  if (!uattr) {
    const void* fns[] = {reinterpret_cast<const void*>(&update_big<16>),
                         reinterpret_cast<const void*>(&update_big<8>),
                         reinterpret_cast<const void*>(&update_big<4>),
                         reinterpret_cast<const void*>(&fixup_big<16>),
                         reinterpret_cast<const void*>(&fixup_big<8>),
                         reinterpret_cast<const void*>(&fixup_big<4>)};
    for (const void* f : fns)
      HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    uattr = true;
  }
  const double fx = std::ldexp(1.0, c.scale_bits);
  if (!delta) {
    hipLaunchKernelGGL(zero_big_gated, dim3(64), dim3(256), 0, c.stream,
                       reinterpret_cast<long long*>(bs), (int64_t)len, gate);
    const dim3 gu(cus, ngrp);
    if (FG == 16)
      hipLaunchKernelGGL(update_big<16>, gu, dim3(1024), ldsu, c.stream, c.x32.as<float>(), c.n,
                         c.n_pad, d, k, c.labels.as<int32_t>(), fx, bs, gate);
    else if (FG == 8)
      hipLaunchKernelGGL(update_big<8>, gu, dim3(1024), ldsu, c.stream, c.x32.as<float>(), c.n,
                         c.n_pad, d, k, c.labels.as<int32_t>(), fx, bs, gate);
    else
      hipLaunchKernelGGL(update_big<4>, gu, dim3(1024), ldsu, c.stream, c.x32.as<float>(), c.n,
                         c.n_pad, d, k, c.labels.as<int32_t>(), fx, bs, gate);
  } else {
    const dim3 gf(kFixSlices, ngrp);
    const float* XA = c.xa32.as<float>();
    const int d4 = d4_of(d);
    if (FG == 16)
      hipLaunchKernelGGL(fixup_big<16>, gf, dim3(1024), ldsu, c.stream, XA, d4, d, k, a.mv1,
                         a.mv1_count, nw1, cap1, a.mv2, a.mv2_count, fx, bs, gate);
    else if (FG == 8)
      hipLaunchKernelGGL(fixup_big<8>, gf, dim3(1024), ldsu, c.stream, XA, d4, d, k, a.mv1,
                         a.mv1_count, nw1, cap1, a.mv2, a.mv2_count, fx, bs, gate);
    else
      hipLaunchKernelGGL(fixup_big<4>, gf, dim3(1024), ldsu, c.stream, XA, d4, d, k, a.mv1,
                         a.mv1_count, nw1, cap1, a.mv2, a.mv2_count, fx, bs, gate);
  }
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(dout, bs, sizeof(long long) * len, hipMemcpyDeviceToDevice, c.stream));
  c.big_valid = true;
  c.big_k = k;
  c.run_valid = false;
  c.lab8_valid = false;
  c.zb_valid = false;
  return true;
}

}  // namespace cdr
