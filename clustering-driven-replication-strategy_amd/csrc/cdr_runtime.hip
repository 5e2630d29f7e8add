// cdr_runtime.hip — context, buffers, point loading / generation and the C ABI
// entry points of libcdr.so (declared in include/cdr.h).
//
// Point layout in HBM: F32X quad-interleaved structure of arrays, F64 planar (xidx() in
// cdr_internal.h), padded to a multiple of 8192 points (the NumPy reduction
// block, see seeding).  Rows i >= n and features f >= d are zero and never
// produce labels, sums or probabilities.
#include <cmath>
#include <cstring>
#include <limits>

#include "cdr_internal.h"

namespace cdr {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

void DevBuf::ensure(size_t nbytes) {
  if (nbytes <= bytes) return;
  release();
  size_t nb = nbytes < 256 ? 256 : nbytes;
  HIP_CHECK(hipMalloc(&p, nb));
  bytes = nb;
}
void DevBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
}
void HostBuf::ensure(size_t nbytes) {
  if (nbytes <= bytes) return;
  release();
  size_t nb = nbytes < 4096 ? 4096 : nbytes;
  HIP_CHECK(hipHostMalloc(&p, nb, hipHostMallocDefault));
  bytes = nb;
}
void HostBuf::release() {
  if (p) (void)hipHostFree(p);
  p = nullptr;
  bytes = 0;
}

// ---------------------------------------------------------------------------
// Point statistics.  Orderable 64-bit keys let atomicMin/atomicMax track fp64
// extrema; `lsb` is the exponent of the lowest set bit of a value, so that
// x * 2^S is an integer for every x iff S >= -min(lsb).
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long ord_key(double v) {
  unsigned long long b = __double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__host__ __device__ inline double key_to_double(unsigned long long k) {
  unsigned long long b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  double v;
  memcpy(&v, &b, 8);
  return v;
}
__device__ __forceinline__ int lsb_exponent(double v) {
  unsigned long long b = __double_as_longlong(v);
  int e = (int)((b >> 52) & 0x7FF);
  unsigned long long m = b & 0xFFFFFFFFFFFFFull;
  if (e == 0) return -1074 + __builtin_ctzll(m);  // subnormal (m != 0)
  m |= (1ull << 52);
  return (e - 1075) + __builtin_ctzll(m);
}

// stats layout (unsigned long long): [0,d) min keys, [d,2d) max keys,
// [2d] -min lsb (as int64 via max), [2d+1] not-fp32-exact flag, [2d+2]
// non-finite flag.
template <typename T>
__global__ void stats_kernel(const T* __restrict__ X, int64_t n, int64_t n_pad,
                             int d, unsigned long long* __restrict__ st) {
  const int f = blockIdx.y;
  double lo = INFINITY, hi = -INFINITY;
  int need = -100000;  // max over values of -lsb
  int not32 = 0, nonfin = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double v = (double)X[xidx(X, f, i, n_pad)];
    if (!isfinite(v)) {
      nonfin = 1;
      continue;
    }
    lo = fmin(lo, v);
    hi = fmax(hi, v);
    if (v != 0.0) need = max(need, -lsb_exponent(v));
    if ((double)(float)v != v) not32 = 1;
  }
  // wave reduction
  for (int o = 32; o > 0; o >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, o));
    hi = fmax(hi, __shfl_xor(hi, o));
    need = max(need, __shfl_xor(need, o));
    not32 |= __shfl_xor(not32, o);
    nonfin |= __shfl_xor(nonfin, o);
  }
  if ((threadIdx.x & 63) == 0) {
    if (lo <= hi) {
      atomicMin(&st[f], ord_key(lo));
      atomicMax(&st[d + f], ord_key(hi));
    }
    atomicMax(&st[2 * d], (unsigned long long)(need + 200000));
    if (not32) atomicOr(&st[2 * d + 1], 1ull);
    if (nonfin) atomicOr(&st[2 * d + 2], 1ull);
  }
}

__global__ void rowmajor_to_soa64(const double* __restrict__ src, int64_t rows,
                                  int d, int64_t row0, int64_t n_pad,
                                  double* __restrict__ dst) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
       t < rows * d; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = t / d;
    int f = (int)(t - r * d);
    dst[xidx(dst, f, row0 + r, n_pad)] = src[t];
  }
}

// Between the two layouts (xidx): element t of the quad layout (x32) is
// feature 4 (t / (4 n_pad)) + t % 4 of point (t / 4) % n_pad; count = d4 n_pad.
__global__ void soa32_to_soa64(const float* __restrict__ src, int64_t count, int64_t n_pad,
                               double* __restrict__ dst) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = t / (4 * n_pad), r = t - q * 4 * n_pad;
    dst[xidx(dst, 4 * q + (r & 3), r >> 2, n_pad)] = (double)src[t];
  }
}

__global__ void soa64_to_soa32(const double* __restrict__ src, int64_t count, int64_t n_pad,
                               float* __restrict__ dst) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = t / (4 * n_pad), r = t - q * 4 * n_pad;
    dst[t] = (float)src[xidx(src, 4 * q + (r & 3), r >> 2, n_pad)];
  }
}

// ---------------------------------------------------------------------------
// Synthetic generator (integer-only, counter based).  Mirror: oracle/synth.py.
//   blob(i)      = mulhi32(splitmix64(seed ^ 0xB10B...) ^ i ..)
//   center(b,f)  = 2^21 + splitmix64(...) % (3 * 2^22)        (u24 units)
//   noise(i,f)   = 13 * (sum of four 16-bit lanes of splitmix64(...) - 131070)
//   x            = clamp(center + noise, 0, 2^24 - 1) * 2^-24
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void generate_kernel(float* __restrict__ X, int64_t row_begin,
                                int64_t n_local, int64_t n_pad, int d,
                                int n_blobs, uint64_t seed) {
  const uint64_t s_blob = splitmix64(seed ^ 0xB10B5EEDull);
  const uint64_t s_cent = splitmix64(seed ^ 0xCE27E25ull);
  const uint64_t s_noise = splitmix64(seed ^ 0x9015Eull);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_local;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t row = (uint64_t)(row_begin + i);
    const uint64_t hb = splitmix64(s_blob + row);
    const uint64_t b = ((hb >> 32) * (uint64_t)n_blobs) >> 32;
    for (int f = 0; f < d; ++f) {
      const uint64_t hc = splitmix64(s_cent + b * (uint64_t)d + (uint64_t)f);
      const int64_t center = (int64_t)(1u << 21) + (int64_t)(hc % (3ull << 22));
      const uint64_t hn = splitmix64(s_noise + row * (uint64_t)d + (uint64_t)f);
      const int64_t s = (int64_t)(hn & 0xFFFF) + (int64_t)((hn >> 16) & 0xFFFF) +
                        (int64_t)((hn >> 32) & 0xFFFF) + (int64_t)(hn >> 48);
      int64_t u = center + 13 * (s - 131070);
      u = u < 0 ? 0 : (u > 0xFFFFFF ? 0xFFFFFF : u);
      X[xidx(X, f, i, n_pad)] = (float)u * (1.0f / 16777216.0f);
    }
  }
}

static int grid_for(int64_t work, int threads, int cap = 4096) {
  int64_t g = (work + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

static void run_stats(Ctx& c, bool f32, std::vector<unsigned long long>& st) {
  const int d = c.d;
  DevBuf dst;
  dst.ensure(sizeof(unsigned long long) * (2 * d + 3));
  std::vector<unsigned long long> init(2 * d + 3, 0);
  for (int f = 0; f < d; ++f) {
    init[f] = ~0ull;
    init[d + f] = 0ull;
  }
  init[2 * d] = 0;
  HIP_CHECK(hipMemcpyAsync(dst.p, init.data(), init.size() * 8,
                           hipMemcpyHostToDevice, c.stream));
  dim3 grid(grid_for(c.n, 256, 1024), d);
  if (f32)
    hipLaunchKernelGGL(stats_kernel<float>, grid, dim3(256), 0, c.stream,
                       c.x32.as<float>(), c.n, c.n_pad, d, dst.as<unsigned long long>());
  else
    hipLaunchKernelGGL(stats_kernel<double>, grid, dim3(256), 0, c.stream,
                       c.x64.as<double>(), c.n, c.n_pad, d, dst.as<unsigned long long>());
  HIP_CHECK(hipGetLastError());
  st.assign(2 * d + 3, 0);
  HIP_CHECK(hipMemcpyAsync(st.data(), dst.p, st.size() * 8,
                           hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  dst.release();
  c.st_local = st;
}

// Decide the storage mode and the screen transform from the statistics.
// n_sum: the number of rows a cluster sum can run over (the whole data set:
// n_total when this context holds one shard of it).
static void decide_mode(Ctx& c, const std::vector<unsigned long long>& st,
                        bool have_f64_copy, int64_t n_sum) {
  const int d = c.d;
  if (st[2 * d + 2])
    CDR_FAIL(CDR_ERR_NAN, "Probabilities contain NaN");  // non-finite input
  c.fmin.assign(d, 0.0);
  c.fmax.assign(d, 0.0);
  c.absmax = 0.0;
  for (int f = 0; f < d; ++f) {
    if (st[f] <= st[d + f]) {  // (an empty shard before cdr_points_restat: no range)
      c.fmin[f] = key_to_double(st[f]);
      c.fmax[f] = key_to_double(st[d + f]);
    }
    c.absmax = std::fmax(c.absmax, std::fmax(std::fabs(c.fmin[f]), std::fabs(c.fmax[f])));
  }
  const long long need = (long long)st[2 * d] - 200000;
  int S = need < 0 ? 0 : (int)need;
  bool f32x = (st[2 * d + 1] == 0) && S <= 1000;
  if (f32x && c.absmax > 0) {
    const double m = std::ldexp(c.absmax, S);
    if (!(m < 1073741824.0)) f32x = false;  // |x|2^S < 2^30
    // Every partial sum of a cluster stays below 2^53 grid units, so NumPy's
    // sequential fp64 mean (src/kmeans_plusplus.py:41) never rounds and equals
    // the exact int64 sum converted once: the F32X promise.
    if (!(m * (double)(n_sum > 0 ? n_sum : 1) < 9007199254740992.0)) f32x = false;
  }
  c.mode = f32x ? CDR_MODE_F32X : CDR_MODE_F64;
  c.scale_bits = f32x ? S : 0;
  // screen transform: centre each feature at its midrange, scale so |xhat| <= 1
  c.mu.assign(d, 0.0f);
  double maxdev = 0.0;
  for (int f = 0; f < d; ++f) {
    c.mu[f] = (float)(0.5 * (c.fmin[f] + c.fmax[f]));
    if (f32x) {  // on the data grid, so that x - mu is a whole number of grid steps
      const float g = (float)std::ldexp(std::rint(std::ldexp((double)c.mu[f], S)), -S);
      if (std::isfinite(g)) c.mu[f] = g;
    }
    maxdev = std::fmax(maxdev, std::fmax(c.fmax[f] - (double)c.mu[f],
                                         (double)c.mu[f] - c.fmin[f]));
  }
  c.sigma = 0;
  if (maxdev > 0) {
    int e;
    std::frexp(maxdev, &e);  // maxdev in [2^(e-1), 2^e)
    c.sigma = -e;            // maxdev * 2^sigma < 1
  }
  std::vector<float> ms(d);
  for (int f = 0; f < d; ++f) ms[f] = (float)(-std::ldexp((double)c.mu[f], c.sigma));
  // Pre-centred screen copy xt = (x - mu) 2^sigma (screen32.hip) is exact in
  // fp32 when every |x - mu| is < 2^24 grid steps, mu is itself on the grid and
  // the smallest step 2^(sigma - S) is a normal float.
  c.pre_ok = c.mode == CDR_MODE_F32X && c.n > 0 && (c.sigma - S) >= -126;
  for (int f = 0; f < d; ++f)
    if (!(st[f] <= st[d + f])) c.pre_ok = false;
  for (int f = 0; f < d && c.pre_ok; ++f) {
    const double mu = (double)c.mu[f];
    if (std::ldexp(std::rint(std::ldexp(mu, S)), -S) != mu) c.pre_ok = false;
    const double dev = std::fmax(c.fmax[f] - mu, mu - c.fmin[f]);
    if (!(std::ldexp(dev, S) < 16777216.0)) c.pre_ok = false;
    if ((double)ms[f] != -std::ldexp(mu, c.sigma)) c.pre_ok = false;
  }
  c.xt_valid = false;
  c.f64x_e_ok = false;
  c.seed16_valid = false;
  c.xs_valid = false;
  c.xh_valid = false;
  c.xb_valid = false;
  c.xa_valid = false;
  c.big_valid = false;
  c.mu_s.ensure(sizeof(float) * (d > 0 ? d : 1));
  HIP_CHECK(hipMemcpyAsync(c.mu_s.p, ms.data(), sizeof(float) * d,
                           hipMemcpyHostToDevice, c.stream));
  if (c.mode == CDR_MODE_F32X && have_f64_copy) {
    c.x32.ensure(sizeof(float) * (size_t)d4_of(d) * c.n_pad);
    hipLaunchKernelGGL(soa64_to_soa32, dim3(grid_for((int64_t)d4_of(d) * c.n_pad, 256)),
                       dim3(256), 0, c.stream, c.x64.as<double>(),
                       (int64_t)d4_of(d) * c.n_pad, c.n_pad, c.x32.as<float>());
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(c.stream));
    c.x64.release();
  }
  c.have_labels = false;
  c.run_valid = false;
  c.lab8_valid = false;
  c.zb_valid = false;
  c.big_valid = false;
  c.seed_scanned = false;
}

static void reset_points(Ctx& c, int64_t n, int32_t d) {
  if (n < 0 || d <= 0) CDR_FAIL(CDR_ERR_ARG, "points: need n >= 0 and d >= 1");
  c.x32.release();
  c.x64.release();
  c.xt32.release();
  c.xt_valid = false;
  c.f64x_e_ok = false;
  c.seed16_valid = false;
  c.xs16.release();
  c.xh16.release();
  c.zb.release();
  c.xa32.release();
  c.xs_valid = false;
  c.xh_valid = false;
  c.xb16.release();
  c.xb_valid = false;
  c.xa_valid = false;
  c.big_valid = false;
  c.pre_ok = false;
  c.n = n;
  c.d = d;
  c.n_pad = ceil_div(n > 0 ? n : 1, kSeedBlock) * kSeedBlock;
  c.run_valid = false;
  c.lab8_valid = false;
  c.zb_valid = false;
  c.ll_on = false;
  c.labels.ensure(sizeof(int32_t) * c.n_pad);
  HIP_CHECK(hipMemsetAsync(c.labels.p, 0, sizeof(int32_t) * c.n_pad, c.stream));
}

void points_analyze_and_store(Ctx& c, const double* hX) {
  const int d = c.d;
  c.x64.ensure(sizeof(double) * (size_t)d4_of(d) * c.n_pad);
  HIP_CHECK(hipMemsetAsync(c.x64.p, 0, sizeof(double) * (size_t)d4_of(d) * c.n_pad, c.stream));
  const int64_t chunk_rows = std::max<int64_t>(1, (int64_t)(32 << 20) / d);
  DevBuf stage;
  stage.ensure(sizeof(double) * (size_t)std::min<int64_t>(chunk_rows, std::max<int64_t>(c.n, 1)) * d);
  for (int64_t r0 = 0; r0 < c.n; r0 += chunk_rows) {
    const int64_t rows = std::min(chunk_rows, c.n - r0);
    HIP_CHECK(hipMemcpyAsync(stage.p, hX + r0 * d, sizeof(double) * rows * d,
                             hipMemcpyHostToDevice, c.stream));
    hipLaunchKernelGGL(rowmajor_to_soa64, dim3(grid_for(rows * d, 256)), dim3(256), 0,
                       c.stream, stage.as<double>(), rows, d, r0, c.n_pad,
                       c.x64.as<double>());
    HIP_CHECK(hipGetLastError());
  }
  HIP_CHECK(hipStreamSynchronize(c.stream));
  stage.release();
  std::vector<unsigned long long> st;
  run_stats(c, false, st);
  decide_mode(c, st, true, c.n);
}

void points_generate(Ctx& c, int64_t n_total, int64_t row_begin, int32_t n_blobs,
                     uint64_t seed) {
  if (n_blobs < 1) CDR_FAIL(CDR_ERR_ARG, "generate: n_blobs must be >= 1");
  if (row_begin < 0 || row_begin + c.n > n_total)
    CDR_FAIL(CDR_ERR_ARG, "generate: rows out of range");
  c.x32.ensure(sizeof(float) * (size_t)d4_of(c.d) * c.n_pad);
  HIP_CHECK(hipMemsetAsync(c.x32.p, 0, sizeof(float) * (size_t)d4_of(c.d) * c.n_pad, c.stream));
  hipLaunchKernelGGL(generate_kernel, dim3(grid_for(c.n, 256, 8192)), dim3(256), 0,
                     c.stream, c.x32.as<float>(), row_begin, c.n, c.n_pad, c.d,
                     n_blobs, seed);
  HIP_CHECK(hipGetLastError());
  std::vector<unsigned long long> st;
  run_stats(c, true, st);
  decide_mode(c, st, false, n_total);
  if (c.mode != CDR_MODE_F32X)
    CDR_FAIL(CDR_ERR_STATE, "generate: synthetic data must be F32X");
}

__global__ void gather_rows_kernel(const float* __restrict__ x32,
                                   const double* __restrict__ x64,
                                   const int64_t* __restrict__ idx, int64_t m,
                                   int d, int64_t n_pad, double* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < m * d;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = t / d;
    int f = (int)(t - r * d);
    int64_t i = idx[r];
    out[t] = x32 ? (double)x32[xidx(x32, f, i, n_pad)] : x64[xidx(x64, f, i, n_pad)];
  }
}

}  // namespace cdr

using namespace cdr;

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

const char* cdr_last_error(void) { return g_last_error.c_str(); }
int cdr_version(void) { return 1; }

int cdr_device_count(int* out) {
  CDR_TRY
  if (!out) CDR_FAIL(CDR_ERR_ARG, "null out");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *out = (e == hipSuccess) ? n : 0;
  CDR_CATCH
}

int cdr_create(int device, cdr_ctx** out) {
  CDR_TRY
  if (!out) CDR_FAIL(CDR_ERR_ARG, "null out");
  int n = 0;
  HIP_CHECK(hipGetDeviceCount(&n));
  if (device < 0 || device >= n)
    CDR_FAIL(CDR_ERR_ARG, "device index out of range (" + std::to_string(n) + " devices)");
  HIP_CHECK(hipSetDevice(device));
  cdr_ctx* h = new cdr_ctx();
  h->c.device = device;
  hipError_t e = hipStreamCreateWithFlags(&h->c.stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete h;
    HIP_CHECK(e);
  }
  h->c.own_stream = true;
#ifdef CDR_EXPERIMENTS
  if (const char* ab = exp_env("CDR_SCREEN_ABLATE")) h->c.screen_ablate = atoi(ab);
#endif
  *out = h;
  CDR_CATCH
}

int cdr_destroy(cdr_ctx* h) {
  CDR_TRY
  if (!h) return CDR_OK;
  Ctx& c = h->c;
  (void)hipSetDevice(c.device);
  (void)hipStreamSynchronize(c.stream);
  comm_release(c);
  DevBuf* bufs[] = {&c.comm_buf, &c.x32, &c.x64, &c.xt32, &c.muf, &c.mu_s, &c.labels, &c.cent64, &c.frag,
                    &c.partials, &c.out_sums, &c.fb_list, &c.fb_count, &c.f64_sums,
                    &c.f64_counts, &c.dmin, &c.blocksums, &c.xfer, &c.cend,
                    &c.seed_scalar, &c.med_vals, &c.med_off, &c.med_out, &c.med_tmp,
                    &c.med_tmp2, &c.ev_file, &c.ev_op, &c.ev_client, &c.ev_ts,
                    &c.ev_primary, &c.ev_out, &c.ev_scratch, &c.ev_scratch2,
                    &c.fin_counts, &c.fin_creation, &c.fin_out, &c.fin_red, &c.run_sums,
                    &c.gb_tilepref, &c.gb_chunk, &c.gb_rsum, &c.gb_part, &c.gb_small, &c.gb_res, &c.gb_bbase,
                    &c.gb_p1, &c.gb_p2, &c.gb_hist2, &c.gb_list, &c.gb_slots, &c.sim_cnt, &c.sim_off,
                    &c.sim_tmp, &c.sim_ms, &c.sim_mbase, &c.x_small, &c.x_buf, &c.x_prim, &c.f64x_A, &c.f64x_cnt, &c.f64x_E,
                    &c.f64x_T, &c.f64x_walk, &c.f64x_G, &c.f64x_GS, &c.f64x_GC, &c.f64x_prof, &c.f64x_E2, &c.f64x_ord, &c.f64x_dirty, &c.med_hist,
                    &c.fb_accum, &c.q_acc, &c.xs16, &c.xa32, &c.xb16, &c.big_sums, &c.big_chunks, &c.seed_near, &c.seed_cents, &c.seed_ccd, &c.seg_tails, &c.seg_ents, &c.seg_scan, &c.seg_items, &c.seg_meta, &c.seed_tail_plan, &c.seed_x16, &c.seed_e16, &c.seed_mu, &c.seed_run_buf, &c.mv_list, &c.lab8, &c.zb, &c.xh16, &c.bnd, &c.t_acc, &c.dmin32, &c.bs32, &c.cent32r, &c.mv_count, &c.ll_C, &c.ll_new, &c.ll_sums, &c.ll_ref,
                    &c.ll_state};
  for (DevBuf* b : bufs) b->release();
  c.h_small.release();
  c.h_up.release();
  if (c.up_event) (void)hipEventDestroy(c.up_event);
  for (hipEvent_t& e : c.prof_pool)
    if (e) (void)hipEventDestroy(e);
  if (c.own_stream && c.stream) (void)hipStreamDestroy(c.stream);
  delete h;
  CDR_CATCH
}

int cdr_set_stream(cdr_ctx* h, void* s) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  if (s == nullptr) {
    if (!c.own_stream) {
      HIP_CHECK(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
      c.own_stream = true;
    }
  } else {
    if (c.own_stream) HIP_CHECK(hipStreamDestroy(c.stream));
    c.stream = (hipStream_t)s;
    c.own_stream = false;
  }
  CDR_CATCH
}

int cdr_synchronize(cdr_ctx* h) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  HIP_CHECK(hipSetDevice(h->c.device));
  HIP_CHECK(hipStreamSynchronize(h->c.stream));
  CDR_CATCH
}

int cdr_points_load_f64(cdr_ctx* h, const double* X, int64_t n, int32_t d) {
  CDR_TRY
  if (!h || (!X && n > 0)) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  reset_points(c, n, d);
  points_analyze_and_store(c, X);
  CDR_CATCH
}

int cdr_points_generate(cdr_ctx* h, int64_t n_total, int64_t row_begin,
                        int64_t n_local, int32_t d, int32_t n_blobs, uint64_t seed) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  reset_points(c, n_local, d);
  points_generate(c, n_total, row_begin, n_blobs, seed);
  CDR_CATCH
}

int cdr_points_stats(cdr_ctx* h, uint64_t* st) {
  CDR_TRY
  if (!h || !st) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  if (c.mode == 0 || c.st_local.size() != (size_t)(2 * c.d + 3))
    CDR_FAIL(CDR_ERR_STATE, "no points loaded");
  for (size_t i = 0; i < c.st_local.size(); ++i) st[i] = c.st_local[i];
  CDR_CATCH
}

int cdr_points_restat(cdr_ctx* h, const uint64_t* st, int64_t n_sum) {
  CDR_TRY
  if (!h || !st) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  if (c.mode == 0) CDR_FAIL(CDR_ERR_STATE, "no points loaded");
  const int d = c.d;
  std::vector<unsigned long long> g(st, st + 2 * d + 3);
  // the combined statistics must cover this shard's
  for (int f = 0; f < d && c.n > 0; ++f)
    if (g[f] > c.st_local[f] || g[d + f] < c.st_local[d + f])
      CDR_FAIL(CDR_ERR_ARG, "restat: statistics do not cover this shard");
  const int old_mode = c.mode;
  const std::vector<unsigned long long> keep = c.st_local;
  decide_mode(c, g, false, n_sum);
  c.st_local = keep;
  if (old_mode == CDR_MODE_F32X && c.mode == CDR_MODE_F64) {
    // another shard is not on an fp32 grid: this one's exact fp32 values
    // become its fp64 copy
    const int64_t cnt = (int64_t)d4_of(d) * c.n_pad;
    c.x64.ensure(sizeof(double) * (size_t)cnt);
    hipLaunchKernelGGL(soa32_to_soa64, dim3(grid_for(cnt, 256)), dim3(256), 0, c.stream,
                       c.x32.as<float>(), cnt, c.n_pad, c.x64.as<double>());
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(c.stream));
    c.x32.release();
  } else if (old_mode == CDR_MODE_F64 && c.mode == CDR_MODE_F32X) {
    CDR_FAIL(CDR_ERR_ARG, "restat: a shard stored as F64 cannot become F32X");
  }
  HIP_CHECK(hipStreamSynchronize(c.stream));
  CDR_CATCH
}

int cdr_points_info(cdr_ctx* h, int64_t* n, int32_t* d, int32_t* mode,
                    int32_t* scale_bits) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  if (n) *n = h->c.n;
  if (d) *d = h->c.d;
  if (mode) *mode = h->c.mode;
  if (scale_bits) *scale_bits = h->c.scale_bits;
  CDR_CATCH
}

int cdr_points_get_rows(cdr_ctx* h, const int64_t* idx, int64_t m, double* out) {
  CDR_TRY
  if (!h || (m > 0 && (!idx || !out))) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  if (c.mode == 0) CDR_FAIL(CDR_ERR_STATE, "no points loaded");
  for (int64_t r = 0; r < m; ++r)
    if (idx[r] < 0 || idx[r] >= c.n) CDR_FAIL(CDR_ERR_ARG, "row index out of range");
  if (m == 0) return CDR_OK;
  HIP_CHECK(hipSetDevice(c.device));
  DevBuf di, dout;
  di.ensure(sizeof(int64_t) * m);
  dout.ensure(sizeof(double) * m * c.d);
  HIP_CHECK(hipMemcpyAsync(di.p, idx, sizeof(int64_t) * m, hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(m * c.d, 256)), dim3(256), 0,
                     c.stream, c.mode == CDR_MODE_F32X ? c.x32.as<float>() : nullptr,
                     c.mode == CDR_MODE_F64 ? c.x64.as<double>() : nullptr,
                     di.as<int64_t>(), m, c.d, c.n_pad, dout.as<double>());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(out, dout.p, sizeof(double) * m * c.d, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  CDR_CATCH
}

double cdr_host_seq_sum(const double* v, int64_t n, double init) {
  volatile double s = init;  // keep strict left-to-right fp64 adds
  for (int64_t i = 0; i < n; ++i) s = s + v[i];
  return s;
}

}  // extern "C"
