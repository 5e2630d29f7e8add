// loop.hip — device-resident Lloyd loop: src/kmeans_plusplus.py:31-48 with
// no host round trip per step.
//
// The reference's loop needs the host after every step: the means (:41), the
// empty-cluster reseed from the global legacy RNG (:43) and the convergence
// test on np.linalg.norm (:45-48).  Here a step is enqueued as
//
//   [plan32_kernel]  screen32  reduce32  publish32  (all-reduce)  ll_finalize
//
// and the host only polls a status word every few steps:
// * ll_finalize forms the means exactly as the host does (fp64 ldexp of the
//   int64 fixed-point sums, one correctly rounded division: the same bits),
//   the shift^2 and the inertia, and moves the centroids forward;
// * it STOPS the loop (state[0] = 0; every later kernel of the enqueued steps
//   then exits at its first instruction) when a cluster is empty (the host
//   draws np.random.randint in j order), when the shift is within a relative
//   1e-9 of tol (the host decides with np.linalg.norm itself) or converged;
// * plan32_kernel stops it when the centroids leave the fp16 split range
//   (the host then takes that step on the host-plan path).
// Every decision the device takes is therefore the reference's decision.
//
// Inertia (north_star; the reference computes none): sum_i ||x_i - c_l(i)||^2
// of the step's assignment, from the exact cluster sums by
//   I = sum_i ||x_i - r||^2 - 2 sum_j (c_j - r).(S_j - n_j r) + sum_j n_j ||c_j - r||^2
// with r a data row (x - r exact on the grid); sum_i ||x_i - r||^2 is one
// pass over the points per run (cdr_points_sqdev; all-reduced once when the
// points are sharded).
#include <cmath>
#include <cstring>

#include "cdr_internal.h"

namespace cdr {

enum : long long { kLLRun = 0, kLLConverged = 1, kLLEmpty = 2, kLLHostPlan = 3, kLLAmbiguous = 4 };
constexpr int kLLState = 8;  // int64 words of ll_state

bool screen32_supported(const Ctx& c, int k);
bool screen32_step(Ctx& c, const double* C, int k, long long* dout, long long* hout, bool prof,
                   float* dbg, float* thr_out, long long* gate);
void plan32_point_side(const Ctx& c, double& xxmax, double& l1x);
void lloyd_step_f32x(Ctx& c, const double* C, int32_t k, int64_t* out, bool out_dev);

// One workgroup.  sums: (k, d+1) int64 fixed-point sums | counts (after the
// all-reduce).  Cnew (k*d means, then k counts as int64) is always written;
// C moves to Cnew unless the loop stops for the host.
__global__ __launch_bounds__(256) void ll_finalize(const long long* __restrict__ sums, int k,
                                                   int d, int sbits, int round32, double tol,
                                                   double margin, double x2,
                                                   const double* __restrict__ ref,
                                                   double* __restrict__ C,
                                                   double* __restrict__ Cnew,
                                                   long long* __restrict__ state) {
  if (state[0] == 0) return;
  __shared__ double r_ss[256], r_cross[256], r_quad[256];
  __shared__ int r_empty[256];
  __shared__ int move;
  const int t = threadIdx.x;
  const int d1 = d + 1;
  double ss = 0.0, cross = 0.0, quad = 0.0;
  int empty = 0;
  long long* cnt_out = reinterpret_cast<long long*>(Cnew + (size_t)k * d);
  for (int j = t; j < k; j += blockDim.x) cnt_out[j] = sums[(size_t)j * d1 + d];
  for (int e = t; e < k * d; e += blockDim.x) {
    const int j = e / d, f = e - j * d;
    const long long cnt = sums[(size_t)j * d1 + d];
    // the host's np.ldexp(acc.astype(float64), -S) / counts (kmeans_plusplus.py)
    const double sj = ldexp((double)sums[(size_t)j * d1 + f], -sbits);
    double m = sj / (double)cnt;
    if (round32) m = (double)(float)m;  // new_centroids has X's dtype (float32)
    Cnew[e] = m;
    if (cnt == 0) {
      empty = 1;
      continue;
    }
    const double c = C[e];
    const double df = m - c;
    ss += df * df;
    const double ct = c - ref[f];
    cross += ct * (sj - (double)cnt * ref[f]);
    quad += (double)cnt * (ct * ct);
  }
  r_ss[t] = ss;
  r_cross[t] = cross;
  r_quad[t] = quad;
  r_empty[t] = empty;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {  // fixed tree: deterministic
    if (t < o) {
      r_ss[t] += r_ss[t + o];
      r_cross[t] += r_cross[t + o];
      r_quad[t] += r_quad[t + o];
      r_empty[t] |= r_empty[t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    const double sst = r_ss[0];
    const double inertia = x2 - 2.0 * r_cross[0] + r_quad[0];
    long long reason = kLLRun;
    int mv = 0;
    if (r_empty[0]) {
      reason = kLLEmpty;
    } else {
      const double sh = sqrt(sst);
      mv = 1;
      if (tol > 0.0 && !(sh > tol * (1.0 + margin))) {
        if (sh < tol * (1.0 - margin)) {
          reason = kLLConverged;  // shift < tol: the reference breaks after moving
        } else {
          reason = kLLAmbiguous;  // too close to call in fp64: the host decides
          mv = 0;
        }
      }
    }
    if (mv) state[1] += 1;
    if (reason != kLLRun) {
      state[0] = 0;
      state[2] = reason;
    }
    state[3] = __double_as_longlong(sst);
    state[4] = __double_as_longlong(inertia);
    move = mv;
  }
  __syncthreads();
  if (move)
    for (int e = t; e < k * d; e += blockDim.x) C[e] = Cnew[e];
}

// Per-block partial sums of ||x_i - r||^2 (features in order, fp64).
__global__ __launch_bounds__(256) void sqdev_kernel(const float* __restrict__ X, int64_t n,
                                                    int64_t n_pad, int d,
                                                    const double* __restrict__ ref,
                                                    double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double p = 0.0;
    for (int f = 0; f < d; ++f) {
      const double v = (double)X[xidx(f, i, n_pad)] - ref[f];
      p += v * v;
    }
    s += p;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void ll_set_state(long long* __restrict__ state, long long active, long long add_steps,
                             long long reason) {
  if (threadIdx.x == 0) {
    state[0] = active;
    state[1] += add_steps;
    state[2] = reason;
  }
}

static double points_sqdev(Ctx& c, const double* ref_host) {
  if (c.mode != CDR_MODE_F32X) CDR_FAIL(CDR_ERR_UNSUPPORTED, "sqdev: points are not F32X");
  const int nb = 1024;
  DevBuf dref, part;
  dref.ensure(sizeof(double) * c.d);
  part.ensure(sizeof(double) * nb);
  HIP_CHECK(hipMemcpyAsync(dref.p, ref_host, sizeof(double) * c.d, hipMemcpyHostToDevice,
                           c.stream));
  hipLaunchKernelGGL(sqdev_kernel, dim3(nb), dim3(256), 0, c.stream, c.x32.as<float>(), c.n,
                     c.n_pad, c.d, dref.as<double>(), part.as<double>());
  HIP_CHECK(hipGetLastError());
  std::vector<double> h(nb);
  HIP_CHECK(hipMemcpyAsync(h.data(), part.p, sizeof(double) * nb, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  double s = 0.0;
  for (double v : h) s += v;
  return s;
}

static void ll_require(const Ctx& c) {
  if (!c.ll_on) CDR_FAIL(CDR_ERR_STATE, "lloyd loop: cdr_lloyd_begin first");
}

static void ll_read_state(Ctx& c, long long* st) {
  HIP_CHECK(hipMemcpyAsync(st, c.ll_state.p, sizeof(long long) * kLLState, hipMemcpyDeviceToHost,
                           c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));
}

}  // namespace cdr

using namespace cdr;

extern "C" {

int cdr_points_sqdev(cdr_ctx* h, const double* ref, double* out) {
  CDR_TRY
  if (!h || !ref || !out) CDR_FAIL(CDR_ERR_ARG, "null argument");
  HIP_CHECK(hipSetDevice(h->c.device));
  *out = points_sqdev(h->c, ref);
  CDR_CATCH
}

int cdr_lloyd_begin(cdr_ctx* h, const double* C, int32_t k, double tol, int32_t flags,
                    const double* ref, double x2_total) {
  CDR_TRY
  if (!h || !C || !ref) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  if (c.mode != CDR_MODE_F32X)
    CDR_FAIL(CDR_ERR_UNSUPPORTED, "lloyd loop: points are not F32X (use cdr_lloyd_step_f64)");
  if (k < 1) CDR_FAIL(CDR_ERR_ARG, "k must be >= 1");
  const int d = c.d;
  c.ll_k = k;
  c.ll_flags = flags;
  c.ll_tol = tol;
  c.ll_x2 = std::isnan(x2_total) ? points_sqdev(c, ref) : x2_total;
  c.ll_devplan = screen32_supported(c, k) && !std::getenv("CDR_NO_DEVPLAN");
  plan32_point_side(c, c.ll_xxmax, c.ll_l1x);
  c.ll_C.ensure(sizeof(double) * (size_t)k * d);
  c.ll_new.ensure(sizeof(double) * (size_t)k * (d + 1));
  c.ll_sums.ensure(sizeof(long long) * (size_t)k * (d + 1));
  c.ll_ref.ensure(sizeof(double) * 2 * d);
  c.ll_state.ensure(sizeof(long long) * kLLState);
  std::vector<double> rm(2 * d);
  for (int f = 0; f < d; ++f) {
    rm[f] = ref[f];
    rm[d + f] = (double)c.mu[f];
  }
  const long long st0[kLLState] = {1, 0, kLLRun, 0, 0, 0, 0, 0};
  HIP_CHECK(hipMemcpyAsync(c.ll_C.p, C, sizeof(double) * (size_t)k * d, hipMemcpyHostToDevice,
                           c.stream));
  HIP_CHECK(hipMemcpyAsync(c.ll_ref.p, rm.data(), sizeof(double) * 2 * d, hipMemcpyHostToDevice,
                           c.stream));
  HIP_CHECK(hipMemcpyAsync(c.ll_state.p, st0, sizeof(st0), hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipStreamSynchronize(c.stream));  // rm and st0 live on this stack
  c.ll_on = true;
  c.ll_enqueued = 0;
  c.ll_hostplan_once = false;
  // the first step recomputes the running sums from scratch (see resume)
  c.run_valid = false;
  CDR_CATCH
}

int cdr_lloyd_enqueue_assign(cdr_ctx* h, int64_t* dsums) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  ll_require(c);
  long long* dout = dsums ? reinterpret_cast<long long*>(dsums) : c.ll_sums.as<long long>();
  long long* state = c.ll_state.as<long long>();
  if (c.ll_devplan && !c.ll_hostplan_once) {
    const bool prof = prof_step_begin(c);
    screen32_step(c, nullptr, c.ll_k, dout, nullptr, prof, nullptr, nullptr, state);
    if (prof) prof_mark(c, 2);
    c.last_k = c.ll_k;
    c.have_labels = true;
    c.last_screened = true;
    c.last_fallback = -1;
  } else {
    // host plan (shapes screen32 does not cover, or one step after the
    // device plan's range guard stopped the loop): needs C on the host
    long long st[kLLState];
    ll_read_state(c, st);
    c.ll_hostplan_once = false;
    if (st[0]) {
      std::vector<double> Ch((size_t)c.ll_k * c.d);
      HIP_CHECK(hipMemcpy(Ch.data(), c.ll_C.p, sizeof(double) * Ch.size(), hipMemcpyDeviceToHost));
      lloyd_step_f32x(c, Ch.data(), c.ll_k, reinterpret_cast<int64_t*>(dout), true);
    }
  }
  c.ll_enqueued += 1;
  CDR_CATCH
}

int cdr_lloyd_enqueue_finalize(cdr_ctx* h, const int64_t* dsums) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  ll_require(c);
  const long long* sums =
      dsums ? reinterpret_cast<const long long*>(dsums) : c.ll_sums.as<long long>();
  const int kd = c.ll_k * c.d;
  const bool r32 = (c.ll_flags & 1) != 0;
  // fp64 sum of kd squares errs by < kd 2^-53 relative; float32 centroids are
  // compared by NumPy in float32 (kd 2^-23)
  const double margin = r32 ? std::ldexp((double)(kd + 2), -22) : 1e-9;
  hipLaunchKernelGGL(ll_finalize, dim3(1), dim3(256), 0, c.stream, sums, c.ll_k, c.d, c.scale_bits,
                     r32 ? 1 : 0, c.ll_tol, margin, c.ll_x2, c.ll_ref.as<double>(),
                     c.ll_C.as<double>(), c.ll_new.as<double>(), c.ll_state.as<long long>());
  HIP_CHECK(hipGetLastError());
  CDR_CATCH
}

int cdr_lloyd_status(cdr_ctx* h, int64_t* status, double* values) {
  CDR_TRY
  if (!h || !status) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  ll_require(c);
  long long st[kLLState];
  ll_read_state(c, st);
  status[0] = st[0];
  status[1] = st[1];
  status[2] = st[2];
  status[3] = c.ll_enqueued;
  if (values) {
    double ss, in;
    memcpy(&ss, &st[3], 8);
    memcpy(&in, &st[4], 8);
    values[0] = std::sqrt(ss);
    values[1] = in;
  }
  CDR_CATCH
}

int cdr_lloyd_read(cdr_ctx* h, double* C, double* means, int64_t* counts) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  ll_require(c);
  const size_t kd = (size_t)c.ll_k * c.d;
  HIP_CHECK(hipStreamSynchronize(c.stream));
  if (C) HIP_CHECK(hipMemcpy(C, c.ll_C.p, sizeof(double) * kd, hipMemcpyDeviceToHost));
  if (means) HIP_CHECK(hipMemcpy(means, c.ll_new.p, sizeof(double) * kd, hipMemcpyDeviceToHost));
  if (counts)
    HIP_CHECK(hipMemcpy(counts, c.ll_new.as<double>() + kd, sizeof(long long) * c.ll_k,
                        hipMemcpyDeviceToHost));
  CDR_CATCH
}

int cdr_lloyd_resume(cdr_ctx* h, const double* C, int32_t add_steps, int32_t host_plan_once) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  ll_require(c);
  if (C)
    HIP_CHECK(hipMemcpyAsync(c.ll_C.p, C, sizeof(double) * (size_t)c.ll_k * c.d,
                             hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(ll_set_state, dim3(1), dim3(64), 0, c.stream, c.ll_state.as<long long>(), 1LL,
                     (long long)add_steps, (long long)kLLRun);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipStreamSynchronize(c.stream));  // C belongs to the caller
  c.ll_hostplan_once = host_plan_once != 0;
  // Steps enqueued after the stop did nothing, but the host marked the
  // running sums valid after each of them; a full (non-DELTA) step that was
  // among them never zeroed and rebuilt them.  The next step starts afresh.
  c.run_valid = false;
  CDR_CATCH
}

int cdr_lloyd_end(cdr_ctx* h) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  h->c.ll_on = false;
  CDR_CATCH
}

}  // extern "C"
