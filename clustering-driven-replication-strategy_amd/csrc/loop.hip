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
#include <cstdio>
#include <cstring>

#include "cdr_internal.h"
#include "fin32.h"
#include "plan32.h"

namespace cdr {

constexpr int kLLState = 8;  // int64 words of ll_state

bool screen32_supported(const Ctx& c, int k);
bool screen32_step(Ctx& c, const double* C, int k, long long* dout, long long* hout, bool prof,
                   float* dbg, float* thr_out, long long* gate);
void plan32_point_side(const Ctx& c, double& xxmax, double& l1x);
void lloyd_step_f32x(Ctx& c, const double* C, int32_t k, int64_t* out, bool out_dev);
void zh_rebase(Ctx& c, const long long* gate);  // screen32.hip
constexpr int kRebaseEvery = 4;  // finalizes between 2-byte rebase opportunities

constexpr int kFinThreads = 512;
constexpr int kFinLds = 64 * 17;  // (k, d+1) cells staged in LDS (screen32 shapes)

// One workgroup.  Cnew is always written; C moves to Cnew unless the loop
// stops for the host, and then the next step's screen plan is built from it.
// Every global read is issued in independent batches (one workgroup: latency,
// not bandwidth, sets its time).
__global__ __launch_bounds__(kFinThreads) void ll_finalize(FinArgs a) {
  long long* __restrict__ state = a.state;
  const int k = a.k, d = a.d;
  double* __restrict__ C = a.C;
  double* __restrict__ Cnew = a.Cnew;
  const int cells = k * (d + 1);
  __shared__ long long lsum[kFinLds];
  __shared__ double lC[kFinLds];
  __shared__ double lref[2 * 64];
  // screen32 shapes: every input of the step is loaded in one batch (state,
  // all slices of the sums, the centroids, ref / mu) into LDS
  const bool staged = cells <= kFinLds && d <= 64;
  const double* __restrict__ ref = staged ? lref : a.ref;
  const double* __restrict__ Cin = staged ? lC : C;
  if (staged) {
    constexpr int PER = (kFinLds + kFinThreads - 1) / kFinThreads;
    long long p[PER][kRunSlices];
    double cv[PER];
    double rv = 0.0;
    const long long st0 = state[0];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * kFinThreads;
#pragma unroll
      for (int sl = 0; sl < kRunSlices; ++sl)
        p[i][sl] = (c < cells && sl < a.nslices) ? a.sums[(size_t)sl * cells + c] : 0;
      cv[i] = c < k * d ? C[c] : 0.0;
    }
    if (threadIdx.x < 2 * d) rv = a.ref[threadIdx.x];
    if (st0 == 0) return;  // uniform: the loop has stopped
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * kFinThreads;
      long long v = 0;
#pragma unroll
      for (int sl = 0; sl < kRunSlices; ++sl) v += p[i][sl];
      if (c < cells) lsum[c] = v;
      if (c < k * d) lC[c] = cv[i];
    }
    if (threadIdx.x < 2 * d) lref[threadIdx.x] = rv;
    __syncthreads();
  } else if (state[0] == 0) {
    return;
  }
  auto sum_at = [&](size_t e) -> long long {
    if (staged) return lsum[e];
    long long v = 0;
    for (int sl = 0; sl < a.nslices; ++sl) v += a.sums[(size_t)sl * cells + e];
    return v;
  };
  __shared__ double r_ss[kFinThreads], r_cross[kFinThreads], r_quad[kFinThreads];
  __shared__ int r_empty[kFinThreads];
  __shared__ int move, plan_next;
  const int t = threadIdx.x;
  const int d1 = d + 1;
  double ss = 0.0, cross = 0.0, quad = 0.0;
  int empty = 0;
  long long* cnt_out = reinterpret_cast<long long*>(Cnew + (size_t)k * d);
  for (int j = t; j < k; j += blockDim.x) cnt_out[j] = sum_at((size_t)j * d1 + d);
  if (a.fbc) {  // (uniform)
    const int fb = block_sum_counts(a.fbc, a.nwaves);
    if (t == 0) {
      a.fbc[a.nwaves] = 0;
      a.fbc[a.nwaves + 1] = fb;
      if (a.fb_acc) a.fb_acc[0] += fb;
    }
  }
#pragma unroll 4
  for (int e = t; e < k * d; e += blockDim.x) {
    const int j = e / d, f = e - j * d;
    const long long cnt = sum_at((size_t)j * d1 + d);
    // the host's np.ldexp(acc.astype(float64), -S) / counts (kmeans_plusplus.py)
    const double sj = ldexp((double)sum_at((size_t)j * d1 + f), -a.sbits);
    double m = sj / (double)cnt;
    if (a.round32) m = (double)(float)m;  // new_centroids has X's dtype (float32)
    Cnew[e] = m;
    if (cnt == 0) {
      empty = 1;
      continue;
    }
    const double c = Cin[e];
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
  for (int o = kFinThreads / 2; o > 0; o >>= 1) {  // fixed tree: deterministic
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
    const double inertia = a.x2 - 2.0 * r_cross[0] + r_quad[0];
    long long reason = kLLRun;
    int mv = 0;
    if (r_empty[0]) {
      reason = kLLEmpty;
    } else {
      const double sh = sqrt(sst);
      mv = 1;
      if (a.tol > 0.0 && !(sh > a.tol * (1.0 + a.margin))) {
        if (sh < a.tol * (1.0 - a.margin)) {
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
    plan_next = mv && reason == kLLRun;  // the loop goes on: plan its next step
  }
  __syncthreads();
  if (!move) return;
  for (int e = t; e < k * d; e += blockDim.x) {
    const double m = Cnew[e];  // this thread's own store above
    C[e] = m;
    if (staged) lC[e] = m;
  }
  // the next step's plan from the new centroids
  if (a.plan && plan_next) {
    __syncthreads();
    plan32_build(staged ? lC : Cnew, k, d, a.QH, a.MT, ref + d, a.sc, a.xxmax, a.l1x, state,
                 a.plan);
  }
}

// ll_finalize for the screen32 device plan (k <= 64, d <= 16), written for
// latency: a single workgroup between two full-GPU launches (fin32.h).  The
// fused screen32bs runs the same body in its last workgroup instead.
__global__ __launch_bounds__(512) void ll_finalize32(FinArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[kFin32Lds];
  fin32_body<512>(a, lds);
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
      const double v = (double)X[xidx(X, f, i, n_pad)] - ref[f];
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

void plan32_launch(Ctx& c, int k, int QH, int MT);  // screen32.hip
bool big_supported(const Ctx& c, int k);              // screen_big.hip
void big_plan_device(Ctx& c, int k, const double* dC, const double* dmu, const long long* gate);
bool big_step_dev(Ctx& c, int k, long long* dout, bool prof, const long long* gate);
void prof_end_screened(Ctx& c);                       // lloyd.hip

// Large-k plan of the loop's current centroids (begin, resume, and after
// each finalize that moved them); ll_ref + d holds mu as fp64.
static void ll_plan_big(Ctx& c) {
  big_plan_device(c, c.ll_k, c.ll_C.as<double>(), c.ll_ref.as<double>() + c.d,
                  c.ll_state.as<long long>());
}

static void ll_plan_shape(const Ctx& c, int& QH, int& MT) {
  QH = d4_of(c.d) / 4 <= 2 ? 1 : 2;
  MT = c.ll_k <= 32 ? 1 : 2;
}

// Device plan of the loop's current centroids (begin, resume); the plan
// buffer is sized for the screen32 layout of (k, d).
static void ll_plan(Ctx& c) {
  int QH, MT;
  ll_plan_shape(c, QH, MT);
  c.frag.ensure(plan32_layout(MT, c.ll_k, c.d).all);
  plan32_launch(c, c.ll_k, QH, MT);
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
  c.ll_devplan = screen32_supported(c, k) && !exp_env("CDR_NO_DEVPLAN");
  c.ll_devbig = !c.ll_devplan && big_supported(c, k) && !exp_env("CDR_NO_DEVPLAN");
  plan32_point_side(c, c.ll_xxmax, c.ll_l1x);
  c.ll_C.ensure(sizeof(double) * (size_t)k * d);
  c.ll_new.ensure(sizeof(double) * (size_t)k * (d + 1));
  c.ll_sums.ensure(sizeof(long long) * (size_t)k * (d + 1));
  c.ll_ref.ensure(sizeof(double) * 2 * d);
  c.ll_state.ensure(sizeof(long long) * kLLState);
  // screen32b's drift bounds (kept by ll_finalize32 only)
  const bool fin_old = exp_env("CDR_FIN_OLD") && std::atoi(exp_env("CDR_FIN_OLD"));
  c.bnd_ok = c.ll_devplan && !fin_old;
  c.bnd.ensure(kBndBytes);
  HIP_CHECK(hipMemsetAsync(c.bnd.p, 0, c.bnd.bytes, c.stream));
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
  c.ll_fin_count = 0;
  c.ll_hostplan_once = false;
  // the first step recomputes the running sums from scratch (see resume)
  c.run_valid = false;
  c.lab8_valid = false;
  c.zb_valid = false;
  c.big_valid = false;
  if (c.ll_devplan) ll_plan(c);
  if (c.ll_devbig) ll_plan_big(c);
  CDR_CATCH
}

}  // extern "C"

namespace cdr {

static void ll_enqueue_assign(Ctx& c, int64_t* dsums) {
  long long* dout = dsums ? reinterpret_cast<long long*>(dsums) : c.ll_sums.as<long long>();
  long long* state = c.ll_state.as<long long>();
  if (c.ll_devplan && !c.ll_hostplan_once) {
    const bool prof = prof_step_begin(c);
    // single process: no published copy, ll_finalize reads the running sums
    screen32_step(c, nullptr, c.ll_k, dsums ? dout : nullptr, nullptr, prof, nullptr, nullptr,
                  state);
    // (after the step: it may allocate run_sums)
    c.ll_fin_sums = dsums ? dout : c.run_sums.as<long long>();
    c.ll_fin_slices = dsums ? 1 : kRunSlices;
    c.ll_fin_devstep = true;
    c.last_k = c.ll_k;
    c.have_labels = true;
    c.last_screened = true;
    c.last_fallback = -1;
  } else if (c.ll_devbig && !c.ll_hostplan_once) {
    // large k: screen_big on the plan big_plan_kernel built after the last
    // finalize; the sums go to dout, the loop state gates every kernel
    const bool prof = prof_step_begin(c);
    if (!big_step_dev(c, c.ll_k, dout, prof, state))
      CDR_FAIL(CDR_ERR_STATE, "lloyd loop: large-k step not supported");
    if (prof) prof_end_screened(c);
    c.ll_fin_sums = dout;
    c.ll_fin_slices = 1;
    c.ll_fin_devstep = false;
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
    c.ll_fin_sums = dout;
    c.ll_fin_slices = 1;
    c.ll_fin_devstep = false;
    if (st[0]) {
      std::vector<double> Ch((size_t)c.ll_k * c.d);
      HIP_CHECK(hipMemcpy(Ch.data(), c.ll_C.p, sizeof(double) * Ch.size(), hipMemcpyDeviceToHost));
      lloyd_step_f32x(c, Ch.data(), c.ll_k, reinterpret_cast<int64_t*>(dout), true);
    }
  }
  c.ll_enqueued += 1;
}

// The finalize's arguments for the step just assigned.
FinArgs ll_fin_args(Ctx& c) {
  const int kd = c.ll_k * c.d;
  const bool r32 = (c.ll_flags & 1) != 0;
  FinArgs a;
  a.sums = c.ll_fin_sums;
  a.nslices = c.ll_fin_slices;
  a.k = c.ll_k;
  a.d = c.d;
  a.sbits = c.scale_bits;
  a.round32 = r32 ? 1 : 0;
  a.tol = c.ll_tol;
  // fp64 sum of kd squares errs by < kd 2^-53 relative; float32 centroids are
  // compared by NumPy in float32 (kd 2^-23)
  a.margin = r32 ? std::ldexp((double)(kd + 2), -22) : 1e-9;
  a.x2 = c.ll_x2;
  a.ref = c.ll_ref.as<double>();
  a.C = c.ll_C.as<double>();
  a.Cnew = c.ll_new.as<double>();
  a.state = c.ll_state.as<long long>();
  a.fbc = c.ll_fin_devstep ? c.fb_count.as<int>() : nullptr;
  a.nwaves = c.fb_regions;
  c.fb_accum.ensure(2 * sizeof(long long));
  a.fb_acc = c.prof_on ? c.fb_accum.as<long long>() : nullptr;
  a.plan = c.ll_devplan ? static_cast<unsigned char*>(c.frag.p) : nullptr;
  ll_plan_shape(c, a.QH, a.MT);
  a.sc = std::ldexp(1.0, c.sigma);
  a.xxmax = c.ll_xxmax;
  a.l1x = c.ll_l1x;
  a.bnd = c.bnd_ok ? c.bnd.as<long long>() : nullptr;
  // 2-byte words: a rebase may be decided every kRebaseEvery-th finalize
  // (the first one sets the base), each followed by zh_rebase_kernel
  a.rebase_ok = c.ll_fin_count % kRebaseEvery == 0 ? 1 : 0;
  a.abl = 0;
  a.tprof = nullptr;
#ifdef CDR_EXPERIMENTS
  if (const char* e = exp_env("CDR_FIN_ABL")) a.abl = std::atoi(e);
  static unsigned long long* fin_tp = nullptr;
  if (exp_env("CDR_FIN_TPROF")) {
    if (!fin_tp) HIP_CHECK(hipMalloc(&fin_tp, sizeof(unsigned long long) * 16));
    HIP_CHECK(hipMemsetAsync(fin_tp, 0, sizeof(unsigned long long) * 16, c.stream));
    a.tprof = fin_tp;
  }
  if (exp_env("CDR_FIN_NOPLAN")) a.plan = nullptr;  // timing experiments only
#endif
  return a;
}

static void ll_enqueue_finalize(Ctx& c, const int64_t* dsums) {
  if (dsums && reinterpret_cast<const long long*>(dsums) != c.ll_fin_sums)
    CDR_FAIL(CDR_ERR_ARG, "lloyd finalize: pass the buffer given to the assign");
  const FinArgs a = ll_fin_args(c);
  // screen32 device plan: the latency-oriented finalize (CDR_FIN_OLD=1: the
  // generic one, for comparisons)
  static const bool fin_old = exp_env("CDR_FIN_OLD") && std::atoi(exp_env("CDR_FIN_OLD"));
  if (a.plan && c.ll_k <= 64 && c.d <= 16 && a.nslices <= kRunSlices && !fin_old) {
    hipLaunchKernelGGL(ll_finalize32, dim3(1), dim3(512), 0, c.stream, a);
    HIP_CHECK(hipGetLastError());
#ifdef CDR_EXPERIMENTS
    if (a.tprof) {  // phase times (us from the start; 100 MHz counter), to stderr
      unsigned long long h[16];
      HIP_CHECK(hipMemcpyAsync(h, a.tprof, sizeof(h), hipMemcpyDeviceToHost, c.stream));
      HIP_CHECK(hipStreamSynchronize(c.stream));
      fprintf(stderr, "FINTP");
      for (int i = 1; i < 10; ++i)
        fprintf(stderr, " %d:%.2f", i, h[i] ? (double)(h[i] - h[0]) * 0.01 : -1.0);
      fprintf(stderr, "\n");
    }
#endif
    if (a.rebase_ok && a.bnd) zh_rebase(c, c.ll_state.as<long long>());  // (gated on the device)
  } else {
    hipLaunchKernelGGL(ll_finalize, dim3(1), dim3(kFinThreads), 0, c.stream, a);
  }
  HIP_CHECK(hipGetLastError());
  c.ll_fin_count += 1;
  if (c.ll_devbig) ll_plan_big(c);  // the next step's plan (skipped once the loop stopped)
  if (c.ll_fin_devstep && c.prof_cur >= 0) prof_mark(c, 2);
}

}  // namespace cdr

extern "C" {

int cdr_lloyd_enqueue_assign(cdr_ctx* h, int64_t* dsums) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  ll_require(c);
  ll_enqueue_assign(c, dsums);
  CDR_CATCH
}

int cdr_lloyd_enqueue_finalize(cdr_ctx* h, const int64_t* dsums) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  ll_require(c);
  ll_enqueue_finalize(c, dsums);
  CDR_CATCH
}

int cdr_lloyd_enqueue_steps(cdr_ctx* h, int32_t m) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  if (m < 0) CDR_FAIL(CDR_ERR_ARG, "m must be >= 0");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  ll_require(c);
  // with a communicator: the step's sums go to comm_buf, which RCCL sums in
  // place over the ranks on this stream before the finalize reads it
  const size_t cells = (size_t)c.ll_k * (c.d + 1);
  int64_t* buf = nullptr;
  if (c.comm) {
    c.comm_buf.ensure(sizeof(long long) * cells);
    buf = c.comm_buf.as<int64_t>();
  }
  for (int32_t i = 0; i < m; ++i) {
    ll_enqueue_assign(c, buf);
    if (c.comm) comm_allreduce_i64(c, reinterpret_cast<long long*>(buf), cells);
    ll_enqueue_finalize(c, buf);
  }
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
  c.ll_hostplan_once = host_plan_once != 0;
  if (c.ll_devplan && !c.ll_hostplan_once) ll_plan(c);
  if (c.ll_devbig && !c.ll_hostplan_once) ll_plan_big(c);
  HIP_CHECK(hipStreamSynchronize(c.stream));  // C belongs to the caller
  // Steps enqueued after the stop did nothing, but the host marked the
  // running sums valid after each of them; a full (non-DELTA) step that was
  // among them never zeroed and rebuilt them.  The next step starts afresh.
  c.run_valid = false;
  c.lab8_valid = false;
  c.zb_valid = false;
  c.big_valid = false;
  CDR_CATCH
}

int cdr_lloyd_end(cdr_ctx* h) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  h->c.ll_on = false;
  CDR_CATCH
}

}  // extern "C"
