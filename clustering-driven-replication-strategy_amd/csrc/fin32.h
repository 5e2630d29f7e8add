// fin32.h — the device loop's finalize for screen32 device plans (k <= 64,
// d <= 16): the means, the stop decision, the drift bounds
// and the next step's plan, as a body that runs on one workgroup of 512
// threads (ll_finalize32, loop.hip) or 256.  (Run by the last workgroup of
// screen32bs instead of its own launch it cost 14-25 us more per step: the
// tail's spills and a cold single-workgroup finalize)
//
// The body is written for 512 "virtual threads" vt: vt owns row j = vt / 8
// and the feature pair 2 (vt % 8), 2 (vt % 8) + 1 of it, from the loads of
// the sums to the plan entries of those two elements.  A workgroup of NT
// threads runs 512 / NT of them per thread: thread t of wave w takes the
// virtual threads 128 w + 64 v + lane (v < 512 / NT), i.e. the same lane of
// the virtual waves 2 w + v, so every shuffle and every per-wave partial is
// the 512-thread one and the reductions (shift, inertia) keep one
// association whatever NT is: the same bits from both kernels.
//   loads (every slice of its cells, its centroid values: one round trip)
//   -> means, shift / inertia terms -> wave sums -> [sync] -> the decision
//   (every thread, from the 8 wave partials) -> fp16 halves, fp32 centroid,
//   row values staged -> [sync] -> row sums (one thread per row, the host's
//   order), nearest-centroid distances (8 lanes per row) -> maxima -> [sync]
//   -> bounds (every thread) -> fragments, C operand, prune block.
// Same results as ll_finalize + plan32_build (same fp64 operations per value;
// the row sums in the same sequential order).
#pragma once
#include "cdr_internal.h"
#include "plan32.h"

namespace cdr {

enum : long long { kLLRun = 0, kLLConverged = 1, kLLEmpty = 2, kLLHostPlan = 3, kLLAmbiguous = 4 };

struct FinArgs {
  const long long* sums;  // nslices x (k, d+1) int64 fixed-point sums | counts
  int nslices;
  int k, d, sbits, round32;
  double tol, margin, x2;
  const double* ref;  // inertia reference row (d), then mu (d)
  double* C;          // current centroids (k x d)
  double* Cnew;       // k x d means, then k counts (int64)
  long long* state;
  // screen32's fallback counter (device plan steps): fbc[nwaves] -> [nwaves+1]
  int* fbc;
  int nwaves;
  long long* fb_acc;
  // device plan of the next step (null: host plan)
  unsigned char* plan;
  int QH, MT;
  double sc, xxmax, l1x;
  // screen32b's drift bounds (Ctx::bnd; null: not kept): when the centroids
  // move, W_j += M + delta_j (int64, 2^-40 units, rounded up), with
  // delta_j >= ||chat_j(new) - chat_j(old)|| and M = max_j delta_j; then W_j
  // rounded up and down to fp32 for the next screen, and the 2-byte words'
  // tables (plan32.h kBnd*)
  long long* bnd;
  // a rebase of the 2-byte words may be decided at this step (the host then
  // runs zh_rebase_kernel before the next screen; screen32.hip)
  int rebase_ok;
  int abl;  // timing experiments only (0 in the product build)
  unsigned long long* tprof;  // (experiments build: phase timestamps, thread 0)
};

// fp64 -> fp32 rounded up / down (W_j for screen32b)
__device__ inline float f32_up(double v) {
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, INFINITY);
  return f;
}
__device__ inline float f32_dn(double v) {
  float f = (float)v;
  if ((double)f > v) f = nextafterf(f, -INFINITY);
  return f;
}

// The finalize's arguments for the current step (loop.hip; host).
FinArgs ll_fin_args(Ctx& c);

// LDS the body needs (the caller's)
constexpr size_t kFin32Lds = 2 * (64 * 16 * 2) + 64 * 16 * 8 + 64 * 16 * 4 + 64 * 8 +
                             8 * 8 * 9 + 8 * 4 * 2;

template <int NT>
__device__ __forceinline__ void fin32_body(const FinArgs& a, unsigned char* __restrict__ lds) {
  static_assert(NT == 512 || NT == 256, "512 virtual threads");
  constexpr int V = 512 / NT;
  long long* __restrict__ state = a.state;
  const int t = threadIdx.x;
#ifdef CDR_EXPERIMENTS
#define FIN_TP(i) \
  if (a.tprof && t == 0) a.tprof[i] = __builtin_amdgcn_s_memrealtime()
#else
#define FIN_TP(i)
#endif
  FIN_TP(0);
  if (a.abl & 8) {  // (the step still counts, so the host's polling goes on)
    if (t == 0) state[1] += 1;
    return;
  }
  // LDS carve-up
  _Float16* m2h = reinterpret_cast<_Float16*>(lds);
  _Float16* m2l = m2h + 64 * 16;
  double* vrow = reinterpret_cast<double*>(m2l + 64 * 16);
  float* c32 = reinterpret_cast<float*>(vrow + 64 * 16);
  double* cc = reinterpret_cast<double*>(c32 + 64 * 16);
  double* r_ss = cc + 64;
  double* r_cross = r_ss + 8;
  double* r_quad = r_cross + 8;
  double* r_dm = r_quad + 8;
  double* r_A = r_dm + 8;
  double* x_cc = r_A + 8;
  double* x_l1 = x_cc + 8;
  double* x_ca = x_l1 + 8;
  double* x_ec = x_ca + 8;
  int* r_empty = reinterpret_cast<int*>(x_ec + 8);
  int* r_fb = r_empty + 8;

  const int k = a.k, d = a.d, d1 = d + 1, cells = k * d1;
  const int lane = t & 63, w = t >> 6;
  int vt[V], vw[V], j[V], f0[V];
  bool row[V], v0[V], v1[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    vt[v] = NT == 512 ? t : 128 * w + 64 * v + lane;
    vw[v] = vt[v] >> 6;
    j[v] = vt[v] >> 3;
    f0[v] = 2 * (vt[v] & 7);
    row[v] = j[v] < k;
    v0[v] = row[v] && f0[v] < d;
    v1[v] = row[v] && f0[v] + 1 < d;
  }
  // ---- loads (the slices of the sums: per virtual thread, below) ----
  double c0[V], c1[V], r0[V], r1[V], mu0[V], mu1[V];
  bool whead[V];
  long long w_old[V], g_old[V];
  unsigned char* const bb = reinterpret_cast<unsigned char*>(a.bnd);
#pragma unroll
  for (int v = 0; v < V; ++v) {
    c0[v] = v0[v] ? a.C[j[v] * d + f0[v]] : 0.0;
    c1[v] = v1[v] ? a.C[j[v] * d + f0[v] + 1] : 0.0;
    r0[v] = v0[v] ? a.ref[f0[v]] : 0.0;
    r1[v] = v1[v] ? a.ref[f0[v] + 1] : 0.0;
    mu0[v] = v0[v] ? a.ref[d + f0[v]] : 0.0;
    mu1[v] = v1[v] ? a.ref[d + f0[v] + 1] : 0.0;
    whead[v] = a.bnd && row[v] && (vt[v] & 7) == 0;
    w_old[v] = whead[v] ? a.bnd[j[v]] : 0;
    // the 2-byte words' base (plan32.h kBnd*)
    g_old[v] = whead[v] ? reinterpret_cast<const long long*>(bb + kBndG)[j[v]] : 0;
  }
  int hdr0 = 0, e0c = 0;
  if (a.bnd) {
    hdr0 = reinterpret_cast<const int*>(bb + kBndHdr)[0];
    e0c = reinterpret_cast<const int*>(bb + kBndHdr)[2];
  }
  const long long st0 = state[0];
  // the per-wave fallback counts (the step's total: the decision sync below)
  // (eight loads in flight per thread: a rolled loop waited for each one)
  int fbv = 0;
  if (a.fbc) {
    int acc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = t + u * NT;
      acc[u] = i < a.nwaves ? a.fbc[i] : 0;
    }
    for (int i = t + 8 * NT; i < a.nwaves; i += NT) acc[0] += a.fbc[i];
#pragma unroll
    for (int u = 0; u < 8; ++u) fbv += acc[u];
  }
  // ---- means, shift / inertia terms ----
  double* __restrict__ Cnew = a.Cnew;
  long long* cnt_out = reinterpret_cast<long long*>(Cnew + (size_t)k * d);
  double m0[V], m1[V], dlt[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    // every slice's cells of this virtual thread in one round trip
    long long s0[kRunSlices], s1[kRunSlices], sn[kRunSlices];
#pragma unroll
    for (int sl = 0; sl < kRunSlices; ++sl) {
      const bool on = sl < a.nslices;
      const long long* base = a.sums + (size_t)sl * cells + (size_t)j[v] * d1;
      s0[sl] = on && v0[v] ? base[f0[v]] : 0;
      s1[sl] = on && v1[v] ? base[f0[v] + 1] : 0;
      sn[sl] = on && row[v] ? base[d] : 0;
    }
    long long S0 = 0, S1 = 0, cnt = 0;
#pragma unroll
    for (int sl = 0; sl < kRunSlices; ++sl) {
      S0 += s0[sl];
      S1 += s1[sl];
      cnt += sn[sl];
    }
    if (v == 0) {  // (after the first loads: their round trip overlaps the state's)
      if (st0 == 0) return;  // uniform: the loop has stopped
      if (a.abl & 1) {  // (timing: the loads only)
        if (S0 + S1 + cnt == 0x7fffffffffffffffll || c0[0] + r0[0] == 0x1p1000) state[7] = 1;
        if (t == 0) state[1] += 1;
        return;
      }
    }
    if (row[v] && (vt[v] & 7) == 0) cnt_out[j[v]] = cnt;
    // the host's np.ldexp(acc.astype(float64), -S) / counts (kmeans_plusplus.py)
    const double sj0 = ldexp((double)S0, -a.sbits), sj1 = ldexp((double)S1, -a.sbits);
    m0[v] = sj0 / (double)cnt;
    m1[v] = sj1 / (double)cnt;
    if (a.round32) {
      m0[v] = (double)(float)m0[v];
      m1[v] = (double)(float)m1[v];
    }
    if (v0[v]) Cnew[j[v] * d + f0[v]] = m0[v];
    if (v1[v]) Cnew[j[v] * d + f0[v] + 1] = m1[v];
    double ss = 0.0, cross = 0.0, quad = 0.0;
    int empty = row[v] && cnt == 0;
    if (row[v] && cnt != 0) {
      if (v0[v]) {
        const double df = m0[v] - c0[v], ct = c0[v] - r0[v];
        ss += df * df;
        cross += ct * (sj0 - (double)cnt * r0[v]);
        quad += (double)cnt * (ct * ct);
      }
      if (v1[v]) {
        const double df = m1[v] - c1[v], ct = c1[v] - r1[v];
        ss += df * df;
        cross += ct * (sj1 - (double)cnt * r1[v]);
        quad += (double)cnt * (ct * ct);
      }
    }
    // how far centroid j moves (its 8 threads' features; screen32b's drift):
    // fp64 errs by < 20 2^-53 relative here, sc is a power of two
    double dq = 0.0;
    if (v0[v]) dq += (m0[v] - c0[v]) * (m0[v] - c0[v]);
    if (v1[v]) dq += (m1[v] - c1[v]) * (m1[v] - c1[v]);
    dq += __shfl_xor(dq, 1);
    dq += __shfl_xor(dq, 2);
    dq += __shfl_xor(dq, 4);
    dlt[v] = sqrt(dq) * a.sc * (1.0 + 0x1p-45);
    double dmx = row[v] ? dlt[v] : 0.0;
#pragma unroll
    for (int o = 32; o >= 8; o >>= 1) dmx = fmax(dmx, __shfl_xor(dmx, o));
    int fbw = v == 0 ? fbv : 0;  // (the fallback total: integers, any grouping)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {  // fixed pattern: deterministic
      ss += __shfl_xor(ss, o);
      cross += __shfl_xor(cross, o);
      quad += __shfl_xor(quad, o);
      empty |= __shfl_xor(empty, o);
      fbw += __shfl_xor(fbw, o);
    }
    if (lane == 0) {
      r_dm[vw[v]] = dmx;
      r_ss[vw[v]] = ss;
      r_cross[vw[v]] = cross;
      r_quad[vw[v]] = quad;
      r_empty[vw[v]] = empty;
      r_fb[vw[v]] = fbw;
    }
    if constexpr (V > 1) asm volatile("" ::: "memory");  // (one virtual thread's loads at a time)
  }
  FIN_TP(1);
  __syncthreads();
  FIN_TP(2);
  if (t == 0 && a.fbc) {
    int fb = 0;
    for (int q = 0; q < 8; ++q) fb += r_fb[q];
    a.fbc[a.nwaves] = 0;
    a.fbc[a.nwaves + 1] = fb;
    if (a.fb_acc) a.fb_acc[0] += fb;
  }
  // ---- the decision (every thread, the same fixed order) ----
  double sst = 0.0, crs = 0.0, qd = 0.0;
  int emp = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    sst += r_ss[q];
    crs += r_cross[q];
    qd += r_quad[q];
    emp |= r_empty[q];
  }
  long long reason = kLLRun;
  int mv = 0;
  if (emp) {
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
  if (t == 0) {
    if (mv) state[1] += 1;
    if (reason != kLLRun) {
      state[0] = 0;
      state[2] = reason;
    }
    state[3] = __double_as_longlong(sst);
    state[4] = __double_as_longlong(a.x2 - 2.0 * crs + qd);
  }
  if (!mv) return;
  double M = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q) M = fmax(M, r_dm[q]);
  long long wn[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    if (v0[v]) a.C[j[v] * d + f0[v]] = m0[v];
    if (v1[v]) a.C[j[v] * d + f0[v] + 1] = m1[v];
    wn[v] = 0;
    if (whead[v]) {  // screen32b's drift bounds of this move
      double inc = (M + dlt[v]) * (1.0 + 0x1p-50);
      if (!(inc < 0x1p10)) inc = 0x1p10;  // (NaN too)
      // saturating: past 2^52 units the fp64 value is no longer exact and
      // every bound test fails from then on (W up = inf)
      wn[v] = w_old[v] >= (1LL << 60) ? w_old[v] : w_old[v] + (long long)ceil(ldexp(inc, 40));
      a.bnd[j[v]] = wn[v];
      const double wvv = ldexp((double)wn[v], -40);
      float* wf = reinterpret_cast<float*>(a.bnd + 64);
      wf[j[v]] = wn[v] < (1LL << 52) ? f32_up(wvv) : INFINITY;
      wf[64 + j[v]] = f32_dn(wvv);
    }
  }
  if (a.bnd) {  // (uniform) the 2-byte words' tables
    // A_j = W_j - G_j: what the current base has accumulated.  Rebase (G_j =
    // W_j, every kept word re-encoded by the next screen) when the base was
    // never set, when the code's 2^-6 truncation of A reaches half the
    // step's drift budget (A > 32 M), when the drift has fallen to twice the
    // code floor 2^E0 (margins near M would not be representable), or when
    // A nears the code range (2^(E0 + 16)).  The floor follows the drift,
    // E0 = floor(log2(M / 64)) (a margin below M is spent within a step;
    // the range reaches ~1000 M), so a decaying drift rebases rarely
#pragma unroll
    for (int v = 0; v < V; ++v) {
      double am = whead[v] ? ldexp((double)(wn[v] - g_old[v]), -40) : 0.0;
#pragma unroll
      for (int o = 32; o >= 8; o >>= 1) am = fmax(am, __shfl_xor(am, o));
      if (lane == 0) r_A[vw[v]] = am;
    }
    __syncthreads();
    double Amax = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) Amax = fmax(Amax, r_A[q]);
    // (only at the steps the host follows with zh_rebase_kernel)
    const bool rebase = a.rebase_ok &&
                        (hdr0 == 0 || (M > 0.0 && (Amax > 32.0 * M || ldexp(1.0, e0c + 1) > M)) ||
                         Amax > ldexp(1.0, e0c + 14));
    int e0n = e0c;
    if (rebase) {
      if (M > 0.0) e0n = ilogb(M * 0x1p-6);
      else if (hdr0 == 0) e0n = -20;
      e0n = e0n < -120 ? -120 : (e0n > 100 ? 100 : e0n);
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      if (!whead[v]) continue;
      const int jj = j[v];
      const bool exact = wn[v] < (1LL << 52);  // (saturated W: every test fails)
      const long long g_new = rebase ? wn[v] : g_old[v];
      reinterpret_cast<long long*>(bb + kBndG)[jj] = g_new;
      // (the words are in the new base when the next screen tests them)
      reinterpret_cast<unsigned*>(bb + kBndT)[jj] =
          exact ? zb16_thr(f32_up(ldexp((double)(wn[v] - g_new), -40)), e0n) : 1022u;
      reinterpret_cast<float*>(bb + kBndWdg)[jj] =
          exact ? f32_dn(ldexp((double)(wn[v] - g_new), -40)) : -1.0f;
      reinterpret_cast<float*>(bb + kBndDG)[jj] =
          rebase ? f32_up(ldexp((double)(g_new - g_old[v]), -40)) : 0.0f;
    }
    if (t == 0) {
      int* hd = reinterpret_cast<int*>(bb + kBndHdr);
      hd[0] = 1;
      hd[1] = e0c;
      hd[2] = e0n;
      hd[3] = rebase ? 1 : 0;
    }
  }
  FIN_TP(3);
  if (!a.plan || reason != kLLRun || (a.abl & 2)) return;
  // ---- the next step's plan (plan32_build, per element) ----
  unsigned char* __restrict__ plan = a.plan;
  const int QH = a.QH, MT = a.MT;
  const Plan32Layout L = plan32_layout(MT, k, d);
  plan_h8* frag = reinterpret_cast<plan_h8*>(plan);
  float* cinit = reinterpret_cast<float*>(plan + L.cinit);
  double* cent = reinterpret_cast<double*>(plan + L.cent);
  float* pc = reinterpret_cast<float*>(plan + L.prune);
  float* pE = pc + 64 * kPrStr;
  float* ph = pE + 64;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int jj = j[v];
    const double vv[2] = {v0[v] ? (m0[v] - mu0[v]) * a.sc : 0.0,
                          v1[v] ? (m1[v] - mu1[v]) * a.sc : 0.0};
    const double mm[2] = {m0[v], m1[v]};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int f = f0[v] + u;
      const double x = vv[u];
      const _Float16 hi = f64_to_f16(x);
      const _Float16 lo = f64_to_f16(x - (double)hi);
      m2h[jj * 16 + f] = f64_to_f16(-2.0 * (double)hi);
      m2l[jj * 16 + f] = f64_to_f16(-2.0 * (double)lo);
      vrow[jj * 16 + f] = x;
      const float cf = (float)x;
      c32[jj * 16 + f] = cf;
      pc[jj * kPrStr + f] = cf;
      if (row[v] && f < d) cent[jj * d + f] = mm[u];
    }
    const int p = vt[v] & 7;
    if (p < 2) pc[jj * kPrStr + 16 + 2 * p] = 0.0f, pc[jj * kPrStr + 17 + 2 * p] = 0.0f;
  }
  FIN_TP(4);
  __syncthreads();
  FIN_TP(5);
  // ---- row sums (host order), nearest-centroid distances, maxima ----
  double ec[V], sm[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int jj = j[v];
    double s = 0.0, l1 = 0.0, ca = 0.0, e2 = 0.0;
    const bool head = (vt[v] & 7) == 0 && row[v];
    if (head) {
      for (int f = 0; f < d; ++f) {
        const double x = vrow[jj * 16 + f];
        s += x * x;
        l1 += fabs(x);
        ca = fmax(ca, fabs(x));
        const double r = (double)c32[jj * 16 + f] - x;  // exact
        e2 += r * r;
      }
      cc[jj] = s;
    }
    ec[v] = plan32_prune_ec(e2, s);
    double smv = INFINITY;  // smallest squared distance of c32_j to another c32
    if (row[v] && !(a.abl & 4)) {
      // own row in registers, four partial sums per pair (a short dependency
      // chain; every term >= 0 and at most 6 roundings on any path, within
      // plan32_prune_h's 2^-44 margin)
      float cj[16];
#pragma unroll
      for (int f = 0; f < 16; ++f) cj[f] = c32[jj * 16 + f];
      for (int q = vt[v] & 7; q < k; q += 8) {
        if (q == jj) continue;
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int f = 0; f < 16; ++f) {
          const double df = (double)cj[f] - (double)c32[q * 16 + f];  // exact
          acc[f & 3] += df * df;
        }
        smv = fmin(smv, (acc[0] + acc[1]) + (acc[2] + acc[3]));
      }
    }
    if (v == 0) FIN_TP(6);
    smv = fmin(smv, __shfl_xor(smv, 1));
    smv = fmin(smv, __shfl_xor(smv, 2));
    smv = fmin(smv, __shfl_xor(smv, 4));
    sm[v] = smv;
    double ccmax = head ? s : 0.0, l1c = head ? l1 : 0.0, cabs = head ? ca : 0.0,
           ecmax = head ? ec[v] : 0.0;
#pragma unroll
    for (int o = 32; o >= 8; o >>= 1) {  // max is exact: any order
      ccmax = fmax(ccmax, __shfl_xor(ccmax, o));
      l1c = fmax(l1c, __shfl_xor(l1c, o));
      cabs = fmax(cabs, __shfl_xor(cabs, o));
      ecmax = fmax(ecmax, __shfl_xor(ecmax, o));
    }
    if (lane == 0) {
      x_cc[vw[v]] = ccmax;
      x_l1[vw[v]] = l1c;
      x_ca[vw[v]] = cabs;
      x_ec[vw[v]] = ecmax;
    }
  }
  FIN_TP(7);
  __syncthreads();
  FIN_TP(8);
  double ccmax = 0.0, l1c = 0.0, cabs = 0.0, ecmax = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    ccmax = fmax(ccmax, x_cc[q]);
    l1c = fmax(l1c, x_l1[q]);
    cabs = fmax(cabs, x_ca[q]);
    ecmax = fmax(ecmax, x_ec[q]);
  }
  if (!(cabs <= 1024.0)) {  // fp16 split range (and NaN) guard: the host plans this step
    if (t == 0) {
      state[0] = 0;
      state[2] = kLLHostPlan;
    }
    return;
  }
  double D;
  float thr0;
  plan32_bounds(ccmax, l1c, a.xxmax, a.l1x, QH, D, thr0);
  if (t == 0) {
    reinterpret_cast<float*>(plan + L.thr)[0] = thr0;
    reinterpret_cast<float*>(plan + L.thr)[1] = (float)D;
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    if ((vt[v] & 7) == 0) {
      pE[j[v]] = plan32_prune_E(plan32_prune_dn(a.xxmax), row[v] ? ec[v] : 0.0);
      ph[j[v]] = row[v] ? plan32_prune_h(sm[v], ec[v], ecmax) : INFINITY;
    }
  }
  for (int idx = t; idx < MT * 64; idx += NT) {  // the layout of plan32_lane
    const int m = idx >> 6, ln = idx & 63;
    const int h = ln >> 5, jr = 32 * m + (ln & 31);
    plan_h8 A1, A3;
    for (int i = 0; i < 8; ++i) {
      A1[i] = (_Float16)0.0f;
      A3[i] = (_Float16)0.0f;
    }
    for (int uq = 0; uq < QH; ++uq)
      for (int i = 0; i < 4; ++i) {
        const int f = 4 * (QH * h + uq) + i;
        if (jr >= k || f >= d) continue;
        const _Float16 x = m2h[jr * 16 + f], y = m2l[jr * 16 + f];
        if (QH == 1) {
          A1[i] = x;
          A1[4 + i] = x;
          A3[i] = y;
        } else {
          A1[4 * uq + i] = x;
          A3[4 * uq + i] = y;
        }
      }
    frag[(m * 2 + 0) * 64 + ln] = A1;
    frag[(m * 2 + 1) * 64 + ln] = A3;
  }
  for (int idx = t; idx < MT * 16 * 64; idx += NT) {
    const int ln = idx & 63, mi = idx >> 6, m = mi >> 4, i = mi & 15;
    const int rw = 32 * m + 8 * (i >> 2) + 4 * (ln >> 5) + (i & 3);
    cinit[idx] = rw < k ? (float)(cc[rw] + D) : 1.0e30f;
  }
  FIN_TP(9);
#undef FIN_TP
}

}  // namespace cdr
