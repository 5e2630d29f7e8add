// cdr_internal.h — shared definitions for the libcdr HIP sources (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <string>
#include <vector>

#include "../../include/cdr.h"

namespace cdr {

// Error plumbing: every C entry point is wrapped in CDR_TRY / CDR_CATCH so a
// failure never escapes as a C++ exception across the C ABI.
void set_error(const std::string& msg);

struct Error {
  int code;
  std::string msg;
};

#define CDR_FAIL(code_, msg_)                  \
  do {                                         \
    throw ::cdr::Error{(code_), (msg_)};       \
  } while (0)

#define HIP_CHECK(expr)                                                       \
  do {                                                                        \
    hipError_t e_ = (expr);                                                   \
    if (e_ != hipSuccess)                                                     \
      CDR_FAIL(CDR_ERR_HIP, std::string(#expr " failed: ") +                 \
                                hipGetErrorString(e_) + " @" + __FILE__ +     \
                                ":" + std::to_string(__LINE__));              \
  } while (0)

#define CDR_TRY try {
#define CDR_CATCH                                             \
  }                                                           \
  catch (const ::cdr::Error& e) {                             \
    ::cdr::set_error(e.msg);                                  \
    return e.code;                                            \
  }                                                           \
  catch (const std::exception& e) {                           \
    ::cdr::set_error(std::string("internal: ") + e.what());   \
    return CDR_ERR_STATE;                                     \
  }                                                           \
  return CDR_OK;

// Device buffer that grows on demand (never shrinks until the context dies).
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t nbytes);
  void release();
  template <typename T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// Pinned host staging buffer.
struct HostBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t nbytes);
  void release();
  template <typename T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

constexpr int kSeedBlock = 8192;  // NumPy reduction buffer (add.reduce chunk)
// screen32's running sums are kept in kRunSlices copies (workgroup b adds into
// slice b % kRunSlices: 1/16 of the atomic contention); readers sum them.
constexpr int kRunSlices = 16;

// Point layout in HBM.  F32X points (float, x32): "quad-interleaved SoA",
// features grouped in quads; quad q of point i is 4 consecutive values at
// ((q * n_pad) + i) * 4.  One 16-byte load gives a lane four features of one
// point, and a wave reading quad q of 64 consecutive points reads 1 KiB
// contiguously.  d is padded to d4 = ceil(d/4)*4 with zero features.
// F64 points (double, x64): planar, feature f of point i at f * n_pad + i.
// The F64 kernels read a point's features one at a time, and in quads the
// zero padding (d = 5 -> 8) made every pass over the points read 64 bytes per
// point for 40.  The index follows the element type, so a kernel templated on
// it indexes either copy.
__host__ __device__ __forceinline__ int64_t xidx(const float*, int64_t f, int64_t i, int64_t n_pad) {
  return (((f >> 2) * n_pad) + i) * 4 + (f & 3);
}
__host__ __device__ __forceinline__ int64_t xidx(const double*, int64_t f, int64_t i, int64_t n_pad) {
  return f * n_pad + i;
}
__host__ __device__ __forceinline__ int d4_of(int d) { return (d + 3) & ~3; }
constexpr int kPointGroup = 64;   // points per wave iteration in the screen

// Ablation and A/B switches of the experiments build (-DCDR_EXPERIMENTS,
// libcdr_exp.so): the product library ignores them and always takes the
// default path.  The switches the tests use to reach a tested alternative
// (CDR_BOUNDS, CDR_NO_DELTA, CDR_S32B_SPLIT, CDR_S32BS_SPLIT, CDR_EXACT_ASSIGN,
// CDR_F64_SERIAL, CDR_F64S_FORCE_CHAIN, CDR_GROUPBY_SORT, CDR_GB_BLOCK,
// CDR_GB_BALLOT, CDR_GB_PASS3) are read with getenv in both builds.
inline const char* exp_env(const char* name) {
#ifdef CDR_EXPERIMENTS
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  hipEvent_t ev_begin = nullptr, ev_end = nullptr;

  // ---- points (one shard) ----
  int64_t n = 0;      // real points
  int64_t n_pad = 0;  // padded to a multiple of kSeedBlock (rows >= n are 0)
  int32_t d = 0;
  int32_t mode = 0;        // CDR_MODE_*
  int32_t scale_bits = 0;  // F32X fixed-point scale S
  DevBuf x32;              // F32X: float  [d4/4][n_pad][4]   (xidx)
  DevBuf x64;              // F64 : double [d4][n_pad] planar  (xidx)
  std::vector<double> fmin, fmax;  // per-feature min / max (host)
  // this shard's statistics (run_stats layout, 2d + 3 words): kept so that a
  // sharded caller can combine them over the ranks (cdr_points_restat)
  std::vector<unsigned long long> st_local;
  double absmax = 0.0;
  // screen transform  xhat = (x - mu_f) * 2^sigma
  std::vector<float> mu;
  int32_t sigma = 0;
  DevBuf mu_s;  // float[d]: -mu_f * 2^sigma
  // pre-centred copy for screen32: float [d4/4][n_pad][4] of (x - mu) 2^sigma,
  // exact (pre_ok, decided with the mode); built on the first screen32 step
  DevBuf xt32;
  DevBuf muf;  // int64[d]: mu_f 2^S (screen32 restores x sums from xt sums)
  bool pre_ok = false, xt_valid = false;
  // split screen copy for the DELTA steps (screen32d): fp16 hi / lo of
  // xhat = fma(x, 2^sigma, -mu 2^sigma), tiled [n_pad/32][2 halves][32][16 QH B]
  // (the MFMA B operands as loaded); built once per point set
  DevBuf xs16;
  DevBuf xa32;  // the points row-major (float [n_pad][d4]) for fixup32's gathers
  // large-k screen copy (screen_big_sp): fp16 of the pre-centred points as the
  // MFMA B fragments are loaded, [n_pad/64][2 tiles][DQ chunks][64 lanes] x 16 B
  DevBuf xb16;
  bool xb_valid = false;
  bool xa_valid = false;  // xa32 built (ensure_rowmajor)
  // large-k running sums (screen_big DELTA steps): int64 (k, d+1) of the
  // current labels, valid while only large-k steps of k = big_k wrote them
  DevBuf big_sums;
  DevBuf big_chunks;  // L2 chunk numbering of L1's regions (big_chunk_prefix)
  bool big_valid = false;
  int big_k = 0;
  bool xs_valid = false;
  int xs_qh = 0;
  DevBuf mv_list;   // screen32d: per-wave regions of moved points {pt, old | new << 16}
  DevBuf mv_count;  // int32 per wave

  // ---- Lloyd ----
  DevBuf labels;    // int32[n_pad]
  DevBuf cent32r;   // float[k*d]: the float32 reference runs' centroids
  DevBuf cent64;    // double[k*d]
  DevBuf frag;      // fp16 MFMA A-operand fragments
  DevBuf partials;  // int64 per workgroup k*(d+1)
  DevBuf out_sums;  // int64 k*(d+1) (when caller passes a host pointer)
  DevBuf fb_list;   // int32: one region of fb_cap entries per screen wave
  DevBuf fb_count;  // int32[fb_regions + 1]: per-region counts, then the total
  int fb_regions = 0;
  DevBuf f64_sums;  // double k*d
  DevBuf f64_counts;  // int64 k
  // the device-resident F64 run (cdr_lloyd_f64_run): state {running, steps,
  // reason, shift^2 bits}, the last step's means (k*d) and counts (k)
  DevBuf f64r_state, f64r_keep;
  // f64sum.hip: block sums, counts, predicted binades, transfers, walk counts
  DevBuf f64x_A, f64x_cnt, f64x_E, f64x_T, f64x_walk, f64x_G, f64x_GS, f64x_prof;
  // f64_step_fused: the binade predictions of the last F64 step (two buffers:
  // the one the current transfers use, the next step's), valid for (k, blocks)
  DevBuf f64x_E2;
  DevBuf f64x_GC;  // f64_step_fused: per (cluster, group of 64 blocks) member counts
  DevBuf f64x_ord;  // f64_step_fused: each block's rows in cluster order (uint8 offsets)
  DevBuf f64x_cs;   // f64_cent_prep: the screen's fp32 centroid rows + norms, then its ok flag
  // f64_step_fused's transfer cache (cdr_lloyd_f64_run): per block {labels
  // changed this step, step stamp of its last binade change}, the list of the
  // blocks whose transfers are recomputed, and two list counters
  DevBuf f64x_dirty;
  int f64x_stamp = 0;
  DevBuf f64s_off;  // sharded F64 sums: earlier shards' approximate totals, end binades
  int32_t f64s_k = 0, f64s_nranks = 0, f64s_rank = 0;  // cdr_f64s_begin's step
  bool f64x_e_ok = false;
  int f64x_e_cur = 0, f64x_e_k = 0;
  int64_t f64x_e_nb = 0;
  int64_t f64x_walked = -1;  // blocks re-added element-wise in the last F64 step (-1: serial)
  HostBuf h_small;  // pinned scratch for small D2H
  HostBuf h_up;     // pinned staging of the per-step screen32 upload
  hipEvent_t up_event = nullptr;  // recorded after that upload
  bool up_pending = false;
  int64_t last_fallback = 0;
  // profiling (cdr_profile_*): per profiled step three HIP events on the
  // context stream (step start, after the screen kernel, step end), taken
  // from a pool and only resolved by cdr_profile_read, so that profiling
  // never makes the host wait inside an enqueued loop
  bool prof_on = false;
  int prof_period = 1;     // profile every prof_period-th step (event records
  int64_t prof_seen = 0;   // cost the GPU a few us each)
  std::vector<hipEvent_t> prof_pool;
  size_t prof_used = 0;  // events of this profiling session (4 per step)
  int64_t prof_cur = -1; // first event of the current step's triple, -1 none
  double prof_screen_ms = 0.0, prof_step_ms = 0.0, prof_fb_points = 0.0;
  int64_t prof_launches = 0;
  std::vector<char> prof_sub;  // per recorded step: event 3 (prof_mark_sub) recorded
  double prof_sub_ms = 0.0;    // start -> event 3, summed over those steps
  int64_t prof_sub_launches = 0;
  DevBuf fb_accum;  // int64: fallback points summed over the steps (publish32)
  DevBuf q_acc;     // int64 per screen32p wave: points queued for the k-way screen (profiling)
  char prof_kernel[96] = {0};  // name of the last screen kernel launched
  int fb_layout = -1;     // screen32: nwaves the fb_count buffer was zeroed for
  int fb_total_slot = 0;  // fb_count index holding the last step's fallback total
  int32_t last_k = 0;
  bool have_labels = false;
  bool last_screened = false;
  // screen32 incremental update: exact int64 running sums/counts (k, d+1) that
  // belong to the labels in `labels` (valid after a screen32 step with run_k)
  DevBuf run_sums;
  bool run_valid = false;
  // screen32d's one-byte copy of `labels` (k <= 64): the DELTA screen reads a
  // point's previous label from it (1 B instead of 4 B per point and step);
  // valid while only screen32d / fixup32 wrote the labels since it was built
  DevBuf lab8;
  bool lab8_valid = false;
  // DELTA steps on the pruned screen (screen32p, triangle-inequality
  // certificates) instead of the k-way MFMA screen; switched off when too
  // many points of a step stay uncertified (clusters not separated)
  bool prune_on = true;
  // bounded DELTA steps (screen32b, device loop only): per-point bound words
  // (valid while every step since the last reset was a screen32b step whose
  // centroid move ll_finalize32 accounted in bnd), the row-major hi copy the
  // step gathers from, and the cumulative drifts bnd = int64 W[64] (2^-40
  // units) | float W up [64] | float W down [64]
  DevBuf zb, xh16, bnd, t_acc;
  DevBuf rs_hist;  // radix.hip: per-tile digit counts and digit bases of the fallback sort
  DevBuf s32_dyn;  // screen32bs16's dynamic-tail counters (2 parities x 4 regions x 8 XCDs)
  int s32_dyn_par = 0;  // the parity the next launch claims from
  DevBuf zl, zn;  // split bounded screen: per-wave lists of failed points (screen32bz), lengths
  bool zb_valid = false, xh_valid = false, bnd_ok = false;
  int zb_fmt = 0;  // bound words in zb: 16 (2-byte, screen32bs) or 32 bits
  int64_t ll_fin_count = 0;  // finalizes since lloyd_begin (2-byte rebase schedule)
  int32_t run_k = 0;
  bool last_delta = false;
#ifdef CDR_EXPERIMENTS
  int screen_ablate = 0;  // timing experiments only (never in the product build)
#endif

  // ---- device-resident Lloyd loop (loop.hip) ----
  // ll_C current centroids (k x d fp64), ll_new last means (k x d) + counts
  // (k int64), ll_sums the step's (k, d+1) sums when the caller passes no
  // buffer, ll_ref the inertia reference row + mu (2d fp64), ll_state int64[8]:
  // [0] active, [1] steps done, [2] stop reason, [3] shift^2 bits,
  // [4] inertia bits.
  DevBuf ll_C, ll_new, ll_sums, ll_ref, ll_state;
  bool ll_on = false, ll_devplan = false, ll_hostplan_once = false;
  bool ll_devbig = false;  // large-k shapes: screen_big steps on a device-built plan
  int32_t ll_k = 0, ll_flags = 0;
  double ll_tol = 0.0, ll_x2 = 0.0, ll_xxmax = 0.0, ll_l1x = 0.0;
  int64_t ll_enqueued = 0;
  const long long* ll_fin_sums = nullptr;  // what the next finalize reads
  int ll_fin_slices = 1;
  bool ll_fin_devstep = false;  // the last assign was a device-plan screen32 step

  // ---- native collective (comm.hip): RCCL communicator of the loop ----
  void* comm = nullptr;  // ncclComm_t
  int comm_ranks = 1, comm_rank = 0;
  DevBuf comm_buf;  // the step's (k, d+1) int64 sums, all-reduced in place

  // ---- seeding ----
  DevBuf dmin;        // double[n_pad]
  DevBuf dmin32, bs32;  // float32 reference runs: fp32 dist_sq [n_pad], chunk sums
  // exact pruning of the seeding update (seed.hip seed_prunable): the index
  // of each point's nearest centre so far, the centres, their distances to
  // the newest one
  DevBuf seed_near;   // int32[n_pad]
  DevBuf seed_cents;  // double[count][d]
  DevBuf seed_ccd;    // double[count]
  int seed_count = 0;
  DevBuf blocksums;   // double[nblocks]
  DevBuf xfer;        // per-block transfer records
  DevBuf cend;        // double[nblocks] running value after each block
  DevBuf seg_tails, seg_ents, seg_scan, seg_items, seg_meta;  // cumsum program (seed.hip)
  double seed_prog_total = 0.0;
  bool seed_prog_ready = false;
  long long seed_programs = 0;   // scans run through a cumsum program
  long long seed_fallbacks = 0;  // programs whose guess failed (block walk instead)
  DevBuf seed_x16, seed_e16, seed_mu;  // fp16-certified seeding copy (seed.hip)
  bool seed16_valid = false;
  DevBuf seed_run_buf;  // seed_run: uniforms, picks, S, flags
  // device-resident seeding over sharded rows (seed.hip cdr_seed_shard_*):
  // [u: k-1][picks: k][S, guess, c_mine, c_after, c_last, flags x4, pad]
  DevBuf ss_buf;
  int64_t ss_row_begin = 0, ss_n_total = 0, ss_nbmax = 0;
  int32_t ss_nranks = 0, ss_rank = 0, ss_k = 0, ss_step = 0;
  bool ss_on = false;
  DevBuf seed_tail_plan;  // pairwise layout of the partial last block (seed.hip)
  int64_t seed_tail_m = -1;
  int seed_tail_nleaves = 0, seed_tail_nheights = 0;
  DevBuf seed_scalar; // small device scratch
  double seed_c_in = 0.0;
  bool seed_scanned = false;
  double seed_total = 0.0;
  int64_t nblocks() const { return (n + kSeedBlock - 1) / kSeedBlock; }

  // ---- medians / features scratch ----
  DevBuf med_vals, med_off, med_out, med_tmp, med_tmp2, med_hist;
  int32_t med_k = 0;  // clusters of the grouped rows (cdr_medians_group)
  // timestamp range of the resident events (min, max, any null), computed by
  // the producer that wrote them (events_ts_range, groupby.hip); valid for
  // ev_tsr_n events until another writer of ev_ts clears ev_tsr_valid
  DevBuf ev_tsr;
  bool ev_tsr_valid = false;
  int64_t ev_tsr_n = -1;
  DevBuf ev_file, ev_op, ev_client, ev_ts, ev_primary, ev_out, ev_scratch,
      ev_scratch2;
  DevBuf ev_part;  // int64 per ts_minmax workgroup: min, max
  DevBuf fin_counts, fin_creation, fin_out, fin_red;
  int64_t ev_n = 0, ev_nf = 0;  // resident events of cdr_features_generate
  int32_t ev_cmax = 0;          // largest client id among them (payload width)
  // hand-written group-by (groupby.hip) scratch and what its last run did
  DevBuf gb_tilepref, gb_chunk, gb_rsum, gb_part, gb_small, gb_res, gb_bbase, gb_p1, gb_p2, gb_hist2,
      gb_list, gb_slots;
  DevBuf gb_bbase3, gb_t3;  // a third partition pass (large file counts): bucket bases, tile starts
  DevBuf sim_cnt, sim_off, sim_tmp, sim_ms, sim_mbase;  // simulate.hip scratch
  DevBuf x_small, x_buf, x_prim;                        // exchange.hip scratch
  int gb_last_hand = 0, gb_last_L = 0, gb_last_passes = 0, gb_last_pbytes = 0, gb_last_big = 0,
      gb_last_dense = 0;
  int64_t gb_last_grid = 0;

  // ---- access-log ingest (ingest.hip) ----
  DevBuf ing_log;              // log bytes, zero-padded to a whole tile
  DevBuf ing_blk;              // int64 per tile: record counts, then offsets
  DevBuf ing_tmp;              // int64 per scan part: the tile-count scan's partials (tile_scan_*)
  DevBuf ing_mask;             // uint16 per 16 log bytes: record-terminator mask
  DevBuf ing_ends;             // int64 per record: byte index of its terminator
  DevBuf ing_scalar;           // int64 scratch: totals, error rows, flags
  DevBuf ing_pbytes, ing_poff; // manifest paths: bytes, int64 offsets (n+1)
  DevBuf ing_pkey, ing_pidx;   // path hash table: u64 key, int32 first row
  DevBuf ing_nbytes, ing_noff; // node names
  DevBuf ing_nkey, ing_nidx;   // node hash table
  int64_t ing_nbytes_log = 0, ing_nfiles = -1;
  int32_t ing_nnodes = 0;
  uint64_t ing_pmask = 0, ing_nmask = 0;
};

// ---- launchers implemented in the .hip files ----
void points_analyze_and_store(Ctx& c, const double* host_X);
void points_generate(Ctx& c, int64_t n_total, int64_t row_begin, int32_t n_blobs,
                     uint64_t seed);
void points_finish_analysis(Ctx& c);

void lloyd_step_f32x(Ctx& c, const double* C, int32_t k, int64_t* out,
                     bool out_on_device);
void lloyd_step_f64(Ctx& c, const double* C, int32_t k, double* sums,
                    int64_t* counts);

void seed_reset(Ctx& c);
void seed_update(Ctx& c, const double* cent);
void f32r_seed_update(Ctx& c, const float* cen, int reset, float* total);
void lloyd_step_f32r(Ctx& c, const float* C, int32_t k, double* sums, int64_t* counts);
bool f32_sums_parallel(Ctx& c, int k, double* d_sums);
void seed_scan(Ctx& c, double total, double c_in, double* c_out);
void events_ts_range(Ctx& c, int64_t ne);
void seed_scan_begin(Ctx& c, double total, double c_guess, int64_t* n_items, int64_t* n_fine);
void seed_scan_items(Ctx& c, cdr_seed_item* out, int64_t cap, int64_t* n_items);
void seed_scan_end(Ctx& c, double c_in, double* c_out);
void seed_run(Ctx& c, int64_t first, int k, const double* u, int64_t* picks);
void seed_search(Ctx& c, double c_last, double u, int64_t* idx);

void medians_segmented(Ctx& c, const double* values, const int64_t* offsets,
                       int64_t n_segments, double* out);
void medians_by_label(Ctx& c, int32_t k, double* out);

void features_aggregate(Ctx& c, int64_t n_events, const int32_t* file_idx,
                        const uint8_t* op, const int32_t* client,
                        const int64_t* ts_ms, int64_t n_files,
                        const int32_t* primary, int64_t* out,
                        int64_t* max_ts_ms);
// hand-written group-by of the resident events; false = shape not supported
// (nothing computed, the caller takes the sort-based path)
bool groupby_resident(Ctx& c, int64_t ne, int64_t nf, int64_t* out, int64_t* max_ts);
// exact sequential-order F64 centroid sums in parallel (f64sum.hip); false =
// shape not covered (d < 2 or k > 64)
bool f64_sums_parallel(Ctx& c, int k, double* d_sums, bool pre = false);
// stable LSD radix sort of (key, value) pairs over key bits [0, end_bit)
// (radix.hip); true when the sorted pairs are in (k1, v1)
template <typename K, typename V>
bool radix_sort_pairs(Ctx& c, K* k0, K* k1, V* v0, V* v1, int64_t n, int end_bit);
// sharded F64 sums (f64sum.hip; include/cdr.h cdr_f64s_*)
int f64s_cap();
bool f64s_assign_totals(Ctx& c, int k, const double* dC, double* tot_slot);
void f64s_build(Ctx& c, int k, int nranks, int rank, const double* tot_all, void* prog_all);
void f64s_compose_all(Ctx& c, int k, int nranks, const double* tot_all, const void* prog_all,
                      double* d_sums, long long* d_counts, int* d_status);
void f64s_chain_walk(Ctx& c, int k, double* chain);
// tcache: 0 every transfer formed; 1 every transfer formed and the cache
// started; 2 only the blocks whose labels or binade predictions changed since
// the previous tcache step (the others keep their transfers)
bool f64_step_fused(Ctx& c, int k, const double* dC, double* d_sums,
                    unsigned long long* d_counts, bool prof, const long long* gate = nullptr,
                    int tcache = 0);
void features_finalize(Ctx& c, int64_t n_files, const int64_t* counts,
                       const double* creation_s, double observation_end,
                       double* out);

// comm.hip: SUM all-reduce of n int64 in place on the context stream over the
// context's communicator; release of that communicator
void comm_allreduce_i64(Ctx& c, long long* buf, size_t n);
// SUM all-reduce of n doubles in place; in-place all-gather of `bytes` per rank
// (this rank's part at buf + rank * bytes), both on the context stream
void comm_allreduce_f64(Ctx& c, double* buf, size_t n);
void comm_allgather(Ctx& c, void* buf, size_t bytes);
void comm_release(Ctx& c);

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Profiling (lloyd.hip): prof_step_begin starts a profiled step when
// profiling is on (false otherwise); prof_mark(c, i) records event i of it
// (0 start, 1 after the screen kernel, 2 end); prof_mark_sub(c) records the
// end of the first of the screen's two kernels (split bounded screen).
bool prof_step_begin(Ctx& c);
void prof_mark(Ctx& c, int i);
void prof_mark_sub(Ctx& c);

// The step's fallback total from the screens' per-wave counts fbc[0, nwaves)
// (the DELTA screens write per-wave counts only: thousands of same-address
// atomics at the end of a kernel serialise in L2).  One workgroup, every
// thread calls it; the total is returned on every thread.
__device__ inline int block_sum_counts(const int* __restrict__ fbc, int nwaves) {
  __shared__ int s_total;
  if (threadIdx.x == 0) s_total = 0;
  __syncthreads();
  int v = 0;
  for (int i = threadIdx.x; i < nwaves; i += blockDim.x) v += fbc[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(&s_total, v);
  __syncthreads();
  return s_total;
}

// fp64 -> fp16 with one round-to-nearest-even, identical on host and device
// (the screen fragments are built by both: build_plan32 and plan32_build).
// Branch-free: round to odd into fp32 (truncate, then set the lowest bit when
// inexact), then one RNE fp32 -> fp16 conversion; fp32 keeps 13 bits more than
// fp16, so the two roundings give the correctly rounded fp16 (the classic
// round-to-odd argument).  |v| >= 65520 gives +-inf, NaN stays NaN.
__host__ __device__ inline _Float16 f64_to_f16(double v) {
  const float f = (float)v;  // RNE
  const double back = (double)f;
  unsigned b;
  memcpy(&b, &f, 4);
  b -= (fabs(back) > fabs(v)) ? 1u : 0u;  // one ulp toward zero: truncation
  b |= (back != v) ? 1u : 0u;              // sticky bit: round to odd
  float fo;
  memcpy(&fo, &b, 4);
  return (_Float16)fo;
}

}  // namespace cdr

struct cdr_ctx {
  cdr::Ctx c;
};
