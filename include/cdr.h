/*
 * cdr.h — C ABI of the MI355X (gfx950) clustering hot path.
 *
 * "cdr" = clustering-driven replication.  One shared library, libcdr.so, built
 * from hand-written HIP kernels.  Every entry point takes plain pointers and
 * sizes and returns an int status (CDR_OK == 0).  On failure the message is
 * available from cdr_last_error() (thread-local).
 *
 * The reference (Harounnn/Clustering-Driven-Replication-Strategy) has no FFI:
 * its hot path is NumPy / PySpark code.  Each block below names the reference
 * function it replaces (file:line relative to the reference root).  The Python
 * drop-in modules (kmeans_plusplus.py, scoring.py, compute_features.py) bind
 * these symbols through ctypes; INTEGRATION.md shows the binding.
 *
 * Ownership: host pointers belong to the caller and are only read/written for
 * the duration of the call.  Device buffers belong to the context.  A context
 * is bound to one HIP device and is NOT thread-safe (the reference is
 * single-threaded and uses global NumPy RNG state, src/kmeans_plusplus.py:43).
 * All calls are synchronous from the caller's point of view unless the name
 * ends in _async.
 */
#ifndef CDR_H_
#define CDR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define CDR_OK 0
#define CDR_ERR_ARG 1         /* bad argument  -> Python ValueError            */
#define CDR_ERR_HIP 2         /* HIP runtime    -> Python RuntimeError          */
#define CDR_ERR_NAN 3         /* NaN probabilities (kmeans_plusplus.py:18-19)   */
#define CDR_ERR_STATE 4       /* call order     -> Python RuntimeError          */
#define CDR_ERR_UNSUPPORTED 5 /* shape not supported -> NotImplementedError     */

/* ---- point storage modes (cdr_points_info) ----------------------------- */
/* F32X: every coordinate is an fp32 value on a 2^-S grid with |x|*2^S < 2^31.
 *       Screen + exact fallback assignment; centroid sums are exact int64
 *       fixed point (bit-identical to NumPy's sequential fp64 mean whenever
 *       that mean is itself exact, e.g. 2^-24-grid data).                     */
#define CDR_MODE_F32X 1
/* F64:  arbitrary fp64 data.  Exact fp64 assignment for every point and
 *       sequential per-cluster fp64 sums in row order (NumPy mean order).     */
#define CDR_MODE_F64 2

typedef struct cdr_ctx cdr_ctx;

const char* cdr_last_error(void);
int cdr_version(void);
int cdr_device_count(int* out);

/* Context on HIP device `device`.  Owns a HIP stream unless one is supplied
 * with cdr_set_stream (e.g. torch.cuda.current_stream().cuda_stream).       */
int cdr_create(int device, cdr_ctx** out);
int cdr_destroy(cdr_ctx* ctx);
int cdr_set_stream(cdr_ctx* ctx, void* hip_stream);
int cdr_synchronize(cdr_ctx* ctx);

/* ---- point set (the X of src/main.py:81, one shard per context) -------- */
/* Host row-major float64 (n, d).  Detects the storage mode (see above).     */
int cdr_points_load_f64(cdr_ctx* ctx, const double* X, int64_t n, int32_t d);
/* Synthetic generator (BASELINE configs 2/3/5): rows [row_begin, row_begin +
 * n_local) of an n_total-row data set, generated on the device.  Integer-only
 * counter-based formula; oracle/synth.py is the NumPy mirror.               */
int cdr_points_generate(cdr_ctx* ctx, int64_t n_total, int64_t row_begin,
                        int64_t n_local, int32_t d, int32_t n_blobs,
                        uint64_t seed);
int cdr_points_info(cdr_ctx* ctx, int64_t* n, int32_t* d, int32_t* mode,
                    int32_t* scale_bits);
/* Points sharded over ranks: every rank must use the same
 * storage mode, fixed-point scale S and screen transform, or the int64 sums
 * of the all-reduce and the device loop's stop decisions would differ per
 * rank.  cdr_points_stats: this shard's statistics st[2d + 3] (uint64 order
 * keys of the per-feature minima, then maxima; max(-lsb) + 200000; not-fp32
 * flag; non-finite flag).  cdr_points_restat: re-decide mode / S / transform
 * from statistics combined over every shard (MIN of the minimum keys, MAX of
 * every other word) and the global row count n_sum.                         */
int cdr_points_stats(cdr_ctx* ctx, uint64_t* st);
int cdr_points_restat(cdr_ctx* ctx, const uint64_t* st, int64_t n_sum);
/* Copy local rows idx[0..m) to host as float64 (m, d). */
int cdr_points_get_rows(cdr_ctx* ctx, const int64_t* idx, int64_t m,
                        double* out);

/* ---- k-means++ D^2 seeding: src/kmeans_plusplus.py:3-22 ---------------- */
/* dist_sq := +inf (before the first centre).                                */
int cdr_seed_reset(cdr_ctx* ctx);
/* dist_sq[i] = min(dist_sq[i], (sqrt(pw_d((x_i - c)^2)))^2), NumPy order
 * (kmeans_plusplus.py:14-17), then the 8192-element pairwise block sums of
 * dist_sq (NumPy's blocked add.reduce, used by dist_sq.sum() at :18).  c is
 * one float64 row of length d.                                              */
int cdr_seed_update(cdr_ctx* ctx, const double* c);
/* The reference's float32 seeding step (src/kmeans_plusplus.py:14-18 on a
 * float32 X): dist_sq = min(dist_sq, fp32(norm(X - c))**2) with c float32
 * (reset != 0: dist_sq starts at +inf), *total = dist_sq.sum() in fp32
 * (NumPy's 8192-chunk pairwise order), and the probabilities fp32(dist_sq /
 * total) staged as doubles for cdr_seed_scan(ctx, 1.0, ...) and
 * cdr_seed_search, which then give rng.choice's pick.  CDR_ERR_NAN when the
 * total is not positive and finite.                                        */
int cdr_f32r_seed_update(cdr_ctx* ctx, const float* c, int32_t reset, float* total);
/* Number of 8192-element blocks of this shard and their pairwise sums.     */
int cdr_seed_num_blocks(cdr_ctx* ctx, int64_t* nblocks);
int cdr_seed_block_sums(cdr_ctx* ctx, double* out);
/* Exact sequential cumulative sum of probs = dist_sq / total over this
 * shard, starting from running value c_in (0.0 on the first shard); returns
 * the running value after the shard's last element.  Emulates np.cumsum
 * bit-exactly (Generator.choice, kmeans_plusplus.py:19).                   */
int cdr_seed_scan(cdr_ctx* ctx, double total, double c_in, double* c_out);
/* The same scan in two halves, for sharded seeding without a rank-ordered
 * chain (cdr_dist.seed_sharded replaces kmeans_plusplus.py:19's single
 * np.cumsum over all rows).  _begin builds this shard's cumsum program from
 * a GUESS of the running value at its first element (the sum of the earlier
 * shards' block sums / total); the program is the shard's exact function
 * c_in -> c_out as long as it has no CDR_SEED_FINE item.  _items copies it
 * out; cdr_seed_program_eval runs it on the host (no device, no context).
 * _end takes the exact c_in, fills what cdr_seed_search needs and returns
 * c_out — exact whatever the guess was (it falls back to the block walk).  */
typedef struct {
  int64_t d0, d1; /* RUN: grid steps added for an even / odd entry         */
  double p;       /* CROSS: the element added; CONST: the value            */
  int32_t e;      /* RUN: binade exponent                                   */
  int32_t kind;   /* CDR_SEED_*                                             */
} cdr_seed_item;
enum {
  CDR_SEED_RUN = 0,   /* c in binade e: N += (N odd ? d1 : d0), N < 2^53    */
  CDR_SEED_CROSS = 1, /* c = fl(c + p)                                      */
  CDR_SEED_CONST = 2, /* c = p (a shard whose c_in is known: the first)     */
  CDR_SEED_FINE = 3,  /* element walk of block d0 (device only)             */
  CDR_SEED_MARK = 4,  /* device bookkeeping; no-op                          */
  CDR_SEED_END = 5,
  CDR_SEED_SKIP = 6,  /* empty run                                          */
  CDR_SEED_BAD = 7    /* the guess cannot hold: evaluation fails            */
};
int cdr_seed_scan_begin(cdr_ctx* ctx, double total, double c_guess, int64_t* n_items,
                        int64_t* n_fine);
int cdr_seed_scan_items(cdr_ctx* ctx, cdr_seed_item* out, int64_t cap, int64_t* n_items);
int cdr_seed_scan_end(cdr_ctx* ctx, double c_in, double* c_out);
/* out[0] = scans run through a program, out[1] = of those, the ones whose
 * guess failed and fell back to the exact block walk (same result; counted
 * by the per-step calls — cdr_seed_run gates its fallback on the device).  */
int cdr_seed_stats(cdr_ctx* ctx, int64_t* out);
/* The whole kmeans_plusplus_init (:3-22) on this context's points with no host
 * round trip per step: first = the first row (rng.integers), u[0..k-1) = the
 * uniforms of the k - 1 draws (rng.choice takes one rng.random() each);
 * picks[0..k) = the chosen rows.  CDR_ERR_NAN when a total is not finite and
 * positive ("Probabilities contain NaN").                                   */
int cdr_seed_run(cdr_ctx* ctx, int64_t first, int32_t k, const double* u, int64_t* picks);
/* The reference's float32 seeding (src/kmeans_plusplus.py:3-22 on a float32
 * X, the semantics of cdr_f32r_seed_update) as one device-resident run, like
 * cdr_seed_run: fp32 dist_sq, totals and probabilities, rng.choice's pick per
 * step on the device.  CDR_ERR_NAN as cdr_f32r_seed_update, with the message
 * "probabilities do not sum to 1" (Generator.choice's) when a total overflows
 * to +inf while every dist_sq is finite.                                    */
int cdr_f32r_seed_run(cdr_ctx* ctx, int64_t first, int32_t k, const double* u, int64_t* picks);
/* The same over rows sharded across nranks ranks (whole 8192-row blocks per
 * shard, this context holding rows [row_begin, row_begin + n) of n_total),
 * device-resident: per step three phases, each followed by one collective the
 * caller runs on device buffers —
 *   begin            -> red (d + 4 doubles): SUM all-reduce
 *   phase 0 (red)    -> this rank's slot of the block sums [nranks][nbmax]:
 *                       all-gather
 *   phase 1 (sums)   -> this rank's slot of the programs [nranks][1024 items]:
 *                       all-gather
 *   phase 2 (progs)  -> red: SUM all-reduce
 * (k - 1 steps), then end (red) -> picks[0..k) (global rows), centres (k x d
 * fp64, the picked rows: every rank has them), status 0 ok,
 * 1 "run the host protocol instead" (a program could not be composed, or
 * disagreed with its own scan: seen by every rank through the all-reduce),
 * 2 a total not finite and positive (Probabilities contain NaN).  sizes[3]:
 * bytes per rank of the three buffers.  cdr_seed_run_sharded runs every step
 * with the context's communicator (cdr_comm_init).  Reference:
 * src/kmeans_plusplus.py:3-22.                                               */
int cdr_seed_shard_begin(cdr_ctx* ctx, int64_t row_begin, int64_t n_total, int32_t nranks,
                         int32_t rank, int64_t first, int32_t k, const double* u, double* red,
                         int64_t* sizes);
int cdr_seed_shard_phase(cdr_ctx* ctx, int32_t phase, const void* in, void* out);
int cdr_seed_shard_end(cdr_ctx* ctx, const double* red, int64_t* picks, double* centres,
                       int32_t* status);
int cdr_seed_run_sharded(cdr_ctx* ctx, int64_t row_begin, int64_t n_total, int64_t first, int32_t k,
                         const double* u, int64_t* picks, double* centres, int32_t* status);
/* *ok = 0 when some item does not hold for this c_in (or a FINE item).      */
int cdr_seed_program_eval(const cdr_seed_item* items, int64_t n_items, double c_in,
                          double* c_out, int32_t* ok);
/* searchsorted(cumsum / c_last, u, side='right') restricted to this shard:
 * *idx = local index, or -1 when the crossing is not in this shard.        */
int cdr_seed_search(cdr_ctx* ctx, double c_last, double u, int64_t* idx);

/* ---- Lloyd iteration: src/kmeans_plusplus.py:31-43 --------------------- */
/* One assignment + fused update pass for centroids C (k, d) float64.
 * Labels stay on the device (cdr_lloyd_labels).
 * F32X mode: out (k, d+1) int64 = per-cluster fixed-point sums (value *
 *   2^scale_bits) and counts in column d.  `out_on_device` != 0 means `out`
 *   is a device pointer on this context's device; the kernels then write it
 *   on the context stream without synchronising (for an RCCL all-reduce).
 * F64 mode: use cdr_lloyd_step_f64.                                          */
int cdr_lloyd_step(cdr_ctx* ctx, const double* C, int32_t k, int64_t* out,
                   int32_t out_on_device);
/* F64 mode: exact fp64 assignment; sums (k, d) float64 accumulated in row
 * order exactly like X[labels == j].mean(axis=0)'s sum; counts (k).        */
int cdr_lloyd_step_f64(cdr_ctx* ctx, const double* C, int32_t k, double* sums,
                       int64_t* counts);
/* F64 mode, 2 <= d <= 16, k <= 64: up to max_steps Lloyd steps resident on
 * the device (src/kmeans_plusplus.py:31-48; replaces a host loop of
 * cdr_lloyd_step_f64 + means + shift): each step's exact assignment and
 * sequential sums, then means = sums / counts and shift = ||means - C|| on
 * the device.  info[0] = steps applied (C replaced by the means); info[1] =
 * 0 all max_steps applied, 1 converged (the last applied step had shift <
 * tol), 2 the next step needs the host (an empty cluster, or a shift too
 * close to tol to decide): that step is NOT applied, C_out is the centroids
 * it started from, means_out (k, d) / counts_out (k) are its means and
 * counts, and the labels on the device are its assignment.  C_out (k, d):
 * the centroids after the applied steps.  tol <= 0: never converges.      */
int cdr_lloyd_f64_run(cdr_ctx* ctx, const double* C, int32_t k, int32_t max_steps, double tol,
                      double* C_out, double* means_out, int64_t* counts_out, int32_t* info);
/* The reference's float32 runs (X float32 keeps its dtype,
 * src/kmeans_plusplus.py:6, 33-34, 41): float32 norms in NumPy order, argmin
 * of the fp32 norms, sums (k, d) = the SEQUENTIAL float32 sums of each
 * cluster's rows (returned as doubles holding fp32 values; the caller
 * divides in fp64 and casts to fp32, as np.mean does); counts (k).
 * C: k x d float32.  Points loaded from a float32 array (either mode).  */
int cdr_lloyd_step_f32r(cdr_ctx* ctx, const float* C, int32_t k, double* sums,
                        int64_t* counts);
/* F64 mode, d >= 2, k <= 64: the sums are formed in parallel (csrc/f64sum.hip:
 * per-block parity transfers inside one binade, exact); *walked = blocks of
 * (cluster, feature) sequences re-added element by element in the last step,
 * or -1 when the step used the serial kernel.                               */
int cdr_lloyd_f64_walked(cdr_ctx* ctx, int64_t* walked);
/* Sharded F64 sums (src/kmeans_plusplus.py:33-41 on rows sharded in rank
 * order, float64 data off any grid: src/main.py:81).  Per Lloyd step, with
 * one collective between the calls (buffers are device memory: all ranks'
 * slots, rank r's at offset r x its slot size):
 *   cdr_f64s_begin   assignment (labels) + this shard's approximate
 *                    per-(cluster, feature) totals and member counts into
 *                    its slot of tot_buf; sizes = {tot slot bytes, program
 *                    slot bytes}                       -> all-gather tot_buf
 *   cdr_f64s_build   this shard's program (rank 0: its exact walked sums;
 *                    rank > 0: transfer runs and element lists built from
 *                    the gathered approximate totals) -> all-gather prog_buf
 *   cdr_f64s_finish  every rank composes all programs in rank order: the
 *                    exact sequential sums (k x d) and counts (k); *status
 *                    1 when a program's guess did not hold, the same on
 *                    every rank: then run the rank chain, cdr_f64s_chain on
 *                    rank r (walks its shard from the exact entry
 *                    chain_buf[0, 2 k d) = {sums, any}, leaving its exit
 *                    there) followed by a broadcast of chain_buf from rank r,
 *                    for r = 0 .. nranks - 1 (chain_buf zeroed first).
 * Replaces the sequential NumPy mean (kmeans_plusplus.py:41) over the whole
 * array; 2 <= d <= 16, k <= 64.                                            */
int cdr_f64s_begin(cdr_ctx* ctx, const double* C, int32_t k, int32_t nranks, int32_t rank,
                   void* tot_buf, int64_t* sizes);
int cdr_f64s_build(cdr_ctx* ctx, const void* tot_buf, void* prog_buf);
int cdr_f64s_finish(cdr_ctx* ctx, const void* tot_buf, const void* prog_buf, double* sums,
                    int64_t* counts, int32_t* status);
int cdr_f64s_chain(cdr_ctx* ctx, void* chain_buf);
/* Labels of the last assignment as int64 (np.argmin dtype, :34).           */
int cdr_lloyd_labels(cdr_ctx* ctx, int64_t* labels);
/* Diagnostics of the last step: points the fast screen could not certify
 * and that went through the exact fp64 path.                                */
int cdr_lloyd_stats(cdr_ctx* ctx, int64_t* n_fallback);
/* Profiling: enable != 0 starts collecting HIP-event timings of every
 * enable-th following F32X step (1: every step; the event records cost the GPU
 * a few microseconds each) on the context stream; cdr_profile_read returns
 * out[6] = {screen kernel ms (sum), steps, whole step kernels ms (sum),
 * fallback points (sum), points the pruned screen queued for its k-way MFMA
 * screen (sum), points whose drift bound failed in the bounded screen and were
 * re-decided from their coordinates (sum)}.                                  */
int cdr_profile_reset(cdr_ctx* ctx, int32_t enable);
int cdr_profile_read(cdr_ctx* ctx, double* out);
/* The same session's steps whose screen ran as two kernels (the split bounded
 * screen: screen32bz, then screen32bs): out[2] = {ms from the step start to
 * the end of the first kernel (sum), such steps}.                            */
int cdr_profile_read_sub(cdr_ctx* ctx, double* out);

/* ---- device-resident Lloyd loop: src/kmeans_plusplus.py:31-48 ----------- */
/* The same iterations as cdr_lloyd_step + the host's means / reseed / shift,
 * but the means, the shift and the convergence test run on the device
 * (bit-identical: the same fp64 operations), so steps can be enqueued without
 * a host round trip.  The device STOPS the loop (later enqueued steps do
 * nothing) and reports why whenever the reference's host logic is needed:
 * an empty cluster (np.random.randint reseed, :43), a shift within 1e-9
 * relative of tol (np.linalg.norm decides, :45-47), or centroids outside the
 * fp16 screen range.  F32X points only (CDR_ERR_UNSUPPORTED otherwise).
 *
 * cdr_points_sqdev: sum_i ||x_i - ref||^2 (fp64) of this shard; with ref a
 *   data row this is exact per term; it anchors the inertia.
 * cdr_lloyd_begin: centroids C (k, d); tol (<= 0: never converged); flags bit
 *   0: round the means to float32 (X is float32); ref (d) and x2_total =
 *   cdr_points_sqdev summed over every shard (NaN: this shard alone).
 * cdr_lloyd_enqueue_assign: assignment + fused update of the current
 *   centroids; the (k, d+1) int64 sums go to dsums (device pointer, e.g. the
 *   buffer an RCCL all-reduce sums next) or to an internal buffer (NULL).
 * cdr_lloyd_enqueue_finalize: means / shift / inertia from the (all-reduced)
 *   sums at dsums (NULL: the internal buffer) and the move to the means.
 * cdr_lloyd_status (synchronises): status[4] = {running, steps done, stop
 *   reason (0 running, 1 converged, 2 empty cluster, 3 needs the host plan,
 *   4 shift too close to tol), steps enqueued}; values[2] = {shift, inertia}
 *   of the last finalised step.
 * cdr_lloyd_read: current centroids C (k, d), the last means (k, d, NaN rows
 *   for empty clusters) and counts (k); any pointer may be NULL.
 * cdr_lloyd_resume: after the host took a step itself: C (NULL keeps the
 *   device's), add_steps to the step count, host_plan_once != 0 runs the next
 *   assignment on the host-plan path.                                      */
int cdr_points_sqdev(cdr_ctx* ctx, const double* ref, double* out);
int cdr_lloyd_begin(cdr_ctx* ctx, const double* C, int32_t k, double tol, int32_t flags,
                    const double* ref, double x2_total);
int cdr_lloyd_enqueue_assign(cdr_ctx* ctx, int64_t* dsums);
int cdr_lloyd_enqueue_finalize(cdr_ctx* ctx, const int64_t* dsums);
int cdr_lloyd_status(cdr_ctx* ctx, int64_t* status, double* values);
int cdr_lloyd_read(cdr_ctx* ctx, double* C, double* means, int64_t* counts);
int cdr_lloyd_resume(cdr_ctx* ctx, const double* C, int32_t add_steps, int32_t host_plan_once);
int cdr_lloyd_end(cdr_ctx* ctx);
/* m loop steps enqueued by one call: assign, the SUM all-reduce of the
 * (k, d+1) int64 sums over the context's communicator (cdr_comm_init; none:
 * a single shard), finalize — no host synchronisation and no host code
 * between a step's kernels and its collective.                              */
int cdr_lloyd_enqueue_steps(cdr_ctx* ctx, int32_t m);

/* ---- native collective for the loop: RCCL over xGMI ------------------- */
/* One communicator per context (one process per GPU).  cdr_comm_unique_id
 * writes the 128-byte ncclUniqueId (one rank creates it, the caller
 * broadcasts it); cdr_comm_init joins the nranks-rank communicator as `rank`
 * on the context's device; cdr_comm_destroy leaves it.  librccl is bound at
 * run time; CDR_ERR_UNSUPPORTED when it cannot be loaded.                   */
int cdr_comm_unique_id(void* id128);
int cdr_comm_init(cdr_ctx* ctx, const void* id128, int32_t nranks, int32_t rank);
int cdr_comm_destroy(cdr_ctx* ctx);
/* *ok = 1 when librccl loads and has the entry points (dlopen / dlsym only:
 * unlike cdr_comm_unique_id it starts no bootstrap listener, so every rank may
 * probe with it).                                                            */
int cdr_comm_available(int32_t* ok);
/* The context's communicator: *nranks (0 when it has none) and *rank.       */
int cdr_comm_ranks(cdr_ctx* ctx, int32_t* nranks, int32_t* rank);
/* Name of the last screen kernel launched (for the bench's roofline line);
 * NUL-terminated, truncated to len.                                          */
int cdr_profile_kernel(cdr_ctx* ctx, char* buf, int32_t len);
/* Test hook (not product path): screen values T (n_pad, ceil(k/16)*16) fp32
 * of one F32X step and the certification constants (A0, A1).               */
int cdr_debug_screen(cdr_ctx* ctx, const double* C, int32_t k, float* out_vals,
                     float* thr_a0a1);

/* ---- per-cluster medians: src/scoring.py:40-55 (np.median) ------------- */
/* Segmented median of float64 values: segment s = values[off[s]..off[s+1]).
 * Empty segment -> NaN; any NaN in a segment -> NaN.                        */
int cdr_medians_segmented(cdr_ctx* ctx, const double* values,
                          const int64_t* offsets, int64_t n_segments,
                          double* out);
/* Array-native form: median of every feature of the local
 * points grouped by the labels of the last Lloyd step; out (k, d).          */
int cdr_medians_by_label(cdr_ctx* ctx, int32_t k, double* out);
/* The same in steps, for points sharded over ranks:
 * cdr_medians_group groups this shard's rows by label (counts[k] = local
 * cluster sizes); after a SUM all-reduce of the counts, cdr_medians_begin
 * takes the global sizes and returns the number of radix passes (4 for F32X
 * points, 8 for F64) and the histogram size in uint32 words (k * d * 512);
 * per pass, cdr_medians_pass_hist writes this shard's digit histograms to
 * `hist` (host or device memory), the caller SUM-all-reduces them, and
 * cdr_medians_pass_select consumes the global histograms; cdr_medians_finish
 * writes out (k, d).  Every rank gets the medians of the whole data set.    */
int cdr_medians_group(cdr_ctx* ctx, int32_t k, int64_t* counts);
int cdr_medians_begin(cdr_ctx* ctx, const int64_t* global_counts, int32_t* passes,
                      int64_t* hist_words);
int cdr_medians_pass_hist(cdr_ctx* ctx, int32_t pass, void* hist);
int cdr_medians_pass_select(cdr_ctx* ctx, int32_t pass, const void* hist);
int cdr_medians_finish(cdr_ctx* ctx, double* out);

/* ---- access-log group-by: src/compute_features.py:31-54 ---------------- */
/* Events: file index (row of the manifest, -1 = path not in the manifest),
 * op (1 = WRITE, 2 = READ, other = neither), client id (-1 = null),
 * timestamp in microseconds since the epoch (Spark TimestampType units;
 * INT64_MIN = null: the event counts, the nulls of a file form one more
 * second group, and the max ignores them).
 * primary[f] = client id of file f's primary node (-2 = null).
 * out (n_files, 6) int64: access_freq, writes, reads, local_accesses,
 * total_accesses, max_concurrency (sec = floor(ts_us / 1e6) in fp64, as
 * F.floor(cast(ts as double))).  *max_ts_us = max non-null event timestamp
 * over all events (INT64_MIN when there is none).                          */
int cdr_features_aggregate(cdr_ctx* ctx, int64_t n_events,
                           const int32_t* file_idx, const uint8_t* op,
                           const int32_t* client, const int64_t* ts_us,
                           int64_t n_files, const int32_t* primary,
                           int64_t* out, int64_t* max_ts_us);
/* Config-4 scale runs: a synthetic time-ordered access log generated on
 * the device and kept resident (event e at t0_us + e * span_us / n_events;
 * file uniform over n_files; op WRITE with p = 1/10 else READ; client and
 * primary uniform over 3 datanodes).  cdr_features_aggregate_resident runs
 * the same group-by as cdr_features_aggregate on them (out: host
 * (n_files, 6) or NULL to keep the result on the device);
 * cdr_features_events_read copies the events back (parity tests).          */
int cdr_features_generate(cdr_ctx* ctx, int64_t n_events, int64_t n_files, uint64_t seed,
                          int64_t t0_us, int64_t span_us);
int cdr_features_aggregate_resident(cdr_ctx* ctx, int64_t* out, int64_t* max_ts_us);
/* The reference's access simulator on the device (src/access_simulator.py:
 * 16-60 with src/generator.py:44-45's category weights and primary nodes):
 * files file_begin .. file_begin + n_files - 1 of a manifest, each with a
 * category, jittered read / write rates and locality bias, Poisson arrivals
 * over duration_s seconds from t0_us, timestamps with millisecond precision,
 * clients 0 .. n_clients - 1; the log is left resident sorted by timestamp
 * (file ids local, 0 .. n_files - 1).  *n_events = the events generated.  */
int cdr_features_simulate(cdr_ctx* ctx, int64_t n_files, int64_t file_begin, double duration_s,
                          int32_t n_clients, uint64_t seed, int64_t t0_us, int64_t* n_events);
int cdr_features_events_read(cdr_ctx* ctx, int32_t* file_idx, uint8_t* op, int32_t* client,
                             int64_t* ts_us, int32_t* primary);
/* What the last group-by did: info[0] 1 = hand-written partition + bucket
 * hash path (csrc/groupby.hip), 0 = sort-based path; [1] file-local bits L
 * (2^L files per bucket); [2] partition passes; [3] payload bytes; [4]
 * buckets redone with the global-memory hash; [5] 1 = dense (file, second)
 * grid per bucket, 0 = hash; [6] workgroups of the persistent bucket grid.
 * (info has 7 entries.)                                                    */
int cdr_features_groupby_info(cdr_ctx* ctx, int64_t* info);
/* ---- sharded feature aggregation ------------------ */
/* Rank r owns manifest rows [bounds[r], bounds[r+1]) (nranks + 1 entries,
 * non-decreasing).  cdr_features_exchange_pack: the resident events, grouped
 * by owner rank, as 16-byte records {ts int64, file int32 (global row),
 * client << 8 | op int32} written to `send` (host or device memory, room for
 * every resident event); counts[r] = records for rank r; events outside the
 * manifest are not sent; *max_ts_us = max non-null timestamp over ALL
 * resident events (INT64_MIN if none) for the MAX all-reduce of :48.
 * cdr_features_exchange_unpack: the n records received (host or device
 * memory), all of files [file_begin, file_end), become the resident events
 * with local file ids (and the primaries of those rows move to the front).
 * cdr_features_load_events: host events made resident (the host-tokenised
 * log of a shard).                                                         */
int cdr_features_exchange_pack(cdr_ctx* ctx, int32_t nranks, const int64_t* bounds, void* send,
                               int64_t* counts, int64_t* max_ts_us);
int cdr_features_exchange_unpack(cdr_ctx* ctx, const void* recv, int64_t n, int64_t file_begin,
                                 int64_t file_end);
int cdr_features_load_events(cdr_ctx* ctx, int64_t n, const int32_t* file_idx, const uint8_t* op,
                             const int32_t* client, const int64_t* ts_us, int64_t n_files,
                             const int32_t* primary);
/* Finalisation over sharded rows (:53-94): cdr_features_finalize_stats
 * reduces this rank's n_rows rows to istats[7] = {sum writes, min / max
 * access_freq, min / max writes, min / max concurrency} and dstats[4] = {min /
 * max age, min / max locality} (identities for n_rows == 0); after the SUM /
 * MIN / MAX all-reduce, cdr_features_finalize_apply writes the rows' table
 * with mean(writes) = sum / n_rows_total.  cdr_features_finalize ==
 * stats + apply on one rank.                                               */
int cdr_features_finalize_stats(cdr_ctx* ctx, int64_t n_rows, const int64_t* counts,
                                const double* creation_s, double observation_end,
                                int64_t* istats, double* dstats);
int cdr_features_finalize_apply(cdr_ctx* ctx, int64_t n_rows, const int64_t* counts,
                                const double* creation_s, double observation_end,
                                const int64_t* istats, const double* dstats,
                                int64_t n_rows_total, double* out);
/* Access-log CSV ingest on the device.  Replaces the
 * host read of the log (src/compute_features.py:19-29: spark.read.csv of
 * `ts,path,op,client_node,pid`, to_timestamp; the build's host restatement is
 * compute_features.load_access_log + encode) and the path join against the
 * manifest (:37-41).
 * cdr_ingest_manifest: the manifest's n_files paths (UTF-8 bytes + n_files+1
 *   int64 offsets; an empty string never matches), primary[f] (node id, -2 =
 *   null) and the n_nodes node names whose ids primary uses (bytes + offsets).
 *   Builds device hash tables; CDR_ERR_UNSUPPORTED on a 64-bit hash collision
 *   between distinct strings.
 * cdr_ingest_log: uploads the log bytes and parses them into the resident
 *   events of cdr_features_aggregate_resident (file row or -1, op 1 WRITE /
 *   2 READ / 0, client id or -1 null or -3 not a primary node, ts in
 *   microseconds or INT64_MIN when the timestamp does not parse).
 *   status[6]: records, first bad-timestamp record (-1 none), first record
 *   the device tokeniser does not take (quotes, NUL, lone CR, non-ASCII
 *   timestamp; -1 none), bad-timestamp count, byte span [start, end) from
 *   the end of the previous record to the end of the reported one (blank
 *   lines before it included).  Bad rows are reported in status, not as an error.
 * cdr_ingest_reparse: parses the resident bytes again (benchmarks).        */
int cdr_ingest_manifest(cdr_ctx* ctx, int64_t n_files, const char* path_bytes,
                        const int64_t* path_off, const int32_t* primary, int32_t n_nodes,
                        const char* node_bytes, const int64_t* node_off);
int cdr_ingest_log(cdr_ctx* ctx, const char* bytes, int64_t nbytes, int64_t* status);
int cdr_ingest_reparse(cdr_ctx* ctx, int64_t* status);
/* Finalisation, src/compute_features.py:48-94.  counts: output of
 * cdr_features_aggregate; creation_s: creation_ts_epoch (double seconds, NaN
 * = null -> age 0 as na.fill does); observation_end: max ts in seconds
 * (double).  out (n_files, 10) float64:
 * access_freq, age_seconds, write_ratio, locality, concurrency, then the
 * five *_norm columns.                                                     */
int cdr_features_finalize(cdr_ctx* ctx, int64_t n_files, const int64_t* counts,
                          const double* creation_s, double observation_end,
                          double* out);

/* ---- host helpers (plain C on the host, no device) --------------------- */
/* ((init + v[0]) + v[1]) + ... in fp64, left to right.                      */
double cdr_host_seq_sum(const double* v, int64_t n, double init);

#ifdef __cplusplus
}
#endif
#endif /* CDR_H_ */
