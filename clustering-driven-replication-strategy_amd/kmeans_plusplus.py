"""k-means++ seeding and Lloyd iterations on MI355X (drop-in module).

Replaces the reference's ``src/kmeans_plusplus.py`` for its caller
``src/main.py:12,91``: same module name, same functions, same arguments, same
results.  The host side below only keeps the reference's *control* logic —
the NumPy RNG streams, the iteration loop, the empty-cluster reseed and the
convergence test — and every O(n) operation runs in libcdr.so (HIP, gfx950):

=================================  ==========================================
reference (src/kmeans_plusplus.py)  here
=================================  ==========================================
:9-10   rng.integers first index    host (same Generator, same draw)
:14-17  min_j ||x - c_j||^2         cdr_seed_update: running min, exact fp64
:18     dist_sq.sum()               cdr_seed_update block sums + host seq sum
:19     rng.choice(n, p=probs)      host rng.random() + cdr_seed_scan/search
                                    (bit-exact sequential cumsum emulation)
:33-34  norm + argmin               cdr_lloyd_step: certified MFMA screen +
                                    exact fp64 fallback (identical labels);
                                    float32 X: cdr_lloyd_step_f32r (fp32 norms)
:37-41  X[mask].mean(axis=0)        fused int64 fixed-point sums (F32X) or
                                    row-ordered fp64 sums (F64) / host divide;
                                    float32 X: row-ordered fp32 sums
:43     np.random.randint reseed    host (global legacy RNG, j order)
:45-48  norm(new - old) < tol       host NumPy (same BLAS call)
=================================  ==========================================

One extension, keyword-only: ``max_iter``.  The reference computes
``max(100, number_of_files / 100)``, a float for number_of_files > 10000, so
``range(max_iter)`` raises ``TypeError`` (:29-31).  That behaviour is kept by
default; pass ``max_iter=`` to run large inputs.
"""
from __future__ import annotations

import os
import warnings

import numpy as np

from _cdr import MODE_F32X, MODE_F64, Context, NanProbabilities, default_context, host_seq_sum

__all__ = ["kmeans_plusplus_init", "kmeans"]


def _nan_probabilities() -> None:
    # probs = dist_sq / 0.0 in the reference warns, then Generator.choice raises.
    warnings.warn("invalid value encountered in divide", RuntimeWarning, stacklevel=3)
    raise ValueError("Probabilities contain NaN")


def _seed_on_device(ctx: Context, X: np.ndarray, k: int, random_state) -> np.ndarray:
    """k-means++ D^2 seeding against points already resident in `ctx`."""
    rng = np.random.default_rng(random_state)
    n_samples, n_features = X.shape
    centroids = np.empty((k, n_features), dtype=X.dtype)
    first_idx = rng.integers(0, n_samples)
    centroids[0] = X[first_idx]
    if k > 1 and hasattr(ctx, "seed_run"):
        # every step on the device (cdr_seed_run); rng.choice draws one
        # uniform per step (:19), so the k - 1 draws are taken up front
        u = rng.random(k - 1)
        try:
            picks = ctx.seed_run(first_idx, k, u)
        except NanProbabilities:  # (argument errors stay ValueErrors of their own)
            _nan_probabilities()
        centroids[:] = X[picks]
        return centroids
    if k > 1:
        ctx.seed_reset()
    for i in range(1, k):
        # only the newest centre changes the running minimum
        ctx.seed_update(np.asarray(centroids[i - 1], dtype=np.float64))
        total = host_seq_sum(ctx.seed_block_sums())
        if not (total > 0.0) or total == np.inf:
            _nan_probabilities()
        c_last = ctx.seed_scan(total, 0.0)
        u = rng.random()
        next_idx = ctx.seed_search(c_last, u)
        if next_idx < 0:  # cannot happen: cdf[-1] == 1.0 > u
            raise RuntimeError("k-means++ sampler found no index")
        centroids[i] = X[next_idx]
    return centroids


def _seed_f32r(ctx: Context, X: np.ndarray, k: int, random_state) -> np.ndarray:
    """The reference's seeding on a float32 X (:6, 14-19 in float32): the
    device forms fp32 dist_sq, its fp32 total and fp32 probabilities, then
    the exact float64 cumsum scan and search of Generator.choice as in the
    float64 case with S = 1.  Every step runs on the device
    (cdr_f32r_seed_run): Generator.choice draws exactly one rng.random() per
    step (:19), so the k - 1 draws are taken up front and one readback
    returns the picks.  CDR_F32R_STEPS=1: the per-step host loop instead."""
    rng = np.random.default_rng(random_state)
    n_samples, n_features = X.shape
    centroids = np.empty((k, n_features), dtype=X.dtype)
    first_idx = rng.integers(0, n_samples)
    centroids[0] = X[first_idx]
    if k > 1 and hasattr(ctx, "f32r_seed_run") and not os.environ.get("CDR_F32R_STEPS"):
        u = rng.random(k - 1)
        try:
            picks = ctx.f32r_seed_run(int(first_idx), k, u)
        except NanProbabilities:
            _nan_probabilities()
        centroids[:] = X[picks]
        return centroids
    for i in range(1, k):
        try:
            ctx.f32r_seed_update(centroids[i - 1], reset=(i == 1))
        except NanProbabilities:
            _nan_probabilities()
        c_last = ctx.seed_scan(1.0, 0.0)
        u = rng.random()
        next_idx = ctx.seed_search(c_last, u)
        if next_idx < 0:  # cannot happen: cdf[-1] == 1.0 > u
            raise RuntimeError("k-means++ sampler found no index")
        centroids[i] = X[next_idx]
    return centroids


def _seed(ctx: Context, X: np.ndarray, k: int, random_state) -> np.ndarray:
    if X.dtype == np.float32:
        return _seed_f32r(ctx, X, k, random_state)
    return _seed_on_device(ctx, X, k, random_state)


def kmeans_plusplus_init(X, k, random_state=None, *, context: Context | None = None):
    """D^2 seeding (reference src/kmeans_plusplus.py:3-22)."""
    X = np.asarray(X)
    ctx = context if context is not None else default_context()
    ctx.load_points(X)
    return _seed(ctx, X, k, random_state)


def _cluster_means(ctx: Context, C: np.ndarray, mode: int, scale_bits: int):
    """One assignment + update pass; returns (means (k, d) float64, counts (k,))."""
    k, d = C.shape
    if mode == MODE_F32X:
        acc = ctx.lloyd_step(C)
        counts = acc[:, d]
        # exact: the int64 sum of values on the 2^-S grid, as a float64
        sums = np.ldexp(acc[:, :d].astype(np.float64), -scale_bits)
    else:
        sums, counts = ctx.lloyd_step_f64(C)
    with np.errstate(invalid="ignore", divide="ignore"):
        means = sums / counts[:, None].astype(np.float64)
    return means, counts


def _f64_device_loop(ctx: Context, X: np.ndarray, centroids: np.ndarray, max_iter: int,
                     tol: float) -> np.ndarray:
    """max_iter Lloyd steps (fewer on convergence) of F64 points on the
    device; a step the device hands back (an empty cluster, or a shift too
    close to tol) is finished here exactly as the reference does (:37-48)."""
    n_samples = X.shape[0]
    done = 0
    while done < max_iter:
        C, steps, reason, means, counts = ctx.lloyd_f64_run(centroids, max_iter - done, tol)
        centroids, done = C, done + steps
        if reason == ctx.F64_RUN_CONVERGED:
            break
        if reason != ctx.F64_RUN_HOST:
            break  # every step applied
        new_centroids = np.empty_like(centroids)
        new_centroids[...] = means
        for j in np.flatnonzero(counts == 0):  # j order, as the reference draws (:43)
            new_centroids[j] = X[np.random.randint(0, n_samples)]
        shift = np.linalg.norm(new_centroids - centroids)
        centroids, done = new_centroids, done + 1
        if shift < tol:
            break
    return centroids


def kmeans(X, k, number_of_files=100, tol=1e-4, random_state=None, *,
           max_iter=None, context: Context | None = None):
    """Lloyd's k-means after k-means++ seeding (reference :24-50).

    Returns ``(centroids, labels)``: centroids after the last update, labels
    (int64) from the last assignment — exactly as the reference does.
    """
    X = np.asarray(X)
    n_samples = X.shape[0]
    ctx = context if context is not None else default_context()
    ctx.load_points(X)
    centroids = _seed(ctx, X, k, random_state)

    if max_iter is None:
        max_iter = max(100, number_of_files / 100)
    iters = range(max_iter)  # the reference's TypeError for a float max_iter (:29-31)
    info = ctx.info()
    mode, scale_bits = info["mode"], info["scale_bits"]

    if X.dtype == np.float32:
        # the reference's float32 arithmetic (:6, 33-34, 41): fp32 norms and
        # argmin, sequential fp32 cluster sums; np.mean divides in fp64 (the
        # intp count promotes) and casts the quotient to float32
        ran = False
        for _ in iters:
            ran = True
            sums, counts = ctx.lloyd_step_f32r(centroids)
            with np.errstate(invalid="ignore", divide="ignore"):
                means = sums / counts[:, None].astype(np.float64)
            new_centroids = np.empty_like(centroids)
            new_centroids[...] = means
            for j in np.flatnonzero(counts == 0):  # j order, as the reference draws (:43)
                new_centroids[j] = X[np.random.randint(0, n_samples)]
            shift = np.linalg.norm(new_centroids - centroids)
            centroids = new_centroids
            if shift < tol:
                break
        if not ran:
            raise UnboundLocalError("local variable 'labels' referenced before assignment")
        return centroids, ctx.labels()

    if mode == MODE_F32X and centroids.dtype in (np.float64, np.float32) and len(iters) > 0:
        # device-resident loop: means, shift and convergence on the device,
        # the host only for empty clusters and near-tol shifts (csrc/loop.hip)
        from cdr_dist import device_lloyd

        centroids, st = device_lloyd(ctx, centroids, len(iters), tol,
                                     lambda g: X[g], n_samples, dtype=centroids.dtype)
        ctx.last_inertia = st["inertia"]
        return centroids, ctx.labels()

    if (mode == MODE_F64 and centroids.dtype == np.float64 and len(iters) > 0
            and 2 <= centroids.shape[1] <= 16 and k <= 64):
        # F64: the steps resident on the device (exact assignment, exact
        # sequential sums, means and shift), the host only for empty clusters
        # and near-tol shifts (cdr_lloyd_f64_run)
        return _f64_device_loop(ctx, X, centroids, len(iters), tol), ctx.labels()

    ran = False
    for _ in iters:
        ran = True
        calc = np.asarray(centroids, dtype=np.float64)
        means, counts = _cluster_means(ctx, calc, mode, scale_bits)
        new_centroids = np.empty_like(centroids)
        new_centroids[...] = means
        for j in np.flatnonzero(counts == 0):  # j order, as the reference draws (:43)
            new_centroids[j] = X[np.random.randint(0, n_samples)]
        shift = np.linalg.norm(new_centroids - centroids)
        centroids = new_centroids
        if shift < tol:
            break
    if not ran:
        raise UnboundLocalError("local variable 'labels' referenced before assignment")
    labels = ctx.labels()
    return centroids, labels
