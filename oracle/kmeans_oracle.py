"""NumPy restatement of the reference k-means (TEST INFRASTRUCTURE ONLY).

Follows /root/reference/src/kmeans_plusplus.py line by line but never builds
the (n, k, d) temporaries: distances are computed one centroid at a time in
exactly NumPy's summation order, which makes every result bit-identical to
the reference while using O(n*d) memory:

* ``np.linalg.norm(A, axis=2)`` for float64 is ``sqrt(add.reduce(A*A, axis))``
  (numpy/linalg/_linalg.py, ord=None branch); ``add.reduce`` over a contiguous
  run of d <= 128 values is pairwise_sum's small-n path: sequential from 0.0
  for d < 8, else 8 accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
  plus the d % 8 tail.  ``sqdist_rows`` restates that (kmeans_plusplus.py:15,33).
* ``np.min(..., axis=1)`` over the centroids seen so far equals a running
  ``np.minimum`` (min is exact and order free) (:14-17).
* ``np.argmin(..., axis=1)`` = first index of the minimum, reproduced with a
  strict ``<`` running argmin over centroids (:34).
* Everything else (sum, choice, mean, norm, RNG) calls NumPy itself, as the
  reference does.

``tests/test_oracle.py`` checks this module against NumPy's own reductions
and against golden vectors written by running the reference (gen_golden.py).
"""
from __future__ import annotations

import numpy as np

PW_BLOCK = 128  # numpy pairwise_sum leaf size (PW_BLOCKSIZE)
REDUCE_CHUNK = 8192  # numpy ufunc reduction buffer size


def _pw_leaf_cols(cols):
    """pairwise_sum leaf over a list of equally-shaped arrays (m <= 128)."""
    m = len(cols)
    if m < 8:
        res = np.zeros_like(cols[0]) if m else None
        for c in cols:
            res = res + c
        return res
    r = [cols[j].copy() for j in range(8)]
    mm = m - m % 8
    for i in range(8, mm, 8):
        for j in range(8):
            r[j] = r[j] + cols[i + j]
    res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
    for i in range(mm, m):
        res = res + cols[i]
    return res


def _pairwise_cols(cols):
    m = len(cols)
    if m <= PW_BLOCK:
        return _pw_leaf_cols(cols)
    n2 = m // 2
    n2 -= n2 % 8
    return _pairwise_cols(cols[:n2]) + _pairwise_cols(cols[n2:])


def sqdist_rows(X: np.ndarray, c: np.ndarray) -> np.ndarray:
    """Pre-sqrt squared distances of every row of X to c in NumPy's order."""
    diff = X - c
    s = diff * diff
    cols = [s[:, f] for f in range(s.shape[1])]
    if not cols:
        return np.zeros(X.shape[0])
    return _pairwise_cols(cols)


def pairwise_sum_1d(a: np.ndarray) -> float:
    """np.add.reduce of a contiguous 1-D float64 array: 8192-element chunks,
    pairwise inside each chunk, chunks accumulated from 0.0 left to right."""
    total = 0.0
    for s in range(0, a.size, REDUCE_CHUNK):
        chunk = a[s:s + REDUCE_CHUNK]
        total = total + float(_pairwise_cols([np.float64(v) for v in chunk]))
    return total


def assign(X: np.ndarray, C: np.ndarray, chunk: int = 1 << 20) -> np.ndarray:
    """labels = np.argmin(np.linalg.norm(X[:,None]-C[None], axis=2), axis=1)."""
    n = X.shape[0]
    labels = np.empty(n, dtype=np.int64)
    for s in range(0, n, chunk):
        Xs = X[s:s + chunk]
        best = np.full(Xs.shape[0], np.inf)
        lab = np.zeros(Xs.shape[0], dtype=np.int64)
        for j in range(C.shape[0]):
            r = np.sqrt(sqdist_rows(Xs, C[j]))
            better = r < best
            best = np.where(better, r, best)
            lab[better] = j
        labels[s:s + chunk] = lab
    return labels


def update(X: np.ndarray, labels: np.ndarray, centroids: np.ndarray, n_samples: int):
    """kmeans_plusplus.py:37-43 verbatim (global np.random reseed)."""
    k = centroids.shape[0]
    new_centroids = np.empty_like(centroids)
    for j in range(k):
        mask = labels == j
        if np.any(mask):
            new_centroids[j] = X[mask].mean(axis=0)
        else:
            new_centroids[j] = X[np.random.randint(0, n_samples)]
    return new_centroids


def kmeans_plusplus_init(X, k, random_state=None):
    """kmeans_plusplus.py:3-22 with an incremental running minimum."""
    X = np.asarray(X)
    rng = np.random.default_rng(random_state)
    n_samples, n_features = X.shape
    centroids = np.empty((k, n_features), dtype=X.dtype)
    first_idx = rng.integers(0, n_samples)
    centroids[0] = X[first_idx]
    dist_sq = np.full(n_samples, np.inf, dtype=X.dtype)  # float32 X: fp32 sum and probs (:14-18)
    for i in range(1, k):
        t = np.sqrt(sqdist_rows(X, centroids[i - 1])) ** 2
        dist_sq = np.minimum(dist_sq, t)
        probs = dist_sq / dist_sq.sum()
        next_idx = rng.choice(n_samples, p=probs)
        centroids[i] = X[next_idx]
    return centroids


def kmeans(X, k, number_of_files=100, tol=1e-4, random_state=None, max_iter=None):
    """kmeans_plusplus.py:24-50 (``max_iter`` override for n > 10000)."""
    X = np.asarray(X)
    n_samples = X.shape[0]
    centroids = kmeans_plusplus_init(X, k, random_state=random_state)
    if max_iter is None:
        max_iter = max(100, number_of_files / 100)
    labels = None
    for _ in range(max_iter):
        labels = assign(X, centroids)
        new_centroids = update(X, labels, centroids, n_samples)
        shift = np.linalg.norm(new_centroids - centroids)
        centroids = new_centroids
        if shift < tol:
            break
    return centroids, labels


def lloyd(X: np.ndarray, C: np.ndarray, max_iter: int, tol: float = 1e-4):
    """kmeans_plusplus.py:31-48 from given centroids: (centroids, labels of
    the last assignment, the centroids that assignment used, steps taken)."""
    labels, used, steps = None, C, 0
    for _ in range(max_iter):
        steps += 1
        labels = assign(X, C)
        used = C
        new = update(X, labels, C, X.shape[0])
        shift = np.linalg.norm(new - C)
        C = new
        if shift < tol:
            break
    return C, labels, used, steps


def inertia(X: np.ndarray, C: np.ndarray, labels: np.ndarray, chunk: int = 1 << 20) -> float:
    """sum_i ||x_i - C[labels_i]||^2 in fp64 (north_star's per-step inertia;
    the reference computes none)."""
    tot = 0.0
    for s in range(0, X.shape[0], chunk):
        diff = X[s:s + chunk] - C[labels[s:s + chunk]]
        tot += float(np.sum(diff * diff))
    return tot


def lloyd_partials(X: np.ndarray, C: np.ndarray, scale_bits: int):
    """(labels, int64 fixed-point sums (k, d+1)) for grid data — what one
    device step returns; exact when every x * 2^scale_bits is an integer."""
    labels = assign(X, C)
    k, d = C.shape
    out = np.zeros((k, d + 1), dtype=np.int64)
    q = np.ldexp(X, scale_bits).astype(np.int64)
    np.add.at(out[:, :d], labels, q)
    out[:, d] = np.bincount(labels, minlength=k)
    return labels, out
