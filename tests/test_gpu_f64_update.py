"""F64-mode centroid sums in parallel (csrc/f64sum.hip) against NumPy's
sequential row-order sums (`X[labels == j].mean(axis=0)`,
src/kmeans_plusplus.py:41) and against the serial kernel, plus a whole
k-means at n = 2M on min-max-normalised (non-grid) features against
oracle.kmeans_oracle.kmeans, bit for bit."""
import time

import numpy as np
import pytest

from oracle import kmeans_oracle as ko

pytestmark = pytest.mark.gpu


def _minmax(rng, n, d):
    """Features as compute_features writes them: min-max normalised doubles
    (full 53-bit mantissas, not on any power-of-two grid)."""
    raw = rng.gamma(2.0, 3.0, (n, d)) * rng.random(d) + rng.normal(0, 1, (n, d))
    return (raw - raw.min(axis=0)) / (raw.max(axis=0) - raw.min(axis=0))


def _numpy_sums(X, labels, k):
    out = np.zeros((k, X.shape[1]))
    for j in range(k):
        m = labels == j
        if m.any():
            out[j] = np.add.reduce(X[m], axis=0)  # row-sequential for d >= 2
    return out


def _check_step(ctx, X, C, monkeypatch):
    ctx.load_points(X)
    assert ctx.info()["mode"] == 2
    sums, counts = ctx.lloyd_step_f64(C)
    walked = ctx.f64_walked()
    labels = ctx.labels()
    np.testing.assert_array_equal(labels, ko.assign(X, C))
    np.testing.assert_array_equal(counts, np.bincount(labels, minlength=C.shape[0]))
    np.testing.assert_array_equal(sums, _numpy_sums(X, labels, C.shape[0]))
    monkeypatch.setenv("CDR_F64_SERIAL", "1")
    s2, c2 = ctx.lloyd_step_f64(C)
    monkeypatch.delenv("CDR_F64_SERIAL")
    assert ctx.f64_walked() == -1
    np.testing.assert_array_equal(s2, sums)
    return walked


def test_nonneg_features_few_walks(ctx, monkeypatch):
    rng = np.random.default_rng(1)
    X = _minmax(rng, 300_000, 5)
    C = X[rng.choice(X.shape[0], 8, replace=False)].copy()
    walked = _check_step(ctx, X, C, monkeypatch)
    blocks = -(-X.shape[0] // 256) * 8 * 5
    assert 0 <= walked < 0.05 * blocks, walked


def test_mixed_signs_and_negative_columns(ctx, monkeypatch):
    rng = np.random.default_rng(2)
    X = _minmax(rng, 100_000, 4) - 0.5
    X[:, 3] = -np.abs(X[:, 3]) - 1e-3
    X[::97, 1] = -0.0
    C = X[rng.choice(X.shape[0], 6, replace=False)].copy()
    _check_step(ctx, X, C, monkeypatch)


def test_tiny_clusters_and_signed_zero(ctx, monkeypatch):
    rng = np.random.default_rng(3)
    X = _minmax(rng, 5000, 3)
    X[:10] = [-0.0, 0.0, -0.0]
    X[10] = [50.0, 50.0, 50.0]                        # a one-member cluster
    C = np.vstack([X[:1], X[10:11], X[rng.choice(5000, 4, replace=False)]])
    C[0] = [-0.0, -0.0, -0.0]
    _check_step(ctx, X, C, monkeypatch)


def test_kmeans_2m_minmax_features_bit_exact(ctx):
    """The verdict's size: 2M files x 5 min-max features, k = 8, k-means++
    seeding + Lloyd to convergence (max_iter 60), against the oracle."""
    import kmeans_plusplus as kp

    rng = np.random.default_rng(4)
    X = _minmax(rng, 2_000_000, 5)
    np.random.seed(7)
    t0 = time.perf_counter()
    C, labels = kp.kmeans(X, 8, random_state=42, max_iter=60, context=ctx)
    dt = time.perf_counter() - t0
    np.random.seed(7)
    C_ref, labels_ref = ko.kmeans(X, 8, random_state=42, max_iter=60)
    np.testing.assert_array_equal(C, C_ref)
    np.testing.assert_array_equal(labels, labels_ref)
    # the step time with the parallel sums (reported in the test log)
    ctx.load_points(X)
    ctx.lloyd_step_f64(C)
    ctx.synchronize()
    t1 = time.perf_counter()
    for _ in range(5):
        ctx.lloyd_step_f64(C)
    ctx.synchronize()
    step = (time.perf_counter() - t1) / 5
    print(f"\nF64 2M x 5 k=8: kmeans {dt:.2f} s, one step {step * 1e3:.2f} ms, "
          f"walked blocks {ctx.f64_walked()}")


@pytest.mark.parametrize("n,d,k", [(120_000, 16, 64), (80_000, 20, 10), (60_000, 6, 70),
                                   (50_000, 2, 3), (70_001, 9, 33)])
def test_step_shapes_fused_and_separate(ctx, monkeypatch, n, d, k):
    """The fused assignment + block pass (d <= 16, k <= 64: f64_step_fused),
    the separate passes (d > 16) and the serial sums (k > 64), at ragged n:
    labels = the oracle's, sums = NumPy's sequential sums, = the serial kernel."""
    rng = np.random.default_rng(10 + d + k)
    X = _minmax(rng, n, d)
    C = X[rng.choice(n, k, replace=False)].copy()
    _check_step(ctx, X, C, monkeypatch)
    # a second step from moved centroids (the predictions of the first are not reused)
    C2 = C * 0.75 + 0.125
    _check_step(ctx, X, C2, monkeypatch)
