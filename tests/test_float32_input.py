"""float32 input.  The reference keeps X's dtype for its
centroids (src/kmeans_plusplus.py:6, :37), so with float32 X it seeds and
averages in float32.  tests/golden/kmeans_f32_cases.npz holds the reference's
own runs (oracle/gen_golden.py float32_cases) on float32 X and on the same
values as float64.

The drop-in computes distances in fp64 and rounds the exact cluster means to
float32: on these fixtures the seeds and every label equal the
reference's float32 run, and the centroids are within 1e-5 relative (the
north_star's fp32 tolerance) — not bit-identical, because the reference
accumulates the float32 means sequentially in float32 (up to 11 ulps here)."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "kmeans_f32_cases.npz")


def _cases():
    z = np.load(GOLD)
    for i in range(3):
        n, d, k, seed, rs, npseed = (int(v) for v in z[f"c{i}_meta"])
        yield i, z, k, rs, npseed


def test_reference_float32_vs_float64_fixtures():
    """What the fixtures pin: the reference's float32 and float64 runs agree
    on seeds and labels, and its float32 centroids are NumPy's float32 means
    of the final labels (sequential float32 sums, kmeans_plusplus.py:41)."""
    for i, z, k, rs, npseed in _cases():
        X = z[f"c{i}_X"]
        assert X.dtype == np.float32
        np.testing.assert_array_equal(z[f"c{i}_f32_init"].astype(np.float64), z[f"c{i}_f64_init"])
        np.testing.assert_array_equal(z[f"c{i}_f32_labels"], z[f"c{i}_f64_labels"])
        C32 = z[f"c{i}_f32_centroids"]
        assert C32.dtype == np.float32
        lab = z[f"c{i}_f32_labels"]
        np.testing.assert_array_equal(np.stack([X[lab == j].mean(0) for j in range(k)]), C32)


def test_float32_semantics_of_the_drop_in_within_tolerance():
    """The drop-in's float32 centroids (exact means rounded to float32) stay
    within 1e-5 relative of the reference's float32 centroids."""
    for i, z, k, rs, npseed in _cases():
        X = z[f"c{i}_X"]
        lab = z[f"c{i}_f32_labels"]
        ours = np.stack([np.float32(X[lab == j].astype(np.float64).mean(0)) for j in range(k)])
        np.testing.assert_allclose(ours, z[f"c{i}_f32_centroids"], rtol=1e-5, atol=0)


@pytest.mark.gpu
def test_gpu_kmeans_float32_input(ctx):
    import kmeans_plusplus as kp

    for i, z, k, rs, npseed in _cases():
        X = z[f"c{i}_X"]
        np.random.seed(npseed)
        init = kp.kmeans_plusplus_init(X, k, random_state=rs, context=ctx)
        assert init.dtype == np.float32
        np.testing.assert_array_equal(init, z[f"c{i}_f32_init"])
        np.random.seed(npseed)
        C, labels = kp.kmeans(X, k, number_of_files=X.shape[0], random_state=rs, context=ctx)
        assert C.dtype == np.float32
        np.testing.assert_array_equal(labels, z[f"c{i}_f32_labels"])
        np.testing.assert_allclose(C, z[f"c{i}_f32_centroids"], rtol=1e-5, atol=0)
