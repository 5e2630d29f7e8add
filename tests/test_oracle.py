"""The oracle is pinned before it is trusted: against NumPy's own reductions
and against golden vectors produced by running the reference (gen_golden.py)."""
import json
import os
import warnings

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import kmeans_oracle as ko
from oracle import scoring_oracle, synth


def _cases():
    with open(os.path.join(GOLDEN, "kmeans_cases.json")) as fh:
        meta = json.load(fh)
    arrays = np.load(os.path.join(GOLDEN, "kmeans_cases.npz"))
    out = []
    for i, m in enumerate(meta["cases"]):
        X = synth.generate(*m["gen"]) if "gen" in m else arrays[f"c{i}_X"]
        get = lambda key: arrays[f"c{i}_{key}"] if f"c{i}_{key}" in arrays else None  # noqa
        out.append((m, X, get("init"), get("centroids"), get("labels")))
    return out, meta


CASES, META = _cases()


@pytest.mark.parametrize("d", [1, 2, 3, 5, 7, 8, 9, 15, 16, 17, 24, 33, 64, 100, 128, 129, 300])
def test_sqdist_order_matches_numpy_norm(d):
    rng = np.random.default_rng(d)
    X = rng.random((64, d)) * rng.choice([1e-3, 1.0, 1e3])
    C = rng.random((5, d))
    ref = np.linalg.norm(X[:, None, :] - C[None, :, :], axis=2)
    for j in range(5):
        np.testing.assert_array_equal(np.sqrt(ko.sqdist_rows(X, C[j])), ref[:, j])


@pytest.mark.parametrize("n", [1, 7, 8, 9, 129, 1000, 8192, 8193, 16384, 20000, 100003])
def test_blocked_pairwise_sum_matches_numpy(n):
    a = np.random.default_rng(n).random(n) ** 3
    assert ko.pairwise_sum_1d(a) == a.sum()


def test_mean_order_d1_is_pairwise_and_d2_sequential():
    rng = np.random.default_rng(3)
    for m in (5, 100, 9000, 20000):
        x = rng.random((m, 1)) ** 3
        assert x.mean(axis=0)[0] == ko.pairwise_sum_1d(x[:, 0]) / m
        y = rng.random((m, 2)) ** 3
        s = np.zeros(2)
        for r in range(m):
            s = s + y[r]
        np.testing.assert_array_equal(y.mean(axis=0), s / m)


@pytest.mark.parametrize("case", CASES, ids=[c[0]["name"] for c in CASES])
def test_oracle_matches_reference_golden(case):
    m, X, init, C, labels = case
    np.random.seed(m["np_seed"])
    if m.get("error"):
        with pytest.raises(ValueError, match=m["error"]):
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", RuntimeWarning)
                ko.kmeans_plusplus_init(X, m["k"], random_state=m["rs"])
        return
    got_init = ko.kmeans_plusplus_init(X, m["k"], random_state=m["rs"])
    np.testing.assert_array_equal(got_init, init)
    if m["seed_only"]:
        return
    np.random.seed(m["np_seed"])
    got_C, got_l = ko.kmeans(X, m["k"], number_of_files=X.shape[0], random_state=m["rs"])
    np.testing.assert_array_equal(got_l, labels)
    np.testing.assert_array_equal(got_C, C)


def test_reference_typeerror_recorded():
    assert META["n_gt_10000_error"] == "'float' object cannot be interpreted as an integer"


def test_synth_is_grid_data_and_deterministic():
    a = synth.generate(1000, 0, 1000, 7, 5, 99)
    b = synth.generate(1000, 500, 500, 7, 5, 99)
    np.testing.assert_array_equal(a[500:], b)
    assert a.min() >= 0.0 and a.max() < 1.0
    np.testing.assert_array_equal(np.ldexp(a, 24), np.round(np.ldexp(a, 24)))


def test_scoring_oracle_matches_reference_golden():
    with open(os.path.join(GOLDEN, "scoring_cases.json")) as fh:
        cases = json.load(fh)
    for c in cases:
        s = c["spec"]
        med = scoring_oracle.cluster_medians(s["clusters"])
        for cn, m in med.items():
            for p, v in m.items():
                g = c["medians"][cn][p]
                assert (np.isnan(v) and np.isnan(g)) or v == g
        res = scoring_oracle.classify(s["clusters"], s["global_medians"], s["weights"],
                                      s["directions"], s["replication_factors"])
        assert res == c["result"], c["name"]
    demo = cases[0]
    assert demo["result"] == {"C1": "Hot", "C2": "Archival", "C3": "Archival", "C4": "Hot"}


def test_int64_mean_equals_numpy_mean_only_below_2_53():
    """Why the F32X gate sits at 2^53 grid units: below it NumPy's sequential
    fp64 sum of grid values is exact (so the exact int64 sum converted once is
    the same number); past it the running sum rounds and the two differ."""
    import numpy as np

    small = np.array([2.0 ** 52, 1.0, 1.0, 1.0])  # partial sums < 2^53: exact
    assert np.add.accumulate(small)[-1] == float(int(2 ** 52) + 3)
    big = np.array([2.0 ** 53, 1.0, 1.0])  # past 2^53: each + 1 rounds away
    seq = 0.0
    for v in big:
        seq = seq + v
    assert seq == 2.0 ** 53 and float(int(2 ** 53) + 2) == 2.0 ** 53 + 2
