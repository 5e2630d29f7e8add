"""GPU parity of the per-cluster medians (segmented radix select) and scoring."""
import json
import os
import warnings

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import synth

pytestmark = pytest.mark.gpu


def test_segmented_median_matches_numpy(ctx):
    rng = np.random.default_rng(0)
    segs = [rng.random(int(rng.integers(0, 300))) for _ in range(200)]
    segs += [np.array([-0.0]), np.array([-0.0, -0.0]), np.array([1.0, np.nan, 2.0]),
             np.array([2.0 ** 53 + 1, 2.0 ** 53 + 3]), np.array([1e308, 1e308]),
             np.array([-5.0, 3.0, -1e-300, 7.0]), np.array([]), rng.normal(0, 1e6, 10001),
             np.repeat(rng.random(3), 50), rng.integers(-5, 5, 1000).astype(np.float64)]
    offsets = np.zeros(len(segs) + 1, dtype=np.int64)
    np.cumsum([s.size for s in segs], out=offsets[1:])
    got = ctx.medians_segmented(np.concatenate(segs), offsets)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        exp = np.array([np.median(s) for s in segs])
    np.testing.assert_array_equal(got, exp)  # NaN == NaN for assert_array_equal
    assert str(got[200]) == "0.0" and np.signbit(got[200]) == np.signbit(exp[200])


def test_scoring_matches_reference_golden(ctx):
    from scoring import ClusterClassifier

    with open(os.path.join(GOLDEN, "scoring_cases.json")) as fh:
        cases = json.load(fh)
    for c in cases:
        s = c["spec"]
        clf = ClusterClassifier(s["global_medians"], s["weights"], s["directions"],
                                s["replication_factors"], context=ctx)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            med = clf.compute_cluster_medians(s["clusters"])
            res = clf.classify(s["clusters"])
        for cn, mm in med.items():
            for p, v in mm.items():
                g = c["medians"][cn][p]
                assert (np.isnan(v) and np.isnan(g)) or v == g, (c["name"], cn, p)
        assert res == c["result"], c["name"]


def test_demo_output(ctx, capsys):
    import scoring

    assert scoring.demo(context=ctx) == {"C1": "Hot", "C2": "Archival", "C3": "Archival",
                                         "C4": "Hot"}
    assert "C1 → Hot" in capsys.readouterr().out


def test_medians_by_label_matches_list_path(ctx):
    import kmeans_plusplus as kp
    from scoring import ClusterClassifier

    n, d, k = 50000, 5, 8
    X = synth.generate(n, 0, n, d, k, 21)
    np.random.seed(0)
    C, lab = kp.kmeans(X, k, random_state=42, max_iter=5, context=ctx)
    med = ctx.medians_by_label(k)
    for j in range(k):
        for f in range(d):
            vals = X[lab == j, f]
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", RuntimeWarning)
                assert med[j, f] == np.median(vals) or (np.isnan(med[j, f]) and vals.size == 0)
    names = [f"f{i}" for i in range(d)]
    gm = {nm: 0.5 for nm in names}
    w = {c: {nm: 1.0 for nm in names} for c in ("Hot", "Shared", "Moderate", "Archival")}
    dirs = {"Hot": {nm: 1 for nm in names}, "Shared": {nm: 1 for nm in names},
            "Moderate": {nm: 0 for nm in names}, "Archival": {nm: -1 for nm in names}}
    rf = {"Hot": 3, "Shared": 2, "Moderate": 1, "Archival": 4}
    clf = ClusterClassifier(gm, w, dirs, rf, context=ctx)
    a = clf.classify_labels(k, names)
    lists = {f"C{j}": {nm: X[lab == j, i].tolist() for i, nm in enumerate(names)}
             for j in range(k)}
    assert a == clf.classify(lists)
