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


def _label_medians(X, lab, k):
    out = np.full((k, X.shape[1]), np.nan)
    for j in range(k):
        m = lab == j
        if m.any():
            out[j] = np.median(X[m], axis=0)
    return out


@pytest.mark.parametrize("mode", ["f32x", "f64"])
def test_medians_by_label_shapes(ctx, mode):
    """k = 40 with empty clusters, d = 70 (two 64-feature chunks), repeated
    values, negatives and signed zeros; F32X and F64 points."""
    rng = np.random.default_rng(5 if mode == "f32x" else 6)
    n, d, k = 40_000, 70, 40
    if mode == "f32x":
        X = np.round(rng.normal(0, 4, (n, d)) * 64) / 64  # a 2^-6 grid
    else:
        X = rng.normal(0, 4, (n, d)) * np.pi
    X[::7, 3] = X[0, 3]          # many ties in one column
    X[::11, 5] = -0.0
    X[1::11, 5] = 0.0
    ctx.load_points(X)
    assert ctx.info()["mode"] == (1 if mode == "f32x" else 2)
    C = X[rng.choice(n, k, replace=False)].copy()
    C[-5:] = 1e6                  # empty clusters
    if mode == "f32x":
        ctx.lloyd_step(C)
    else:
        ctx.lloyd_step_f64(C)
    lab = ctx.labels()
    got = ctx.medians_by_label(k)
    exp = _label_medians(X, lab, k)
    np.testing.assert_array_equal(got, exp)
    assert np.isnan(got[-1]).all()


def _med_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    from _cdr import Context
    from cdr_dist import Comm, sharded_medians

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X = np.load(os.path.join(out_dir, "X.npy"))
    C = np.load(os.path.join(out_dir, "C.npy"))
    lo, hi = (X.shape[0] * rank) // world, (X.shape[0] * (rank + 1)) // world
    ctx = Context(0)
    ctx.load_points(X[lo:hi])
    ctx.lloyd_step(C)
    med = sharded_medians(ctx, Comm(dist, None), C.shape[0])
    np.save(os.path.join(out_dir, f"med{rank}.npy"), med)
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_medians_two_ranks(ctx, tmp_path):
    """Two processes on the one GPU, gloo collectives: every rank's medians
    equal the single-process medians of the whole point set (e4)."""
    from test_features_dist import _free_port

    mp = pytest.importorskip("torch.multiprocessing")
    rng = np.random.default_rng(9)
    X = np.round(rng.normal(0, 3, (60_001, 6)) * 256) / 256
    C = X[rng.choice(X.shape[0], 12, replace=False)].copy()
    np.save(tmp_path / "X.npy", X)
    np.save(tmp_path / "C.npy", C)
    mp.spawn(_med_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    ctx.load_points(X)
    ctx.lloyd_step(C)
    single = ctx.medians_by_label(12)
    np.testing.assert_array_equal(single, _label_medians(X, ctx.labels(), 12))
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"med{r}.npy"), single)
